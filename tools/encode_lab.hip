// encode_lab.hip -- A/B lab for the production w = 8 encode kernel's launch
// shape on the bench's C3 layout (96 stripes x RS(10,4) x 4 MiB shards at the
// library's skewed stride): workgroup size (256 / 512 / 1024 threads, i.e. 4 /
// 8 / 16 KiB contiguous per shard per workgroup) and resident workgroups per
// CU (an unused dynamic LDS allocation).  Every variant is checked bit-exact
// against the production launch, then timed in interleaved rounds with HIP
// events.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include -I erasure_coding_test_amd/csrc \
//     tools/encode_lab.hip erasure_coding_test_amd/csrc/gf_host.cpp erasure_coding_test_amd/csrc/matrix_host.cpp \
//     -o tools/encode_lab.bin
//   tools/encode_lab.bin [--stripes 96] [--rounds 7] [--reps 10] [--skew-kib N]
//   tools/encode_lab.bin --skews 10,12,8,6 [--k 12 --m 4 --mib 16 --stripes 24]
//       the production launch on one slab per shard-stride skew (KiB), interleaved
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "gf_host.hpp"
#include "gf_kernels.hpp"
#include "matrix_host.hpp"
#include "shard_stride.hpp"

using namespace ecgpu;
using namespace ecgpu::dev;

#define CK(x)                                                                                 \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) {                                                                   \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                           \
    }                                                                                         \
  } while (0)

namespace lab {
// gf_apply<K, R, UNITS> (VEC 1, 3-bit slices, nt loads and stores) with a
// BS-thread workgroup.
template <int K, int R, int UNITS, int BS>
__global__ __launch_bounds__(BS) void enc_bs(ApplyArgs a) {
  const int64_t col = int64_t(blockIdx.x) * BS + threadIdx.x;
  if (col >= a.nvec) return;
  const int s = blockIdx.y;
  const uint8_t* const* sp = a.src + int64_t(s) * a.src_stride;
  uint8_t* dp[R];
#pragma unroll
  for (int r = 0; r < R; ++r) dp[r] = a.dst[int64_t(s) * a.dst_stride + a.row0 + r];
  u32x4 x[K];
#pragma unroll
  for (int j = 0; j < K; ++j) x[j] = load16t<1>(sp[j], col);
  combine_store<K, R, UNITS, 3, 1>(a, x, dp, col);
}

// Early unit row: for a Vandermonde encode (row 0 and column 0 all ones) row
// 0 is the XOR of the sources, stored right after the loads, before the
// multiply rows 1..R-1 are computed (production stores all R rows at the end).
template <int K, int R>
__global__ __launch_bounds__(256) void enc_early0(ApplyArgs a) {
  const int64_t col = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (col >= a.nvec) return;
  const int s = blockIdx.y;
  const uint8_t* const* sp = a.src + int64_t(s) * a.src_stride;
  uint8_t* dp[R];
#pragma unroll
  for (int r = 0; r < R; ++r) dp[r] = a.dst[int64_t(s) * a.dst_stride + a.row0 + r];
  u32x4 x[K];
#pragma unroll
  for (int j = 0; j < K; ++j) x[j] = load16t<1>(sp[j], col);
  u32x4 r0 = x[0];
#pragma unroll
  for (int j = 1; j < K; ++j) r0 ^= x[j];
  store16t<1>(dp[0], col, r0);
  u32x4 acc[R - 1];
  combine3<K, R - 1, kUnitCol0>((const kconst_u32*)a.ptab + K * kP3Words, x, acc);  // rows 1..R-1
#pragma unroll
  for (int r = 1; r < R; ++r) store16t<1>(dp[r], col, acc[r - 1]);
}
// Persistent, software-pipelined form (round 3 lab): a resident round of
// workgroups walks the (stripe, column block) items; a column's K sources are
// two chunks, double-buffered across items -- chunk 1's loads (and the next
// item's chunk 0) are in flight while the previous chunk is multiplied.  All
// loads and stores unconditional (the last prefetch re-reads the current
// item), so the wait counts are static.
template <int K, int R, int UNITS>
__global__ __launch_bounds__(256) void enc_pipe(ApplyArgs a, int stripes) {
  constexpr int CH = (K + 1) / 2;
  const int64_t nblk = a.nvec / 256, items = nblk * stripes, g = gridDim.x;
  int64_t it = blockIdx.x;
  if (it >= items) return;
  const kconst_u32* ptab = (const kconst_u32*)a.ptab;
  auto load = [&](u32x4 (&x)[CH], int64_t item, int c) {
    const int64_t s = item / nblk, col = (item - s * nblk) * 256 + threadIdx.x;
    const uint8_t* const* sp = a.src + s * a.src_stride;
#pragma unroll
    for (int u = 0; u < CH; ++u)
      if (c * CH + u < K) x[u] = load16t<1>(kload(sp, c * CH + u), col);
  };
  u32x4 b0[CH], b1[CH];
  load(b0, it, 0);
  for (;;) {
    const int64_t nx = it + g < items ? it + g : it;
    Xacc xa[R][4];
    auto apply = [&](const u32x4 (&x)[CH], int c) {
#pragma unroll
      for (int u = 0; u < CH; ++u) {
        const int j = c * CH + u;
        if (j >= K) break;
        Sel3 sl[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) sl[q] = sel3(x[u][q]);
#pragma unroll
        for (int r = 0; r < R; ++r) {
          if (is_unit<UNITS>(r, j)) {
#pragma unroll
            for (int q = 0; q < 4; ++q) xa[r][q].add(x[u][q]);
          } else {
            const kconst_u32* t = ptab + (r * K + j) * kP3Words;
#pragma unroll
            for (int q = 0; q < 4; ++q) mac3(xa[r][q], t, sl[q]);
          }
        }
      }
    };
    load(b1, it, 1);
    apply(b0, 0);
    load(b0, nx, 0);
    apply(b1, 1);
    const int64_t s = it / nblk, col = (it - s * nblk) * 256 + threadIdx.x;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      u32x4 o;
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q] = xa[r][q].value();
      store16t<1>(a.dst[s * a.dst_stride + a.row0 + r], col, o);
    }
    if (nx == it) break;
    it = nx;
  }
}

// The LDS nibble-table engine (gf_apply_lds) with the column's K source loads
// issued BEFORE the per-workgroup table staging and its barrier, so the HBM
// latency of the first (and only) loads overlaps the staging.
template <int K, int R>
__global__ __launch_bounds__(256) void lds_early(ApplyArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t lut[K * 32];
  const int64_t col = int64_t(blockIdx.x) * 256 + threadIdx.x;
  const bool live = col < a.nvec;
  const int s = blockIdx.y;
  const uint8_t* const* sp = a.src + int64_t(s) * a.src_stride;
  u32x4 x[K];
#pragma unroll
  for (int j = 0; j < K; ++j) x[j] = live ? load16t<1>(sp[j], col) : u32x4{0u, 0u, 0u, 0u};
  for (int i = threadIdx.x; i < K * 32; i += 256) {
    const int j = i >> 5, hv = i & 31;
    uint32_t e = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) e |= uint32_t(a.ntab[(r * K + j) * 32 + hv]) << (8 * r);
    lut[i] = e;
  }
  __syncthreads();
  if (!live) return;
  uint8_t* dp[R];
#pragma unroll
  for (int r = 0; r < R; ++r) dp[r] = a.dst[int64_t(s) * a.dst_stride + a.row0 + r];
  lds_u8* lb = (lds_u8*)lut;
  uint32_t e[4][4];
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int b = 0; b < 4; ++b) e[c][b] = 0u;
#pragma unroll
  for (int j = 0; j < K; ++j) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const uint32_t xl = (x[j][c] & 0x0F0F0F0Fu) << 2;
      const uint32_t xh = (x[j][c] >> 2) & 0x3C3C3C3Cu;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const uint32_t sel = 0x0C0C0C00u | uint32_t(b);
        const uint32_t lo = lds_word(lb, __builtin_amdgcn_perm(xl, xl, sel) + uint32_t(j * 128));
        const uint32_t hi = lds_word(lb, __builtin_amdgcn_perm(xh, xh, sel) + uint32_t(j * 128 + 64));
        e[c][b] = xor3(e[c][b], lo, hi);
      }
    }
  }
  u32x4 acc[R];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const uint32_t p01l = __builtin_amdgcn_perm(e[c][1], e[c][0], 0x05010400u);
    const uint32_t p23l = __builtin_amdgcn_perm(e[c][3], e[c][2], 0x05010400u);
    const uint32_t p01h = __builtin_amdgcn_perm(e[c][1], e[c][0], 0x07030602u);
    const uint32_t p23h = __builtin_amdgcn_perm(e[c][3], e[c][2], 0x07030602u);
    acc[0][c] = __builtin_amdgcn_perm(p23l, p01l, 0x05040100u);
    if constexpr (R > 1) acc[1][c] = __builtin_amdgcn_perm(p23l, p01l, 0x07060302u);
    if constexpr (R > 2) acc[2][c] = __builtin_amdgcn_perm(p23h, p01h, 0x05040100u);
    if constexpr (R > 3) acc[3][c] = __builtin_amdgcn_perm(p23h, p01h, 0x07060302u);
  }
#pragma unroll
  for (int r = 0; r < R; ++r) store16t<1>(dp[r], col, acc[r]);
}

// The production body with a workgroup barrier: WHERE 0 after the loads (the
// compiler waits for them first -- the LDS engine's early-load form has the
// same shape), 1 between the arithmetic and the stores, 2 after the loads
// without waiting for them (s_barrier alone).
template <int K, int R, int UNITS, int WHERE>
__global__ __launch_bounds__(256) void enc_sync(ApplyArgs a) {
  const int64_t col = int64_t(blockIdx.x) * 256 + threadIdx.x;
  const bool live = col < a.nvec;
  const int s = blockIdx.y;
  const uint8_t* const* sp = a.src + int64_t(s) * a.src_stride;
  uint8_t* dp[R];
#pragma unroll
  for (int r = 0; r < R; ++r) dp[r] = a.dst[int64_t(s) * a.dst_stride + a.row0 + r];
  u32x4 x[K];
#pragma unroll
  for (int j = 0; j < K; ++j) x[j] = live ? load16t<1>(sp[j], col) : u32x4{0u, 0u, 0u, 0u};
  if constexpr (WHERE == 0) __syncthreads();
  if constexpr (WHERE == 2) __builtin_amdgcn_s_barrier();
  u32x4 acc[R];
  combine<K, R, UNITS, 3>(a, x, acc);
  if constexpr (WHERE == 1) __syncthreads();
  if (!live) return;
#pragma unroll
  for (int r = 0; r < R; ++r) store16t<1>(dp[r], col, acc[r]);
}
// The production body with every source load issued before any arithmetic
// is scheduled: the source pointers are read first, then the K loads, then a
// scheduling barrier.  In the production ISA (hipcc 7.2, gf_apply<10,4,3>)
// the compiler issues six loads, waits for the first (vmcnt(5)) to start the
// selector arithmetic, and issues loads 7-10 a memory latency later -- the
// last two only after the coefficient tables' scalar loads (round 5).
template <int K, int R, int UNITS>
__global__ __launch_bounds__(256) void enc_sb(ApplyArgs a) {
  const int64_t col = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (col >= a.nvec) return;
  const int s = blockIdx.y;
  const uint8_t* const* sp = a.src + int64_t(s) * a.src_stride;
  const uint8_t* src[K];
#pragma unroll
  for (int j = 0; j < K; ++j) src[j] = sp[j];
  uint8_t* dp[R];
#pragma unroll
  for (int r = 0; r < R; ++r) dp[r] = a.dst[int64_t(s) * a.dst_stride + a.row0 + r];
  u32x4 x[K];
#pragma unroll
  for (int j = 0; j < K; ++j) x[j] = load16t<1>(src[j], col);
  __builtin_amdgcn_sched_barrier(0);
  combine_store<K, R, UNITS, 3, 1>(a, x, dp, col);
}
}  // namespace lab

bool g_early0 = false;  // --early0 1: skew mode also times lab::enc_early0 on every slab
bool g_vec2 = false;    // --vec2 1: ... and the production body with two columns per lane (VEC = 2)
bool g_dense = false;   // --dense 1: a C4-like dense 4 x 10 map (no 0 / 1 coefficients) instead of the encode
int g_sched = 0;        // --sched 1: production vs lab::enc_sb (all loads issued before the arithmetic)
bool g_lost = false;    // --lost 1 (with --m 1): the lost-parity decode's map -- row 2 of the RS(k,4) Vandermonde matrix
int g_lds = 0;          // --lds 1: the LDS nibble-table engine (production form and lab forms) beside the v_perm production;
                        // --lds 2: both engines at 3 workgroups per CU under dynamic LDS allocations of several sizes

struct Variant {
  std::string name;
  const void* fn;
  int bs;
  int blocks_per_cu;  // 0: uncapped
  unsigned lds = 0;   // > 0: this dynamic LDS allocation instead of the blocks_per_cu rule
  int cols = 0;       // > 0: columns per workgroup when it is not bs (VEC > 1 forms)
};

// builds the production 3-bit-slice tables (ecgpu_runtime.hip build_tables)
static void build_p3(int c, uint32_t* p3) {
  const auto& T = gf8().mul[c & 0xFF];
  for (int i = 0; i < kP3Words; ++i) p3[i] = 0;
  for (int e = 0; e < 8; ++e) {
    p3[e >> 2] |= uint32_t(T[e]) << (8 * (e & 3));
    p3[2 + (e >> 2)] |= uint32_t(T[e << 3]) << (8 * (e & 3));
  }
  for (int e = 0; e < 4; ++e) p3[4] |= uint32_t(T[e << 6]) << (8 * e);
}

// Shard contents.  HBM throughput depends on the data: the production encode
// on the C3 layout takes 888-900 us on independent random shards (the bench),
// 867-880 us when every shard holds the same random bytes (parity row 0 is
// then all zeros) and 844 us on zeros (tools/probe_step.py,
// profiles/r03_data_dependence.jsonl).  So every data shard here is its own
// 8-B-aligned window of a 2*S random pool: independent-looking shards, whose
// parity is as random as the bench's.
std::vector<uint8_t> random_pool(size_t S, uint64_t seed) {
  std::vector<uint8_t> h(2 * S);
  std::mt19937_64 g(seed);
  for (size_t i = 0; i + 8 <= h.size(); i += 8) {
    const uint64_t x = g();
    std::memcpy(&h[i], &x, 8);
  }
  return h;
}

size_t window(size_t S, int shard) { return (size_t(shard) * 0x9E3779B1ull % (S / 8)) * 8; }

template <int k, int m>
int skew_ab(int stripes, int kib, const std::vector<int>& skews, int rounds, int reps);
template <int k, int m>
int variant_ab(int stripes, size_t S, int skew_kib, int rounds, int reps);
int g_skew_unit = 1024;  // --skew-unit B: the --skews values in units of B bytes (default KiB; a multiple of 256)
int g_sync = 0;  // --sync 1: the production body with workgroup barriers (lab::enc_sync) and the LDS engine, at the library's cap

int main(int argc, char** argv) {
  int stripes = 96, rounds = 7, reps = 10, kk = 10, mm = 4, kib = 4096, skew_kib = -1;
  std::vector<int> skews;
  for (int i = 1; i + 1 < argc; i += 2) {
    const std::string f = argv[i];
    if (f == "--stripes") stripes = std::atoi(argv[i + 1]);
    else if (f == "--rounds") rounds = std::atoi(argv[i + 1]);
    else if (f == "--reps") reps = std::atoi(argv[i + 1]);
    else if (f == "--k") kk = std::atoi(argv[i + 1]);
    else if (f == "--m") mm = std::atoi(argv[i + 1]);
    else if (f == "--mib") kib = 1024 * std::atoi(argv[i + 1]);
    else if (f == "--kib") kib = std::atoi(argv[i + 1]);
    else if (f == "--early0") g_early0 = std::atoi(argv[i + 1]) != 0;
    else if (f == "--vec2") g_vec2 = std::atoi(argv[i + 1]) != 0;
    else if (f == "--dense") g_dense = std::atoi(argv[i + 1]) != 0;
    else if (f == "--lds") g_lds = std::atoi(argv[i + 1]);
    else if (f == "--sync") g_sync = std::atoi(argv[i + 1]);
    else if (f == "--sched") g_sched = std::atoi(argv[i + 1]);
    else if (f == "--lost") g_lost = std::atoi(argv[i + 1]) != 0;
    else if (f == "--skew-kib") skew_kib = std::atoi(argv[i + 1]);
    else if (f == "--skew-unit") g_skew_unit = std::atoi(argv[i + 1]);
    else if (f == "--skews") {
      std::string v = argv[i + 1];
      size_t p = 0;
      while (p < v.size()) {
        const size_t q = v.find(',', p);
        skews.push_back(std::atoi(v.substr(p, q - p).c_str()));
        p = q == std::string::npos ? v.size() : q + 1;
      }
    }
  }
  if (!skews.empty()) {
    if (stripes <= 0) stripes = std::max(1, int((5ll << 30) / ((long long)(kk + mm) * kib * 1024)));  // ~5 GiB per launch
    if (kk == 10 && mm == 4) return skew_ab<10, 4>(stripes, kib, skews, rounds, reps);
    if (kk == 12 && mm == 4) return skew_ab<12, 4>(stripes, kib, skews, rounds, reps);
    if (kk == 6 && mm == 3) return skew_ab<6, 3>(stripes, kib, skews, rounds, reps);
    if (kk == 4 && mm == 2) return skew_ab<4, 2>(stripes, kib, skews, rounds, reps);
    std::fprintf(stderr, "skew A/B covers RS(10,4), RS(12,4), RS(6,3), RS(4,2)\n");
    return 2;
  }
  if (kk == 10 && mm == 4) return variant_ab<10, 4>(stripes, size_t(kib) << 10, skew_kib, rounds, reps);
  if (kk == 6 && mm == 3) return variant_ab<6, 3>(stripes, size_t(kib) << 10, skew_kib, rounds, reps);
  if (kk == 12 && mm == 4) return variant_ab<12, 4>(stripes, size_t(kib) << 10, skew_kib, rounds, reps);
  if (kk == 10 && mm == 1) return variant_ab<10, 1>(stripes, size_t(kib) << 10, skew_kib, rounds, reps);
  if (kk == 6 && mm == 1) return variant_ab<6, 1>(stripes, size_t(kib) << 10, skew_kib, rounds, reps);
  std::fprintf(stderr, "variant A/B covers RS(10,4), RS(6,3), RS(12,4), and (10,1) / (6,1) with --lost 1\n");
  return 2;
}

// Every variant of the selected mode on one slab of `stripes` RS(k,m) stripes
// of S-byte shards at the library's stride (or S + skew_kib KiB).
template <int k, int m>
int variant_ab(int stripes, size_t S, int skew_kib, int rounds, int reps) {
  const size_t stride = skew_kib >= 0 ? S + size_t(skew_kib) * 1024 : size_t(shard_stride(int64_t(S)));
  int* M = vandermonde_coding_matrix(k, m, 8);
  if (g_lost) {  // the re-encode of a lost parity shard: row 2 of RS(k, 4), column 0 a one
    int* M4 = vandermonde_coding_matrix(k, 4, 8);
    for (int j = 0; j < k * m; ++j) M[j] = M4[2 * k + j % k];
    std::free(M4);
  }
  if (g_dense) {
    std::mt19937 gm(4);
    for (int i = 0; i < k * m; ++i) M[i] = 2 + int(gm() % 254);  // no 0 / 1: every term multiplies (C4's decode rows)
  }
  std::vector<uint32_t> ptab(size_t(m) * k * kP3Words);
  for (int r = 0; r < m; ++r)
    for (int j = 0; j < k; ++j) build_p3(M[r * k + j], &ptab[(size_t(r) * k + j) * kP3Words]);
  // the LDS engine's per-coefficient nibble tables (ecgpu_runtime.hip): c*v, then c*(v << 4)
  std::vector<uint8_t> ntab(size_t(m) * k * 32);
  for (int r = 0; r < m; ++r)
    for (int j = 0; j < k; ++j)
      for (int v = 0; v < 16; ++v) {
        ntab[(size_t(r) * k + j) * 32 + v] = uint8_t(single_multiply(M[r * k + j], v, 8));
        ntab[(size_t(r) * k + j) * 32 + 16 + v] = uint8_t(single_multiply(M[r * k + j], v << 4, 8));
      }
  uint8_t* slab = nullptr;
  const size_t slab_bytes = stride * size_t(k + m) * size_t(stripes);
  CK(hipMalloc(&slab, slab_bytes));
  {
    const std::vector<uint8_t> h = random_pool(S, 11);
    for (int s = 0; s < stripes; ++s)
      for (int j = 0; j < k; ++j)
        CK(hipMemcpy(slab + stride * (size_t(s) * (k + m) + j), h.data() + window(S, s * k + j), S,
                     hipMemcpyHostToDevice));
  }
  std::vector<const uint8_t*> hs;
  std::vector<uint8_t*> hd;
  for (int s = 0; s < stripes; ++s) {
    for (int j = 0; j < k; ++j) hs.push_back(slab + stride * (size_t(s) * (k + m) + j));
    for (int r = 0; r < m; ++r) hd.push_back(slab + stride * (size_t(s) * (k + m) + k + r));
  }
  const uint8_t** d_src = nullptr;
  uint8_t** d_dst = nullptr;
  uint32_t* d_ptab = nullptr;
  CK(hipMalloc(&d_src, sizeof(void*) * hs.size()));
  CK(hipMalloc(&d_dst, sizeof(void*) * hd.size()));
  CK(hipMalloc(&d_ptab, 4 * ptab.size()));
  CK(hipMemcpy(d_src, hs.data(), sizeof(void*) * hs.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(d_dst, hd.data(), sizeof(void*) * hd.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(d_ptab, ptab.data(), 4 * ptab.size(), hipMemcpyHostToDevice));
  uint8_t* d_ntab = nullptr;
  CK(hipMalloc(&d_ntab, ntab.size()));
  CK(hipMemcpy(d_ntab, ntab.data(), ntab.size(), hipMemcpyHostToDevice));
  ApplyArgs a{};
  a.ptab = d_ptab;
  a.ntab = d_ntab;
  a.src = d_src;
  a.dst = d_dst;
  a.nvec = int64_t(S / 16);
  a.size = int64_t(S);
  a.byte0 = a.nvec * 16;
  a.src_stride = k;
  a.dst_stride = m;
  a.row0 = 0;
  a.K = k;
  a.R = m;
  a.nt = 1;
  constexpr int U = m == 1 ? kUnitCol0 : kUnitCol0 | kUnitRow0, N = kUnitNone;
  // bs < 0: the persistent pipelined form (a resident round of |bs| workgroups per CU)
  using V = Variant;
  const void* const vperm = reinterpret_cast<const void*>(&gf_apply<k, m, U, 1, 3, 3>);
  const void* const ldsk = reinterpret_cast<const void*>(&gf_apply_lds<k, m>);
  const int cap = k + m <= 9 ? 4 : 3;  // ecgpu_runtime.hip residency_lds_bytes
  const unsigned lds_cap = ((unsigned(163840 / cap) & ~511u) - 128u * k - 4096u) & ~4095u;
  std::vector<Variant> vs = g_sched == 2 ? std::vector<Variant>{  // the R = 1 levers (lost parity)
      V{"prod", vperm, 256, cap},
      V{"vec2_cap2", reinterpret_cast<const void*>(&gf_apply<k, m, U, 2, 3, 3>), 256, 2, 0, 512},
      V{"vec2_cap3", reinterpret_cast<const void*>(&gf_apply<k, m, U, 2, 3, 3>), 256, 3, 0, 512},
      V{"vec2_uncapped", reinterpret_cast<const void*>(&gf_apply<k, m, U, 2, 3, 3>), 256, 0, 0, 512},
      V{"pipe_r3", reinterpret_cast<const void*>(&lab::enc_pipe<k, m, U>), -3, 0},
      V{"pipe_r4", reinterpret_cast<const void*>(&lab::enc_pipe<k, m, U>), -4, 0},
      V{"pipe_r6", reinterpret_cast<const void*>(&lab::enc_pipe<k, m, U>), -6, 0},
      V{"lds_engine", ldsk, 256, cap, lds_cap},
      V{"prod_cap2", vperm, 256, 2},
      V{"bs512_cap2", reinterpret_cast<const void*>(&lab::enc_bs<k, m, U, 512>), 512, 2},
  } : g_sched ? (g_dense ? std::vector<Variant>{
      V{"prod_dense_uncapped", reinterpret_cast<const void*>(&gf_apply<k, m, N, 1, 3, 3>), 256, 0},
      V{"sb_dense_uncapped", reinterpret_cast<const void*>(&lab::enc_sb<k, m, N>), 256, 0},
      V{"prod_dense_cap3", reinterpret_cast<const void*>(&gf_apply<k, m, N, 1, 3, 3>), 256, 3},
      V{"sb_dense_cap3", reinterpret_cast<const void*>(&lab::enc_sb<k, m, N>), 256, 3},
  } : std::vector<Variant>{
      V{"prod", vperm, 256, cap},
      V{"sb", reinterpret_cast<const void*>(&lab::enc_sb<k, m, U>), 256, cap},
      V{"prod_cap_plus1", vperm, 256, cap + 1},
      V{"sb_cap_plus1", reinterpret_cast<const void*>(&lab::enc_sb<k, m, U>), 256, cap + 1},
      V{"prod_uncapped", vperm, 256, 0},
      V{"sb_uncapped", reinterpret_cast<const void*>(&lab::enc_sb<k, m, U>), 256, 0},
  }) : g_sync ? std::vector<Variant>{
      V{"prod", vperm, 256, cap},
      V{"sync_after_loads", reinterpret_cast<const void*>(&lab::enc_sync<k, m, U, 0>), 256, cap},
      V{"sync_before_stores", reinterpret_cast<const void*>(&lab::enc_sync<k, m, U, 1>), 256, cap},
      V{"barrier_no_wait", reinterpret_cast<const void*>(&lab::enc_sync<k, m, U, 2>), 256, cap},
      V{"lds_engine", ldsk, 256, cap, lds_cap},
  } : g_lds == 2 ? std::vector<Variant>{
      V{"prod_bs256_cap3", vperm, 256, 3},
      V{"vperm_dyn41472", vperm, 256, 3, 41472},
      V{"vperm_dyn45056", vperm, 256, 3, 45056},
      V{"vperm_dyn49152", vperm, 256, 3, 49152},
      V{"vperm_dyn52224", vperm, 256, 3, 52224},
      V{"lds_dyn40960", ldsk, 256, 3, 40960},
      V{"lds_dyn45056", ldsk, 256, 3, 45056},
      V{"lds_dyn49152", ldsk, 256, 3, 49152},
      V{"lds_dyn52736", ldsk, 256, 3, 52736},
  } : g_lds ? std::vector<Variant>{
      {"prod_bs256_cap3", reinterpret_cast<const void*>(&gf_apply<k, m, U, 1, 3, 3>), 256, 3},
      {"prod_lds", reinterpret_cast<const void*>(&gf_apply_lds<k, m>), 256, 0},
      {"lds_cap3", reinterpret_cast<const void*>(&gf_apply_lds<k, m>), 256, 3},
      {"lds_cap4", reinterpret_cast<const void*>(&gf_apply_lds<k, m>), 256, 4},
      {"lds_early", reinterpret_cast<const void*>(&lab::lds_early<k, m>), 256, 0},
      {"lds_early_cap3", reinterpret_cast<const void*>(&lab::lds_early<k, m>), 256, 3},
      {"lds_early_cap4", reinterpret_cast<const void*>(&lab::lds_early<k, m>), 256, 4},
  } : g_dense ? std::vector<Variant>{
      {"prod_dense_cap3", reinterpret_cast<const void*>(&gf_apply<k, m, N, 1, 3, 3>), 256, 3},
      {"dense_cap4", reinterpret_cast<const void*>(&gf_apply<k, m, N, 1, 3, 3>), 256, 4},
      {"dense_uncapped", reinterpret_cast<const void*>(&gf_apply<k, m, N, 1, 3, 3>), 256, 0},
      {"pipe_dense_r3", reinterpret_cast<const void*>(&lab::enc_pipe<k, m, N>), -3, 0},
      {"pipe_dense_r4", reinterpret_cast<const void*>(&lab::enc_pipe<k, m, N>), -4, 0},
      {"pipe_dense_r5", reinterpret_cast<const void*>(&lab::enc_pipe<k, m, N>), -5, 0},
  } : std::vector<Variant>{
      {"prod_bs256_cap3", reinterpret_cast<const void*>(&gf_apply<k, m, U, 1, 3, 3>), 256, 3},
      {"bs256_cap4", reinterpret_cast<const void*>(&gf_apply<k, m, U, 1, 3, 3>), 256, 4},
      {"pipe_r3", reinterpret_cast<const void*>(&lab::enc_pipe<k, m, U>), -3, 0},
      {"pipe_r4", reinterpret_cast<const void*>(&lab::enc_pipe<k, m, U>), -4, 0},
      {"bs256_cap2", reinterpret_cast<const void*>(&gf_apply<k, m, U, 1, 3, 3>), 256, 2},
      {"bs512_cap1", reinterpret_cast<const void*>(&lab::enc_bs<k, m, U, 512>), 512, 1},
      {"bs512_cap2", reinterpret_cast<const void*>(&lab::enc_bs<k, m, U, 512>), 512, 2},
      {"bs512_cap3", reinterpret_cast<const void*>(&lab::enc_bs<k, m, U, 512>), 512, 3},
      {"bs1024_cap1", reinterpret_cast<const void*>(&lab::enc_bs<k, m, U, 1024>), 1024, 1},
      {"bs1024_cap2", reinterpret_cast<const void*>(&lab::enc_bs<k, m, U, 1024>), 1024, 2},
  };
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  int dev = 0, lds_cu = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&lds_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev));
  auto lds_of = [&](const Variant& v) -> unsigned {
    if (v.lds > 0) return v.lds;
    if (v.blocks_per_cu <= 0) return 0u;
    const unsigned b = unsigned(lds_cu / v.blocks_per_cu) & ~511u;
    return b > unsigned(lds_cu / (v.blocks_per_cu + 1)) ? b : 0u;
  };
  auto launch = [&](const Variant& v) {
    ApplyArgs args = a;
    int ns = stripes;
    void* kargs[] = {&args, &ns};
    if (v.bs < 0) {  // persistent: one resident round, items = column blocks x stripes
      CK(hipLaunchKernel(v.fn, dim3(unsigned(-v.bs * cus)), dim3(256), kargs, 0, nullptr));
      return;
    }
    const int per = v.cols > 0 ? v.cols : v.bs;
    const dim3 grid(unsigned((a.nvec + per - 1) / per), unsigned(stripes));
    CK(hipLaunchKernel(v.fn, grid, dim3(unsigned(v.bs)), kargs, lds_of(v), nullptr));
  };
  // reference: the production launch; spot-check it against the host
  launch(vs[0]);
  CK(hipDeviceSynchronize());
  std::vector<uint8_t> want(S), got(S);
  {
    std::mt19937_64 g(5);
    for (int n = 0; n < 200; ++n) {
      const int s = int(g() % size_t(stripes));
      const size_t b = g() % S;
      uint8_t col[k];
      for (int j = 0; j < k; ++j) CK(hipMemcpy(&col[j], hs[size_t(s * k + j)] + b, 1, hipMemcpyDeviceToHost));
      for (int r = 0; r < m; ++r) {
        uint8_t e = 0;
        for (int j = 0; j < k; ++j) e ^= uint8_t(single_multiply(M[r * k + j], col[j], 8));
        uint8_t o;
        CK(hipMemcpy(&o, hd[size_t(s * m + r)] + b, 1, hipMemcpyDeviceToHost));  // (dense: M was overwritten above)
        if (o != e) {
          std::fprintf(stderr, "production launch disagrees with the host\n");
          return 1;
        }
      }
    }
  }
  // every variant must reproduce the production outputs (two stripes compared whole)
  std::vector<std::vector<uint8_t>> ref;
  for (int s : {0, stripes - 1})
    for (int r = 0; r < m; ++r) {
      ref.emplace_back(S);
      CK(hipMemcpy(ref.back().data(), hd[size_t(s * m + r)], S, hipMemcpyDeviceToHost));
    }
  for (size_t v = 1; v < vs.size(); ++v) {
    for (int s : {0, stripes - 1})
      for (int r = 0; r < m; ++r) CK(hipMemset(hd[size_t(s * m + r)], 0, S));
    launch(vs[v]);
    CK(hipDeviceSynchronize());
    size_t i = 0;
    for (int s : {0, stripes - 1})
      for (int r = 0; r < m; ++r) {
        CK(hipMemcpy(got.data(), hd[size_t(s * m + r)], S, hipMemcpyDeviceToHost));
        if (got != ref[i++]) {
          std::fprintf(stderr, "variant %s differs\n", vs[v].name.c_str());
          return 1;
        }
      }
  }
  std::vector<std::vector<float>> t(vs.size());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int rd = 0; rd < rounds; ++rd)
    for (size_t v = 0; v < vs.size(); ++v) {
      for (int q = 0; q < 2; ++q) launch(vs[v]);
      for (int q = 0; q < reps; ++q) {
        CK(hipEventRecord(e0, nullptr));
        launch(vs[v]);
        CK(hipEventRecord(e1, nullptr));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        t[v].push_back(ms * 1000.f);
      }
    }
  const double bytes = double(k + m) * double(S) * stripes;
  for (size_t v = 0; v < vs.size(); ++v) {
    std::sort(t[v].begin(), t[v].end());
    const double med = t[v][t[v].size() / 2];
    std::printf("{\"variant\": \"%s\", \"block\": %d, \"blocks_per_cu\": %d, \"dyn_lds\": %u, \"stripes\": %d, \"median_us\": %.1f, "
                "\"min_us\": %.1f, \"GBps\": %.0f, \"frac\": %.4f}\n",
                vs[v].name.c_str(), vs[v].bs, vs[v].blocks_per_cu, lds_of(vs[v]), stripes, med, double(t[v][0]),
                bytes / med / 1e3, bytes / med / 1e3 / 8000.0);
  }
  return 0;
}

// One slab per skew, the production launch (unit structure col 0 / row 0,
// nt loads and stores, the library's residency rule) on each, interleaved.
// Parity of every slab's first and last stripe is checked against the host.
template <int k, int m>
int skew_ab(int stripes, int kib, const std::vector<int>& skews, int rounds, int reps) {
  const size_t S = size_t(kib) << 10;
  int* M = vandermonde_coding_matrix(k, m, 8);
  std::vector<uint32_t> ptab(size_t(m) * k * kP3Words);
  for (int r = 0; r < m; ++r)
    for (int j = 0; j < k; ++j) build_p3(M[r * k + j], &ptab[(size_t(r) * k + j) * kP3Words]);
  uint32_t* d_ptab = nullptr;
  CK(hipMalloc(&d_ptab, 4 * ptab.size()));
  CK(hipMemcpy(d_ptab, ptab.data(), 4 * ptab.size(), hipMemcpyHostToDevice));
  int dev = 0, lds_cu = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&lds_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev));
  const int blocks = k + m <= 9 ? 4 : 3;  // ecgpu_runtime.hip residency_lds_bytes
  const unsigned lds = unsigned(lds_cu / blocks) & ~511u;
  constexpr int U = kUnitCol0 | kUnitRow0;
  const void* fn = reinterpret_cast<const void*>(&gf_apply<k, m, U, 1, 3, 3>);
  const void* fn_e = g_vec2 ? reinterpret_cast<const void*>(&gf_apply<k, m, U, 2, 3, 3>)
                            : reinterpret_cast<const void*>(&lab::enc_early0<k, m>);
  const int per_e = g_vec2 ? 512 : 256;  // columns per workgroup of the variant
  if (g_vec2) g_early0 = true;           // the variant slot times VEC = 2 instead
  struct Slab {
    int skew;
    uint8_t* base;
    size_t stride;
    ApplyArgs a;
    std::vector<float> t, te;
  };
  std::vector<Slab> slabs;
  const std::vector<uint8_t> h = random_pool(S, 17);
  for (int sk : skews) {
    Slab sl{};
    sl.skew = sk;
    sl.stride = ((S + 255) & ~size_t(255)) + size_t(sk) * size_t(g_skew_unit);
    CK(hipMalloc(&sl.base, sl.stride * size_t(k + m) * size_t(stripes)));
    std::vector<const uint8_t*> hs;
    std::vector<uint8_t*> hd;
    for (int s = 0; s < stripes; ++s) {
      for (int j = 0; j < k; ++j) {
        uint8_t* p = sl.base + sl.stride * (size_t(s) * (k + m) + j);
        CK(hipMemcpy(p, h.data() + window(S, s * k + j), S, hipMemcpyHostToDevice));
        hs.push_back(p);
      }
      for (int r = 0; r < m; ++r) hd.push_back(sl.base + sl.stride * (size_t(s) * (k + m) + k + r));
    }
    const uint8_t** d_src = nullptr;
    uint8_t** d_dst = nullptr;
    CK(hipMalloc(&d_src, sizeof(void*) * hs.size()));
    CK(hipMalloc(&d_dst, sizeof(void*) * hd.size()));
    CK(hipMemcpy(d_src, hs.data(), sizeof(void*) * hs.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_dst, hd.data(), sizeof(void*) * hd.size(), hipMemcpyHostToDevice));
    ApplyArgs& a = sl.a;
    a.ptab = d_ptab;
    a.src = d_src;
    a.dst = d_dst;
    a.nvec = int64_t(S / 16);
    a.size = int64_t(S);
    a.byte0 = a.nvec * 16;
    a.src_stride = k;
    a.dst_stride = m;
    a.K = k;
    a.R = m;
    a.nt = 1;
    slabs.push_back(sl);
  }
  auto launch = [&](Slab& sl, const void* f = nullptr) {
    ApplyArgs args = sl.a;
    void* kargs[] = {&args};
    const int per = f == fn_e ? per_e : 256;
    CK(hipLaunchKernel(f ? f : fn, dim3(unsigned((sl.a.nvec + per - 1) / per), unsigned(stripes)), dim3(256), kargs,
                       lds, nullptr));
  };
  for (int pass = 0; pass < (g_early0 ? 2 : 1); ++pass)
  for (auto& sl : slabs) {  // host spot check of stripe 0 and the last (pass 1: enc_early0)
    if (pass == 1) CK(hipMemset(sl.base + sl.stride * size_t(k), 0, sl.stride * size_t(m)));  // stripe 0's parity
    launch(sl, pass ? fn_e : fn);
    CK(hipDeviceSynchronize());
    std::mt19937_64 q(9);
    for (int n = 0; n < 64; ++n) {
      const int s = (n & 1) ? stripes - 1 : 0;
      const size_t b = q() % S;
      uint8_t col[k];
      for (int j = 0; j < k; ++j)
        CK(hipMemcpy(&col[j], sl.base + sl.stride * (size_t(s) * (k + m) + j) + b, 1, hipMemcpyDeviceToHost));
      for (int r = 0; r < m; ++r) {
        uint8_t e = 0, o = 0;
        for (int j = 0; j < k; ++j) e ^= uint8_t(single_multiply(M[r * k + j], col[j], 8));
        CK(hipMemcpy(&o, sl.base + sl.stride * (size_t(s) * (k + m) + k + r) + b, 1, hipMemcpyDeviceToHost));
        if (o != e) {
          std::fprintf(stderr, "skew %d: parity disagrees with the host\n", sl.skew);
          return 1;
        }
      }
    }
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int rd = 0; rd < rounds; ++rd)
    for (auto& sl : slabs) {
      for (int w = 0; w < 2; ++w) launch(sl);
      for (int q = 0; q < reps; ++q) {
        CK(hipEventRecord(e0, nullptr));
        launch(sl);
        CK(hipEventRecord(e1, nullptr));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        sl.t.push_back(ms * 1000.f);
      }
      if (!g_early0) continue;
      for (int w = 0; w < 2; ++w) launch(sl, fn_e);
      for (int q = 0; q < reps; ++q) {
        CK(hipEventRecord(e0, nullptr));
        launch(sl, fn_e);
        CK(hipEventRecord(e1, nullptr));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        sl.te.push_back(ms * 1000.f);
      }
    }
  const double bytes = double(k + m) * double(S) * stripes;
  for (auto& sl : slabs) {
    std::sort(sl.t.begin(), sl.t.end());
    const double med = sl.t[sl.t.size() / 2];
    std::printf("{\"k\": %d, \"m\": %d, \"shard_kib\": %d, \"stripes\": %d, \"skew_kib\": %.2f, \"skew_bytes\": %lld, "
                "\"median_us\": %.1f, \"min_us\": %.1f, \"GBps\": %.0f, \"frac\": %.4f}\n",
                k, m, kib, stripes, sl.skew * double(g_skew_unit) / 1024.0, (long long)sl.skew * g_skew_unit, med,
                double(sl.t[0]), bytes / med / 1e3, bytes / med / 1e3 / 8000.0);
    if (!g_early0) continue;
    std::sort(sl.te.begin(), sl.te.end());
    const double me = sl.te[sl.te.size() / 2];
    std::printf("{\"variant\": \"%s\", \"k\": %d, \"m\": %d, \"shard_kib\": %d, \"stripes\": %d, \"skew_kib\": %d, "
                "\"median_us\": %.1f, \"min_us\": %.1f, \"GBps\": %.0f, \"vs_prod\": %.4f}\n",
                g_vec2 ? "vec2" : "early0", k, m, kib, stripes, sl.skew, me, double(sl.te[0]), bytes / me / 1e3, med / me);
  }
  return 0;
}
