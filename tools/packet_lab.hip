// packet_lab.hip -- A/B lab for the GF(2) bit-matrix packet kernels: an
// RS(10,4) w = 8 bit-matrix encode (jerasure_bitmatrix_encode's map: 80
// source packet rows -> 32 output packet rows per super-packet) over one
// stripe of S-byte device shards at the library's skewed stride.  Variants
// are checked bit-exact against the production kernel, which is checked
// against a host XOR of the same map on sample columns, then timed in
// interleaved rounds with HIP events.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include -I erasure_coding_test_amd/csrc \
//     tools/packet_lab.hip erasure_coding_test_amd/csrc/gf_host.cpp erasure_coding_test_amd/csrc/matrix_host.cpp \
//     -o tools/packet_lab.bin
//   tools/packet_lab.bin [--mib 64] [--ps 4096] [--rounds 9] [--reps 10] [--skew-kib N] [--only name,name]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <type_traits>
#include <vector>

#include "gf_host.hpp"
#include "gf_kernels.hpp"
#include "matrix_host.hpp"
#include "shard_stride.hpp"

using namespace ecgpu;
using namespace ecgpu::dev;

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));   \
      std::exit(1);                                                                             \
    }                                                                                           \
  } while (0)

namespace lab {
// The round-2 form: generic loads of the pointer / mask tables (vector
// loads once a store has been issued).
template <int RT>
__global__ __launch_bounds__(kBlock) void packets16p_r2(PacketArgs a) {
  const int64_t g = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (g >= a.ncols) return;
  int64_t sp, col;
  packet_coords(a, g, &sp, &col);
  const int64_t soff = sp * a.sstride + col * 16, doff = sp * a.dstride + col * 16;
  uint32_t acc[RT][4];
#pragma unroll
  for (int r = 0; r < RT; ++r) acc[r][0] = acc[r][1] = acc[r][2] = acc[r][3] = 0u;
  const int nc = a.nsrc >> 2;
  u32x4 xa[4], xb[4];
  uint32_t ma[4], mb[4];
  auto load4 = [&](u32x4 (&x)[4], uint32_t (&m)[4], int c) {
    const int b = (c < nc ? c : nc - 1) * 4;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      m[u] = a.mask[b + u];
      x[u] = load16t<1>(a.src[b + u] + soff, 0);
    }
  };
  auto apply4 = [&](const u32x4 (&x)[4], const uint32_t (&m)[4]) {
#pragma unroll
    for (int u = 0; u < 4; ++u) xor_masked16<RT, 4>(acc, x[u], m[u]);
  };
  if (nc > 0) {
    load4(xa, ma, 0);
    for (int c = 0; c < nc; c += 2) {
      load4(xb, mb, c + 1);
      apply4(xa, ma);
      if (c + 1 >= nc) break;
      load4(xa, ma, c + 2);
      apply4(xb, mb);
    }
  }
  for (int j = nc * 4; j < a.nsrc; ++j) xor_masked16<RT, 4>(acc, load16t<1>(a.src[j] + soff, 0), a.mask[j]);
#pragma unroll
  for (int r = 0; r < RT; ++r)
    if (r < a.R) store16t<1>(a.dst[r] + doff, 0, u32x4{acc[r][0], acc[r][1], acc[r][2], acc[r][3]});
}
// Output rows split across the waves of a workgroup: SPLIT waves share one
// 64-column block and each keeps RT = 32 / SPLIT rows, so a wave holds
// 4·RT accumulator VGPRs instead of 128 (more waves resident per SIMD); the
// SPLIT waves read the same source lines, the later ones from cache.  NT
// selects non-temporal source loads.
template <int RT, int SPLIT, int NT>
__global__ __launch_bounds__(kBlock) void packets16p_split(PacketArgs a) {
  const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
  const int half = wave % SPLIT;
  const int64_t g = int64_t(blockIdx.x) * (kBlock / SPLIT) + (wave / SPLIT) * 64 + (threadIdx.x & 63);
  if (g >= a.ncols) return;
  int64_t sp, col;
  packet_coords(a, g, &sp, &col);
  const int64_t soff = sp * a.sstride + col * 16, doff = sp * a.dstride + col * 16;
  uint32_t acc[RT][4];
#pragma unroll
  for (int r = 0; r < RT; ++r) acc[r][0] = acc[r][1] = acc[r][2] = acc[r][3] = 0u;
  const int nc = a.nsrc >> 2;
  const int shift = half * RT;
  u32x4 xa[4], xb[4];
  uint32_t ma[4], mb[4];
  auto load4 = [&](u32x4 (&x)[4], uint32_t (&m)[4], int c) {
    const int b = (c < nc ? c : nc - 1) * 4;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      m[u] = a.mask[b + u] >> shift;
      x[u] = load16t<NT>(a.src[b + u] + soff, 0);
    }
  };
  auto apply4 = [&](const u32x4 (&x)[4], const uint32_t (&m)[4]) {
#pragma unroll
    for (int u = 0; u < 4; ++u) xor_masked16<RT, 4>(acc, x[u], m[u]);
  };
  if (nc > 0) {
    load4(xa, ma, 0);
    for (int c = 0; c < nc; c += 2) {
      load4(xb, mb, c + 1);
      apply4(xa, ma);
      if (c + 1 >= nc) break;
      load4(xa, ma, c + 2);
      apply4(xb, mb);
    }
  }
  for (int j = nc * 4; j < a.nsrc; ++j) xor_masked16<RT, 4>(acc, load16t<NT>(a.src[j] + soff, 0), a.mask[j] >> shift);
#pragma unroll
  for (int r = 0; r < RT; ++r)
    if (shift + r < a.R) store16t<1>(a.dst[shift + r] + doff, 0, u32x4{acc[r][0], acc[r][1], acc[r][2], acc[r][3]});
}
// Deeper source pipeline: chunks of CH source rows in NB rotating buffers, so
// (NB - 1) * CH + CH loads of 1 KiB per wave can be in flight (production: 2
// buffers of 4).  More VGPRs (2 waves per SIMD instead of 3) for more bytes
// in flight per SIMD.  Chunk indices past the last full chunk re-read it.
template <int RT, int CH, int NB>
__global__ __launch_bounds__(kBlock) void packets16_ring(PacketArgs a) {
  static_assert(NB == 2 || NB == 3, "ring of 2 or 3 chunk buffers");
  const int64_t g = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (g >= a.ncols) return;
  int64_t sp, col;
  packet_coords(a, g, &sp, &col);
  const int64_t soff = sp * a.sstride + col * 16, doff = sp * a.dstride + col * 16;
  uint32_t acc[RT][4];
#pragma unroll
  for (int r = 0; r < RT; ++r) acc[r][0] = acc[r][1] = acc[r][2] = acc[r][3] = 0u;
  const int nc = a.nsrc / CH;
  u32x4 x[NB][CH];
  uint32_t msk[NB][CH];
  // buffer indices are template constants so the ring stays in registers
  auto load = [&](auto bc, int c) {
    constexpr int b = decltype(bc)::value;
    const int base = (c < nc ? c : nc - 1) * CH;
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      msk[b][u] = a.mask[base + u];
      x[b][u] = load16t<1>(a.src[base + u] + soff, 0);
    }
  };
  auto apply = [&](auto bc) {
    constexpr int b = decltype(bc)::value;
#pragma unroll
    for (int u = 0; u < CH; ++u) xor_masked16<RT, 4>(acc, x[b][u], msk[b][u]);
  };
  auto step = [&](auto bc, int c) -> bool {  // false: past the last chunk
    constexpr int b = decltype(bc)::value;
    load(std::integral_constant<int, (b + NB - 1) % NB>{}, c + b + NB - 1);
    if (c + b >= nc) return false;
    apply(bc);
    return true;
  };
  if (nc > 0) {
    load(std::integral_constant<int, 0>{}, 0);
    if constexpr (NB > 2) load(std::integral_constant<int, 1>{}, 1);
    for (int c = 0; c < nc; c += NB) {
      if (!step(std::integral_constant<int, 0>{}, c)) break;
      if (!step(std::integral_constant<int, 1>{}, c)) break;
      if constexpr (NB > 2)
        if (!step(std::integral_constant<int, 2>{}, c)) break;
    }
  }
  for (int j = nc * CH; j < a.nsrc; ++j) xor_masked16<RT, 4>(acc, load16t<1>(a.src[j] + soff, 0), a.mask[j]);
#pragma unroll
  for (int r = 0; r < RT; ++r)
    if (r < a.R) store16t<1>(a.dst[r] + doff, 0, u32x4{acc[r][0], acc[r][1], acc[r][2], acc[r][3]});
}

// Timing probe, wrong output: the production loop with the masked XOR on
// dwords 2-3 replaced by a single unmasked XOR per source, i.e. ~half the
// VALU work for the same loads and stores -- measures how VALU-bound the
// production kernel is.
template <int RT>
__device__ __forceinline__ void xor_masked16_half(uint32_t (&acc)[RT][4], const u32x4& x, uint32_t m) {
#pragma unroll
  for (int r = 0; r < RT; ++r) {
    const uint32_t sel = uint32_t(int32_t(m << (31 - r)) >> 31);
    acc[r][0] = __builtin_amdgcn_bitop3_b32(acc[r][0], x[0], sel, 0x78);
    acc[r][1] = __builtin_amdgcn_bitop3_b32(acc[r][1], x[1], sel, 0x78);
  }
  acc[0][2] ^= x[2];
  acc[0][3] ^= x[3];
  __builtin_amdgcn_sched_barrier(0);
}

template <int RT>
__global__ __launch_bounds__(kBlock) void packets16p_halfvalu(PacketArgs a) {
  const int64_t g = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (g >= a.ncols) return;
  int64_t sp, col;
  packet_coords(a, g, &sp, &col);
  const int64_t soff = sp * a.sstride + col * 16, doff = sp * a.dstride + col * 16;
  uint32_t acc[RT][4];
#pragma unroll
  for (int r = 0; r < RT; ++r) acc[r][0] = acc[r][1] = acc[r][2] = acc[r][3] = 0u;
  const int nc = a.nsrc >> 2;
  u32x4 xa[4], xb[4];
  uint32_t ma[4], mb[4];
  auto load4 = [&](u32x4 (&x)[4], uint32_t (&m)[4], int c) {
    const int b = (c < nc ? c : nc - 1) * 4;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      m[u] = a.mask[b + u];
      x[u] = load16t<1>(a.src[b + u] + soff, 0);
    }
  };
  auto apply4 = [&](const u32x4 (&x)[4], const uint32_t (&m)[4]) {
#pragma unroll
    for (int u = 0; u < 4; ++u) xor_masked16_half<RT>(acc, x[u], m[u]);
  };
  if (nc > 0) {
    load4(xa, ma, 0);
    for (int c = 0; c < nc; c += 2) {
      load4(xb, mb, c + 1);
      apply4(xa, ma);
      if (c + 1 >= nc) break;
      load4(xa, ma, c + 2);
      apply4(xb, mb);
    }
  }
#pragma unroll
  for (int r = 0; r < RT; ++r)
    if (r < a.R) store16t<1>(a.dst[r] + doff, 0, u32x4{acc[r][0], acc[r][1], acc[r][2], acc[r][3]});
}
}  // namespace lab

struct Variant {
  std::string name;
  const void* fn;
  unsigned lds = 0;  // dynamic LDS per workgroup: an unused allocation that caps residency
  int split = 1;     // waves sharing one column block (grid scales by it)
  bool check = true; // false: a timing probe whose output is deliberately wrong
};

int main(int argc, char** argv) {
  int mib = 64, ps = 4096, rounds = 9, reps = 10, skew_kib = -1;
  std::string only;  // --only a,b: time only the variants whose names contain one of these (the first always runs)
  for (int i = 1; i + 1 < argc; i += 2) {
    const std::string f = argv[i];
    if (f == "--only") only = argv[i + 1];
    if (f == "--mib") mib = std::atoi(argv[i + 1]);
    else if (f == "--ps") ps = std::atoi(argv[i + 1]);
    else if (f == "--rounds") rounds = std::atoi(argv[i + 1]);
    else if (f == "--reps") reps = std::atoi(argv[i + 1]);
    else if (f == "--skew-kib") skew_kib = std::atoi(argv[i + 1]);
  }
  const int k = 10, m = 4, w = 8;
  // the library's stride (shard_stride.hpp), or --skew-kib
  const size_t S = size_t(mib) << 20;
  const size_t stride = skew_kib >= 0 ? S + size_t(skew_kib) * 1024 : size_t(shard_stride(int64_t(S)));
  if (S % (size_t(w) * ps) || ps % 16) {
    std::fprintf(stderr, "S must be a multiple of w * ps, ps of 16\n");
    return 2;
  }
  int* M = vandermonde_coding_matrix(k, m, w);
  int* B = matrix_to_bitmatrix(k, m, w, M);  // (m*w) x (k*w)
  const int nsrc = k * w, R = m * w;
  std::vector<uint32_t> mask(size_t(nsrc), 0);
  for (int r = 0; r < R; ++r)
    for (int j = 0; j < nsrc; ++j)
      if (B[r * nsrc + j]) mask[size_t(j)] |= 1u << r;
  uint8_t* slab = nullptr;
  CK(hipMalloc(&slab, stride * size_t(k + m)));
  {
    std::vector<uint8_t> h(S);
    std::mt19937_64 g(7);
    for (int d = 0; d < k; ++d) {
      for (size_t i = 0; i < S; i += 8) {
        const uint64_t x = g();
        std::memcpy(&h[i], &x, 8);
      }
      CK(hipMemcpy(slab + stride * size_t(d), h.data(), S, hipMemcpyHostToDevice));
    }
  }
  std::vector<const uint8_t*> hs(static_cast<size_t>(nsrc));
  std::vector<uint8_t*> hd(static_cast<size_t>(R));
  for (int j = 0; j < nsrc; ++j) hs[size_t(j)] = slab + stride * size_t(j / w) + size_t(j % w) * size_t(ps);
  for (int r = 0; r < R; ++r) hd[size_t(r)] = slab + stride * size_t(k + r / w) + size_t(r % w) * size_t(ps);
  const uint8_t** d_src = nullptr;
  uint8_t** d_dst = nullptr;
  uint32_t* d_mask = nullptr;
  CK(hipMalloc(&d_src, sizeof(void*) * nsrc));
  CK(hipMalloc(&d_dst, sizeof(void*) * R));
  CK(hipMalloc(&d_mask, 4 * nsrc));
  CK(hipMemcpy(d_src, hs.data(), sizeof(void*) * nsrc, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_dst, hd.data(), sizeof(void*) * R, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_mask, mask.data(), 4 * nsrc, hipMemcpyHostToDevice));
  PacketArgs a{};
  a.src = d_src;
  a.dst = d_dst;
  a.mask = d_mask;
  a.sstride = a.dstride = int64_t(w) * ps;
  a.cpp = ps / 16;
  a.ncols = int64_t(S / (size_t(w) * ps)) * a.cpp;
  a.nsrc = nsrc;
  a.R = R;

  std::vector<Variant> vs = {{"prod_packets16p", reinterpret_cast<const void*>(&gf_xor_packets16p<32>)},
                             {"prod_packets16_c8", reinterpret_cast<const void*>(&gf_xor_packets16<32, 8>)}};
  int dev = 0, lds_cu = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&lds_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev));
  vs.push_back({"ring_c4x2", reinterpret_cast<const void*>(&lab::packets16_ring<32, 4, 2>)});
  vs.push_back({"ring_c4x3", reinterpret_cast<const void*>(&lab::packets16_ring<32, 4, 3>)});
  vs.push_back({"ring_c8x2", reinterpret_cast<const void*>(&lab::packets16_ring<32, 8, 2>)});
  vs.push_back({"ring_c8x3", reinterpret_cast<const void*>(&lab::packets16_ring<32, 8, 3>)});
  vs.push_back({"ring_c6x3", reinterpret_cast<const void*>(&lab::packets16_ring<32, 6, 3>)});
  vs.push_back({"prod_unit16u", reinterpret_cast<const void*>(&gf_xor_packets16u<32, 3>)});
  vs.push_back({"unit16u_wpe1", reinterpret_cast<const void*>(&gf_xor_packets16u<32, 1>)});
  vs.push_back({"probe_halfvalu", reinterpret_cast<const void*>(&lab::packets16p_halfvalu<32>), 0, 1, false});
  if (!only.empty()) {  // keep variant 0 (the reference) and the named ones
    std::vector<Variant> keep{vs[0]};
    for (size_t v = 1; v < vs.size(); ++v)
      for (size_t p0 = 0; p0 <= only.size();) {
        const size_t p1 = std::min(only.find(',', p0), only.size());
        if (vs[v].name.find(only.substr(p0, p1 - p0)) != std::string::npos) {
          keep.push_back(vs[v]);
          break;
        }
        p0 = p1 + 1;
      }
    vs = keep;
  }
  (void)lds_cu;
  auto launch = [&](const Variant& v) {
    PacketArgs args = a;
    void* kargs[] = {&args};
    const int64_t per = kBlock / v.split;
    CK(hipLaunchKernel(v.fn, dim3(unsigned((a.ncols + per - 1) / per)), dim3(kBlock), kargs, v.lds, nullptr));
  };
  launch(vs[0]);
  CK(hipDeviceSynchronize());
  std::vector<std::vector<uint8_t>> want(static_cast<size_t>(m), std::vector<uint8_t>(S));
  for (int i = 0; i < m; ++i) CK(hipMemcpy(want[size_t(i)].data(), slab + stride * size_t(k + i), S, hipMemcpyDeviceToHost));
  {
    // host check: super-packet sp, packet row r of coding device i, byte b
    std::mt19937_64 g(3);
    for (int n = 0; n < 500; ++n) {
      const size_t nsp = S / (size_t(w) * ps);
      const size_t sp = g() % nsp, b = g() % size_t(ps);
      std::vector<uint8_t> src(static_cast<size_t>(nsrc));
      for (int j = 0; j < nsrc; ++j)
        CK(hipMemcpy(&src[size_t(j)], hs[size_t(j)] + sp * size_t(w) * ps + b, 1, hipMemcpyDeviceToHost));
      for (int r = 0; r < R; ++r) {
        uint8_t e = 0;
        for (int j = 0; j < nsrc; ++j)
          if ((mask[size_t(j)] >> r) & 1u) e ^= src[size_t(j)];
        if (want[size_t(r / w)][sp * size_t(w) * ps + size_t(r % w) * ps + b] != e) {
          std::fprintf(stderr, "production kernel disagrees with the host (row %d)\n", r);
          return 1;
        }
      }
    }
  }
  for (size_t v = 1; v < vs.size(); ++v) {
    if (!vs[v].check) continue;
    CK(hipMemset(slab + stride * size_t(k), 0, stride * size_t(m)));
    launch(vs[v]);
    CK(hipDeviceSynchronize());
    std::vector<uint8_t> got(S);
    for (int i = 0; i < m; ++i) {
      CK(hipMemcpy(got.data(), slab + stride * size_t(k + i), S, hipMemcpyDeviceToHost));
      if (got != want[size_t(i)]) {
        std::fprintf(stderr, "variant %s differs (coding %d)\n", vs[v].name.c_str(), i);
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
  const double bytes = double(k + m) * double(S);
  for (size_t v = 0; v < vs.size(); ++v) {
    std::sort(t[v].begin(), t[v].end());
    const double med = t[v][t[v].size() / 2];
    std::printf("{\"kernel\": \"%s\", \"shard_mib\": %d, \"packetsize\": %d, \"median_us\": %.1f, \"min_us\": %.1f, "
                "\"GBps\": %.0f, \"samples\": %zu}\n",
                vs[v].name.c_str(), mib, ps, med, double(t[v][0]), bytes / med / 1e3, t[v].size());
  }
  return 0;
}
