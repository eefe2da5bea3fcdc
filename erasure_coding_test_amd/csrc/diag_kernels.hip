// diag_kernels.hip -- TUNING/DIAGNOSTIC library (libecgpu_diag.so), not the
// product.  Instantiates variants of the production kernel (gf_kernels.hpp)
// so they can be A/B-timed in one process on the MI355X:
//   variant 0: gf_apply_perm<K, R, VEC, MODE> for (K,R) in {(10,4), (10,1)},
//              VEC in {1, 2, 4}, MODE in {table, mask, all-perm, xor-only}
//   variant 1: diag_copy<VEC> -- 1 read + 1 write stream, the HBM reference
//   variant 2: gf_apply_lds<K, R> (north-star LDS nibble tables)
//   variant 11 / 12: read-only probes (K register loads / K LDS-DMA loads per
//              lane, nothing written)
//   variant 13 / 14: production combine, register / LDS-DMA loads, explicit
//              nt bits (loads / stores)
//   variant 15: production combine with inline-asm loads / stores carrying
//              explicit sc0 / sc1 / nt cache bits (cache-policy probe)
//   variant 10: production gf_apply with the round-1 2-bit-slice tables
//              (A/B against variants 4/8, which use the 3-bit-slice ptab)
//   variant 16: diag_xor_mix<K, R> -- the coding launches' exact streams (K
//              nt loads and R nt stores of 16 B per lane, one column per
//              lane, production grid) with no arithmetic beyond one XOR: a
//              reference point for the coding kernels' streams, not a bound
//              (bench.py `xor_stream_probe`)
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "diag_kernels_w8.hpp"

using ecgpu::dev::ApplyArgs;
using ecgpu::dev::u32x4;
using KernelFn = void (*)(ApplyArgs);

namespace {

// ---- read-only probes (variants 11 / 12): how fast can K shard streams be
// READ with this layout, with no write stream?  The XOR of the K columns is
// stored only if it equals a 128-bit constant (never, on random data), so
// the loads stay live and no bytes are written.
__device__ __forceinline__ void sink(const ApplyArgs& a, int s, int64_t col, const u32x4& acc) {
  if (acc.x == 0x9E3779B9u && acc.y == 0x7F4A7C15u && acc.z == 0x85EBCA6Bu && acc.w == 0xC2B2AE35u)
    ecgpu::dev::store16(a.dst[int64_t(s) * a.dst_stride], col, acc, 1);
}

// ---- access-mix ceiling (variant 16): every lane loads its 16-B column of
// the K sources (non-temporal, all issued before use, like gf_apply), folds
// them with XOR and stores the result to the R outputs (non-temporal).
template <int K, int R>
__global__ __launch_bounds__(256) void diag_xor_mix(ApplyArgs a) {
  const int64_t col = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (col >= a.nvec) return;
  const int s = blockIdx.y;
  const uint8_t* const* sp = a.src + int64_t(s) * a.src_stride;
  uint8_t* dp[R];  // every pointer before the first store
#pragma unroll
  for (int r = 0; r < R; ++r) dp[r] = a.dst[int64_t(s) * a.dst_stride + r];
  u32x4 x[K];
#pragma unroll
  for (int j = 0; j < K; ++j) x[j] = ecgpu::dev::load16t<1>(sp[j], col);
  u32x4 acc = x[0];
#pragma unroll
  for (int j = 1; j < K; ++j) acc ^= x[j];
#pragma unroll
  for (int r = 0; r < R; ++r) ecgpu::dev::store16t<1>(dp[r], col, acc);
}

// ---- cache-policy probe (variant 15): the production combine with loads
// and stores issued by inline asm carrying explicit gfx950 cache bits
// (sc0 / sc1 / nt), beyond what __builtin_nontemporal_* can express.
// Loads: 0 "nt", 1 "sc1 nt", 2 "sc0 sc1 nt", 3 "sc0 sc1", 4 "sc1".
// Stores: 0 "nt", 1 "sc1", 2 "sc0 sc1", 3 "sc0 sc1 nt", 4 "sc1 nt".
template <int LP>
__device__ __forceinline__ u32x4 asm_load16(const uint8_t* p) {
  u32x4 v;
  if constexpr (LP == 0) asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(v) : "v"(p) : "memory");
  if constexpr (LP == 1) asm volatile("global_load_dwordx4 %0, %1, off sc1 nt" : "=v"(v) : "v"(p) : "memory");
  if constexpr (LP == 2) asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1 nt" : "=v"(v) : "v"(p) : "memory");
  if constexpr (LP == 3) asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1" : "=v"(v) : "v"(p) : "memory");
  if constexpr (LP == 4) asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(v) : "v"(p) : "memory");
  return v;
}

// Each store is followed by s_nop 1: a VALU write to the data VGPRs of an
// in-flight store wider than 8 bytes needs wait states, which the compiler's
// hazard recognizer inserts for its own stores but not after inline asm
// (without them the next VALU op corrupted the stored data).
template <int SP>
__device__ __forceinline__ void asm_store16(uint8_t* p, const u32x4& v) {
  if constexpr (SP == 0) asm volatile("global_store_dwordx4 %0, %1, off nt\n\ts_nop 1" : : "v"(p), "v"(v) : "memory");
  if constexpr (SP == 1) asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" : : "v"(p), "v"(v) : "memory");
  if constexpr (SP == 2) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" : : "v"(p), "v"(v) : "memory");
  if constexpr (SP == 3) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt\n\ts_nop 1" : : "v"(p), "v"(v) : "memory");
  if constexpr (SP == 4) asm volatile("global_store_dwordx4 %0, %1, off sc1 nt\n\ts_nop 1" : : "v"(p), "v"(v) : "memory");
}

template <int K, int R, int UNITS, int LP, int SP>
__global__ __launch_bounds__(256) void gf_apply_pol(ApplyArgs a) {
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
  for (int j = 0; j < K; ++j) x[j] = asm_load16<LP>(src[j] + col * 16);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int j = 0; j < K; ++j) asm volatile("" : "+v"(x[j]));  // uses stay after the wait
  u32x4 acc[R];
  ecgpu::dev::combine<K, R, UNITS, 3>(a, x, acc);
#pragma unroll
  for (int r = 0; r < R; ++r) asm_store16<SP>(dp[r] + col * 16, acc[r]);
}

template <int K, int R, int U, int LP>
KernelFn pick_sp(int sp) {
  switch (sp) {
    case 0: return &gf_apply_pol<K, R, U, LP, 0>;
    case 1: return &gf_apply_pol<K, R, U, LP, 1>;
    case 2: return &gf_apply_pol<K, R, U, LP, 2>;
    case 3: return &gf_apply_pol<K, R, U, LP, 3>;
    default: return &gf_apply_pol<K, R, U, LP, 4>;
  }
}

template <int K, int R, int U>
KernelFn pick_pol(int lp, int sp) {
  switch (lp) {
    case 0: return pick_sp<K, R, U, 0>(sp);
    case 1: return pick_sp<K, R, U, 1>(sp);
    case 2: return pick_sp<K, R, U, 2>(sp);
    case 3: return pick_sp<K, R, U, 3>(sp);
    default: return pick_sp<K, R, U, 4>(sp);
  }
}

// K register loads per lane (the production kernel's load phase).
template <int K, int NT>
__global__ __launch_bounds__(256) void diag_read_regs(ApplyArgs a) {
  const int64_t col = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (col >= a.nvec) return;
  const int s = blockIdx.y;
  const uint8_t* const* sp = a.src + int64_t(s) * a.src_stride;
  u32x4 x[K];
#pragma unroll
  for (int j = 0; j < K; ++j) x[j] = ecgpu::dev::load16t<NT>(sp[j], col);
  u32x4 acc = x[0];
#pragma unroll
  for (int j = 1; j < K; ++j) acc ^= x[j];
  sink(a, s, col, acc);
}

// Same bytes through LDS-DMA (global_load_lds_dwordx4, nt): each wave
// instruction lands 1 KiB in LDS with no VGPR destination.
template <int K, int NT>
__global__ __launch_bounds__(256) void diag_read_glds(ApplyArgs a) {
  __shared__ __attribute__((aligned(16))) u32x4 buf[4][K][64];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t col = int64_t(blockIdx.x) * 256 + threadIdx.x;  // nvec % 256 == 0 in the probe
  const int s = blockIdx.y;
  const uint8_t* const* sp = a.src + int64_t(s) * a.src_stride;
#pragma unroll
  for (int j = 0; j < K; ++j)
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(sp[j] + col * 16),
                                     (__attribute__((address_space(3))) void*)&buf[w][j][0], 16, 0, NT ? 2 : 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  u32x4 acc = buf[w][0][lane];
#pragma unroll
  for (int j = 1; j < K; ++j) acc ^= buf[w][j][lane];
  sink(a, s, col, acc);
}

template <int K, int R, int V>
KernelFn pick_mode(int mode) {
  switch (mode) {
    case 0: return &ecgpu::dev::gf_apply_perm<K, R, V, 0>;
    case 1: return &ecgpu::dev::gf_apply_perm<K, R, V, 1>;
    case 2: return &ecgpu::dev::gf_apply_perm<K, R, V, 2>;
    default: return &ecgpu::dev::gf_apply_perm<K, R, V, 3>;
  }
}
template <int K, int R>
KernelFn pick_vec(int vec, int mode) {
  switch (vec) {
    case 1: return pick_mode<K, R, 1>(mode);
    case 2: return pick_mode<K, R, 2>(mode);
    default: return pick_mode<K, R, 4>(mode);
  }
}
}  // namespace

extern "C" __attribute__((visibility("default"))) int ecgpu_diag_launch(
    int variant, int K, int R, int vec, int mode, const void* qtab, const void* ntab, const void* src_tab,
    void* dst_tab, int stripes, long long size, unsigned long long unit_mask, unsigned long long zero_mask, int nt,
    void* stream, const void* ptab) {
  KernelFn fn = nullptr;
  if (variant == 0) {
    if (K == 10 && R == 4) fn = pick_vec<10, 4>(vec, mode);
    if (K == 10 && R == 1) fn = pick_vec<10, 1>(vec, mode);
  } else if (variant == 1) {
    // mode = NT bits (bit 0 loads, bit 1 stores); vec in {1, 2, 4}
    using ecgpu::dev::diag_copy;
    KernelFn c1[4] = {&diag_copy<1, 0>, &diag_copy<1, 1>, &diag_copy<1, 2>, &diag_copy<1, 3>};
    KernelFn c2[4] = {&diag_copy<2, 0>, &diag_copy<2, 1>, &diag_copy<2, 2>, &diag_copy<2, 3>};
    KernelFn c4[4] = {&diag_copy<4, 0>, &diag_copy<4, 1>, &diag_copy<4, 2>, &diag_copy<4, 3>};
    fn = (vec == 1 ? c1 : vec == 2 ? c2 : c4)[mode & 3];
  } else if (variant == 3) {
    // persistent streaming form; `vec` = blocks per stripe
    if (K == 10 && R == 4) fn = mode == 3 ? &ecgpu::dev::gf_apply_perm_stream<10, 4, 3>
                                          : &ecgpu::dev::gf_apply_perm_stream<10, 4, 2>;
    if (K == 10 && R == 1) fn = mode == 3 ? &ecgpu::dev::gf_apply_perm_stream<10, 1, 3>
                                          : &ecgpu::dev::gf_apply_perm_stream<10, 1, 2>;
  } else if (variant == 4 || variant == 5) {
    // production gf_apply; `mode` = UnitMask
    vec = 1;
    if (K == 10 && R == 4)
      fn = mode == 0 ? &ecgpu::dev::gf_apply<10, 4, 0> : mode == 1 ? &ecgpu::dev::gf_apply<10, 4, 1>
                                                        : &ecgpu::dev::gf_apply<10, 4, 3>;
    if (K == 10 && R == 1)
      fn = mode == 4 ? &ecgpu::dev::gf_apply<10, 1, 4> : &ecgpu::dev::gf_apply<10, 1, 0>;
  } else if (variant == 6) {
    vec = 1;
    if (K == 10 && R == 4) fn = &ecgpu::dev::gf_apply_occ8<10, 4, 3>;
    if (K == 10 && R == 1) fn = mode == 4 ? &ecgpu::dev::gf_apply_occ8<10, 1, 4> : &ecgpu::dev::gf_apply_occ8<10, 1, 0>;
  } else if (variant == 7) {
    // production body; vec bit0 = stripe-fastest order, bit1 = 8-wave register cap; mode = UnitMask
    const bool occ8 = (vec & 2) != 0;
    if (K == 10 && R == 4)
      fn = occ8 ? &ecgpu::dev::gf_apply_occ8<10, 4, 3> : &ecgpu::dev::gf_apply<10, 4, 3>;
    if (K == 10 && R == 1)
      fn = mode == 4 ? (occ8 ? &ecgpu::dev::gf_apply_occ8<10, 1, 4> : &ecgpu::dev::gf_apply<10, 1, 4>)
                     : (occ8 ? &ecgpu::dev::gf_apply_occ8<10, 1, 0> : &ecgpu::dev::gf_apply<10, 1, 0>);
  } else if (variant == 8) {
    // production gf_apply with VEC columns per lane (vec in {1,2,4}); mode = UnitMask
    if (K == 10 && R == 4)
      fn = vec == 1 ? &ecgpu::dev::gf_apply<10, 4, 3, 1>
                    : vec == 2 ? &ecgpu::dev::gf_apply<10, 4, 3, 2> : &ecgpu::dev::gf_apply<10, 4, 3, 4>;
    if (K == 10 && R == 1)
      fn = vec == 1 ? &ecgpu::dev::gf_apply<10, 1, 4, 1>
                    : vec == 2 ? &ecgpu::dev::gf_apply<10, 1, 4, 2> : &ecgpu::dev::gf_apply<10, 1, 4, 4>;
  } else if (variant == 9) {
    // access-pattern probe: XOR-only gf_apply_perm over (K, R) shapes
    vec = 1;
    if (K == 1 && R == 1) fn = &ecgpu::dev::gf_apply_perm<1, 1, 1, 3>;
    if (K == 2 && R == 2) fn = &ecgpu::dev::gf_apply_perm<2, 2, 1, 3>;
    if (K == 4 && R == 4) fn = &ecgpu::dev::gf_apply_perm<4, 4, 1, 3>;
    if (K == 7 && R == 7) fn = &ecgpu::dev::gf_apply_perm<7, 7, 1, 3>;
    if (K == 10 && R == 4) fn = &ecgpu::dev::gf_apply_perm<10, 4, 1, 3>;
    if (K == 10 && R == 1) fn = &ecgpu::dev::gf_apply_perm<10, 1, 1, 3>;
    if (K == 13 && R == 1) fn = &ecgpu::dev::gf_apply_perm<13, 1, 1, 3>;
    if (K == 4 && R == 1) fn = &ecgpu::dev::gf_apply_perm<4, 1, 1, 3>;
    if (K == 1 && R == 4) fn = &ecgpu::dev::gf_apply_perm<1, 4, 1, 3>;
    if (K == 2 && R == 1) fn = &ecgpu::dev::gf_apply_perm<2, 1, 1, 3>;
  } else if (variant == 10) {
    vec = 1;
    if (K == 10 && R == 4) fn = &ecgpu::dev::gf_apply<10, 4, 3, 1, 2>;
    if (K == 10 && R == 1) fn = mode == 4 ? &ecgpu::dev::gf_apply<10, 1, 4, 1, 2> : &ecgpu::dev::gf_apply<10, 1, 0, 1, 2>;
  } else if (variant == 11) {
    vec = 1;
    if (K == 1) fn = nt ? &diag_read_regs<1, 1> : &diag_read_regs<1, 0>;
    if (K == 4) fn = nt ? &diag_read_regs<4, 1> : &diag_read_regs<4, 0>;
    if (K == 10) fn = nt ? &diag_read_regs<10, 1> : &diag_read_regs<10, 0>;
    if (K == 14) fn = nt ? &diag_read_regs<14, 1> : &diag_read_regs<14, 0>;
  } else if (variant == 13 || variant == 14) {
    // production combine with an explicit cache policy: `vec` = NT bits
    // (bit 0 loads, bit 1 stores); 13 = register loads, 14 = LDS-DMA loads
    using namespace ecgpu::dev;
    const int ntb = vec;
    vec = 1;
#define ECGPU_PICK(KK, RR, UU)                                                                              \
  (variant == 13 ? (ntb == 0 ? &gf_apply<KK, RR, UU, 1, 3, 0> : ntb == 1 ? &gf_apply<KK, RR, UU, 1, 3, 1>   \
                    : ntb == 2 ? &gf_apply<KK, RR, UU, 1, 3, 2> : &gf_apply<KK, RR, UU, 1, 3, 3>)           \
                 : (ntb == 0 ? &gf_apply_dma<KK, RR, UU, 3, 0> : ntb == 1 ? &gf_apply_dma<KK, RR, UU, 3, 1> \
                    : ntb == 2 ? &gf_apply_dma<KK, RR, UU, 3, 2> : &gf_apply_dma<KK, RR, UU, 3, 3>))
    if (K == 10 && R == 4) fn = mode == 0 ? ECGPU_PICK(10, 4, 0) : ECGPU_PICK(10, 4, 3);
    if (K == 10 && R == 1) fn = mode == 4 ? ECGPU_PICK(10, 1, 4) : ECGPU_PICK(10, 1, 0);
    if (K == 6 && R == 3) fn = ECGPU_PICK(6, 3, 3);
#undef ECGPU_PICK
  } else if (variant == 12) {
    vec = 1;
    if (K == 1) fn = nt ? &diag_read_glds<1, 1> : &diag_read_glds<1, 0>;
    if (K == 4) fn = nt ? &diag_read_glds<4, 1> : &diag_read_glds<4, 0>;
    if (K == 10) fn = nt ? &diag_read_glds<10, 1> : &diag_read_glds<10, 0>;
    if (K == 14) fn = nt ? &diag_read_glds<14, 1> : &diag_read_glds<14, 0>;
  } else if (variant == 15) {
    // cache-policy probe: vec = load policy, mode = store policy (gf_apply_pol)
    const int lp = vec;
    vec = 1;
    if (K == 10 && R == 4) fn = pick_pol<10, 4, 3>(lp, mode);
    if (K == 10 && R == 1) fn = pick_pol<10, 1, 4>(lp, mode);
  } else if (variant == 16) {
    vec = 1;
    if (K == 10 && R == 4) fn = &diag_xor_mix<10, 4>;
    if (K == 10 && R == 1) fn = &diag_xor_mix<10, 1>;
    if (K == 6 && R == 3) fn = &diag_xor_mix<6, 3>;
    if (K == 12 && R == 4) fn = &diag_xor_mix<12, 4>;
    if (K == 4 && R == 2) fn = &diag_xor_mix<4, 2>;
  } else if (variant == 2) {
    vec = 1;
    if (K == 10 && R == 4) fn = &ecgpu::dev::gf_apply_lds<10, 4>;
    if (K == 10 && R == 1) fn = &ecgpu::dev::gf_apply_lds<10, 1>;
  }
  if (!fn) return -2;
  ApplyArgs a{};
  a.qtab = static_cast<const ecgpu::dev::u32x4*>(qtab);
  a.ntab = static_cast<const uint8_t*>(ntab);
  a.ptab = static_cast<const uint32_t*>(ptab);
  a.src = static_cast<const uint8_t* const*>(src_tab);
  a.dst = static_cast<uint8_t* const*>(dst_tab);
  a.nvec = size / 16;
  a.size = size;
  a.byte0 = a.nvec * 16;
  a.unit_mask = unit_mask;
  a.zero_mask = zero_mask;
  a.src_stride = variant == 1 ? 1 : K;
  a.dst_stride = variant == 1 ? 1 : R;
  a.row0 = 0;
  a.K = K;
  a.R = R;
  a.nt = nt;
  const long long per_block = 256LL * (variant == 0 || variant == 1 || variant == 8 ? vec : 1);
  dim3 grid(unsigned((a.nvec + per_block - 1) / per_block), unsigned(stripes));
  if (variant == 3) grid = dim3(unsigned(vec), unsigned(stripes));
  if (variant == 7) {
    a.stripe_fast = vec & 1;
    grid = a.stripe_fast ? dim3(unsigned(stripes), unsigned((a.nvec + 255) / 256))
                         : dim3(unsigned((a.nvec + 255) / 256), unsigned(stripes));
  }
  if (variant == 5) {  // stripe-fastest block order
    a.stripe_fast = 1;
    grid = dim3(unsigned(stripes), unsigned((a.nvec + 255) / 256));
  }
  void* args[] = {&a};
  // ECGPU_DIAG_LDS: dynamic LDS bytes per block, unused by the kernels -- caps
  // resident blocks per CU at 160 KiB / bytes (occupancy experiments).
  const char* lds_env = std::getenv("ECGPU_DIAG_LDS");
  const unsigned lds = lds_env ? unsigned(std::atoi(lds_env)) : 0u;
  return hipLaunchKernel(reinterpret_cast<const void*>(fn), grid, dim3(256), args, lds,
                         static_cast<hipStream_t>(stream)) == hipSuccess ? 0 : -3;
}
