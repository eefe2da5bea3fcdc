// diag_kernels_w8.hpp -- measurement-only w = 8 kernel forms, compiled into
// libecgpu_diag.so (diag_kernels.hip) and never into libecgpu.so, so an edit
// here leaves the production kernels' build ID -- and the PMC records keyed to
// it -- unchanged (erasure_coding_test_amd/build.py).  Each was measured
// against the production gf_apply and not kept: the round-1
// 2-bit PERM form with its coefficient-class modes, LDS-DMA loads, an
// occupancy-8 register budget, a persistent streaming form; plus the copy
// kernel behind the bench's copy ceiling.
#pragma once
#include "gf_kernels.hpp"

namespace ecgpu {
namespace dev {

// How a launch treats coefficients 0 and 1.
enum CoefMode : int {
  kClassFromTable = 0,  // test the (s_load'ed) table word: 0 -> skip, unit -> XOR
  kClassFromMask = 1,   // test kernarg bit masks (no load on the branch path)
  kAllPerm = 2,         // no test: every coefficient through v_perm
  kXorOnly = 3,         // DIAGNOSTIC: XOR all sources, ignore coefficients
};

// acc ^= c * v for one 16-byte column; sel = the four 2-bit selector words.
// Tables come from `qt` (global qtab, or the block's LDS copy).
template <int MODE, typename QPtr>
__device__ __forceinline__ void mac16(const ApplyArgs& a, QPtr qt, int idx, const u32x4& v, const u32x4 (&sel)[4],
                                      u32x4& acc) {
  if (MODE == kXorOnly) {
    acc ^= v;
    return;
  }
  if (MODE == kClassFromMask) {
    if ((a.zero_mask >> idx) & 1u) return;
    if ((a.unit_mask >> idx) & 1u) {
      acc ^= v;
      return;
    }
  }
  const u32x4 q = qt[idx];
  if (MODE == kClassFromTable) {
    if (q.x == 0u) return;      // coefficient 0
    if (q.x == kQ0Unit) {       // coefficient 1
      acc ^= v;
      return;
    }
  }
  acc.x ^= gf_mul_perm(q, sel[0].x, sel[1].x, sel[2].x, sel[3].x);
  acc.y ^= gf_mul_perm(q, sel[0].y, sel[1].y, sel[2].y, sel[3].y);
  acc.z ^= gf_mul_perm(q, sel[0].z, sel[1].z, sel[2].z, sel[3].z);
  acc.w ^= gf_mul_perm(q, sel[0].w, sel[1].w, sel[2].w, sel[3].w);
}

// ---------------------------------------------------------------- PERM ----
// Lane l of block b handles 16-byte columns b*VEC*256 + v*256 + l (v < VEC)
// of every shard of stripe blockIdx.y: all K*VEC loads are issued before
// any arithmetic, then R*VEC 16-byte stores.
template <int K, int R, int VEC, int MODE>
__global__ __launch_bounds__(kBlock) void gf_apply_perm(ApplyArgs a) {
  const int64_t col0 = int64_t(blockIdx.x) * (VEC * kBlock) + threadIdx.x;
  if (col0 >= a.nvec) return;
  const int s = blockIdx.y;
  const uint8_t* const* sp = a.src + int64_t(s) * a.src_stride;
  uint8_t* dp[R];  // all pointers before the first store (see gf_apply_body)
#pragma unroll
  for (int r = 0; r < R; ++r) dp[r] = a.dst[int64_t(s) * a.dst_stride + a.row0 + r];

  bool live[VEC];
#pragma unroll
  for (int v = 0; v < VEC; ++v) live[v] = (col0 + v * kBlock) < a.nvec;

  u32x4 x[VEC][K];
  if (a.nt) {
#pragma unroll
    for (int v = 0; v < VEC; ++v)
#pragma unroll
      for (int j = 0; j < K; ++j) x[v][j] = live[v] ? load16(sp[j], col0 + v * kBlock, 1) : u32x4{0u, 0u, 0u, 0u};
  } else {
#pragma unroll
    for (int v = 0; v < VEC; ++v)
#pragma unroll
      for (int j = 0; j < K; ++j) x[v][j] = live[v] ? load16(sp[j], col0 + v * kBlock, 0) : u32x4{0u, 0u, 0u, 0u};
  }

  u32x4 acc[VEC][R];
#pragma unroll
  for (int v = 0; v < VEC; ++v)
#pragma unroll
    for (int r = 0; r < R; ++r) acc[v][r] = u32x4{0u, 0u, 0u, 0u};

#pragma unroll
  for (int j = 0; j < K; ++j) {
#pragma unroll
    for (int v = 0; v < VEC; ++v) {
      const u32x4 xv = x[v][j];
      u32x4 sel[4];
      if (MODE != kXorOnly) {
        sel[0] = xv & kLo2;
        sel[1] = (xv >> 2) & kLo2;
        sel[2] = (xv >> 4) & kLo2;
        sel[3] = (xv >> 6) & kLo2;
      }
#pragma unroll
      for (int r = 0; r < R; ++r) mac16<MODE>(a, a.qtab, r * K + j, xv, sel, acc[v][r]);
    }
  }

  if (a.nt) {
#pragma unroll
    for (int v = 0; v < VEC; ++v)
      if (live[v])
#pragma unroll
        for (int r = 0; r < R; ++r) store16(dp[r], col0 + v * kBlock, acc[v][r], 1);
  } else {
#pragma unroll
    for (int v = 0; v < VEC; ++v)
      if (live[v])
#pragma unroll
        for (int r = 0; r < R; ++r) store16(dp[r], col0 + v * kBlock, acc[v][r], 0);
  }
}

// LDS-DMA form: the K source columns of a lane arrive by
// global_load_lds_dwordx4 (one 1 KiB piece per wave-instruction, written to
// LDS at wave base + lane*16, no VGPR destination) instead of register
// loads; the lane reads back only its own 16 B, so no barrier is needed,
// just the wait on the VM counter.  K KiB of LDS per wave.
template <int K, int R, int UNITS, int SLICES = 3, int NT = 3>
__global__ __launch_bounds__(kBlock) void gf_apply_dma(ApplyArgs a) {
  __shared__ __attribute__((aligned(16))) u32x4 stage[kBlock / 64][K][64];
  const int s = blockIdx.y;
  const int64_t col = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (col >= a.nvec) return;
  const int w = __builtin_amdgcn_readfirstlane(int(threadIdx.x) >> 6);
  const int lane = threadIdx.x & 63;
  const uint8_t* const* sp = a.src + int64_t(s) * a.src_stride;
  // all pointers first (scalar loads), then the DMA issue
  const uint8_t* src[K];
#pragma unroll
  for (int j = 0; j < K; ++j) src[j] = sp[j];
  uint8_t* dp[R];
#pragma unroll
  for (int r = 0; r < R; ++r) dp[r] = a.dst[int64_t(s) * a.dst_stride + a.row0 + r];
#pragma unroll
  for (int j = 0; j < K; ++j)
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src[j] + col * 16),
                                     (__attribute__((address_space(3))) void*)&stage[w][j][0], 16, 0,
                                     (NT & 1) ? 2 : 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  u32x4 x[K];
#pragma unroll
  for (int j = 0; j < K; ++j) x[j] = stage[w][j][lane];
  combine_store<K, R, UNITS, SLICES, (NT >> 1)>(a, x, dp, col);
}

// Same body, register budget capped for 8 waves/SIMD (<= 64 VGPRs).
template <int K, int R, int UNITS>
__global__ __launch_bounds__(kBlock, 8) void gf_apply_occ8(ApplyArgs a) {
  gf_apply_body<K, R, UNITS, 1>(a);
}

// ------------------------------------------------------ PERM, streaming ----
// Persistent-per-stripe form: gridDim.x blocks share one stripe, block b
// walks a CONTIGUOUS run of columns [b*chunk, (b+1)*chunk) 256 columns at a
// time, and the K loads of step i+1 are issued before step i is computed and
// stored (register double buffer), so every wave keeps K*16 B per lane in
// flight while it computes.  Each shard is then read as gridDim.x long
// sequential streams instead of interleaved 4 KiB pieces.
template <int K, int R, int MODE>
__global__ __launch_bounds__(kBlock) void gf_apply_perm_stream(ApplyArgs a) {
  __shared__ u32x4 lq[R * K];
  for (int i = threadIdx.x; i < R * K; i += kBlock) lq[i] = a.qtab[i];
  __syncthreads();
  const int s = blockIdx.y;
  const int64_t steps_total = (a.nvec + kBlock - 1) / kBlock;
  const int64_t steps_per_block = (steps_total + gridDim.x - 1) / gridDim.x;
  const int64_t step0 = int64_t(blockIdx.x) * steps_per_block;
  const int64_t step_end = step0 + steps_per_block < steps_total ? step0 + steps_per_block : steps_total;
  if (step0 >= step_end) return;
  const uint8_t* const* sp = a.src + int64_t(s) * a.src_stride;
  uint8_t* dp[R];  // all pointers before the first store (see gf_apply_body)
#pragma unroll
  for (int r = 0; r < R; ++r) dp[r] = a.dst[int64_t(s) * a.dst_stride + a.row0 + r];
  const uint8_t* src[K];
#pragma unroll
  for (int j = 0; j < K; ++j) src[j] = sp[j];

  u32x4 cur[K], nxt[K];
  int64_t col = step0 * kBlock + threadIdx.x;
#pragma unroll
  for (int j = 0; j < K; ++j) cur[j] = col < a.nvec ? load16(src[j], col, a.nt) : u32x4{0u, 0u, 0u, 0u};
  for (int64_t step = step0; step < step_end; ++step) {
    const int64_t ncol = col + kBlock;
    const bool more = step + 1 < step_end;
    if (more) {
#pragma unroll
      for (int j = 0; j < K; ++j) nxt[j] = ncol < a.nvec ? load16(src[j], ncol, a.nt) : u32x4{0u, 0u, 0u, 0u};
    }
    u32x4 acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = u32x4{0u, 0u, 0u, 0u};
    // Re-read the tables from LDS every step (uniform address: broadcast
    // ds_read_b128).  Hoisted out of the loop they would be parked in
    // R*K*4 VGPRs and cut occupancy to 2 waves/SIMD.
    lds_u32x4* qt = (lds_u32x4*)lq;
    asm volatile("" : "+v"(qt));
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const u32x4 xv = cur[j];
      u32x4 sel[4];
      if (MODE != kXorOnly) {
        sel[0] = xv & kLo2;
        sel[1] = (xv >> 2) & kLo2;
        sel[2] = (xv >> 4) & kLo2;
        sel[3] = (xv >> 6) & kLo2;
      }
#pragma unroll
      for (int r = 0; r < R; ++r) mac16<MODE>(a, qt, r * K + j, xv, sel, acc[r]);
    }
    if (col < a.nvec) {
#pragma unroll
      for (int r = 0; r < R; ++r) store16(dp[r], col, acc[r], a.nt);
    }
    if (more) {
#pragma unroll
      for (int j = 0; j < K; ++j) cur[j] = nxt[j];
    }
    col = ncol;
  }
}

// DIAGNOSTIC: streaming copy of shard 0 -> dst 0 (the HBM ceiling reference).
// NT: bit 0 = non-temporal loads, NT >> 1 = store policy (store16t).
template <int VEC, int NT = 1>
__global__ __launch_bounds__(kBlock) void diag_copy(ApplyArgs a) {
  const int64_t col0 = int64_t(blockIdx.x) * (VEC * kBlock) + threadIdx.x;
  const int s = blockIdx.y;
  const uint8_t* sp = a.src[int64_t(s) * a.src_stride];
  uint8_t* dp = a.dst[int64_t(s) * a.dst_stride];
  u32x4 x[VEC];
#pragma unroll
  for (int v = 0; v < VEC; ++v)
    if (col0 + v * kBlock < a.nvec) x[v] = load16t<NT & 1>(sp, col0 + v * kBlock);
#pragma unroll
  for (int v = 0; v < VEC; ++v)
    if (col0 + v * kBlock < a.nvec) store16t<(NT >> 1)>(dp, col0 + v * kBlock, x[v]);
}

}  // namespace dev
}  // namespace ecgpu
