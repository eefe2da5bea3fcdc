// gf_kernels_packets.hpp -- GF(2) bit-matrix / schedule coding over packet rows
// (jerasure_bitmatrix_* / jerasure_schedule_*).  Included through gf_kernels.hpp.
#pragma once
#include "gf_kernels_w8.hpp"

namespace ecgpu {
namespace dev {

// ------------------------------------------- GF(2) packet coding ----
// Bit-matrix and XOR-schedule coding (jerasure.cpp:301-345, :1153-1192): a
// device is w packets of `packetsize` bytes per super-packet, and every
// output packet row is the XOR of a set of source packet rows (the host
// replays the reference's memcpy / XOR sequence symbolically, so aliasing
// and schedules that reuse earlier outputs fold into one map).  A "packet
// view" is base + sp * stride + [0, packetsize) for super-packet sp.  Lane g
// handles 8 bytes of one packet column; output rows <= RT per launch, the
// row set of source j is the wave-uniform bit mask mask[j], applied as
// acc ^= x & sext(bit) (one SALU bit extract + one v_bitop3 per term).
struct PacketArgs {
  const uint8_t* const* src;  // [nsrc] packet-view bases
  uint8_t* const* dst;        // [R] packet-view bases
  const uint32_t* mask;       // [nsrc] bit r: source feeds output row r
  int64_t sstride, dstride;   // bytes between super-packets (sources / outputs)
  int64_t cpp;                // 8-byte columns per packet (words kernel) or bytes per packet (bytes kernel)
  int64_t ncols;              // super-packets * cpp
  int nsrc, R;
};


__device__ __forceinline__ void packet_coords(const PacketArgs& a, int64_t g, int64_t* sp, int64_t* col) {
  if (a.ncols <= 0xFFFFFFFFll) {  // 32-bit division unless the launch is huge
    const uint32_t q = uint32_t(g) / uint32_t(a.cpp);
    *sp = q;
    *col = int64_t(uint32_t(g) - q * uint32_t(a.cpp));
  } else {
    *sp = g / a.cpp;
    *col = g - *sp * a.cpp;
  }
}

template <int RT>
__device__ __forceinline__ void xor_masked(uint32_t (&acc)[RT][2], const u32x2& x, uint32_t m) {
  // Row selectors as wave-uniform SALU values.  (Extracting them in VGPRs
  // with v_bfe_i32 avoids the compiler's SGPR spills to VGPR lanes but was
  // slower: 269 vs 240 us per 64 MiB RS(10,4) bit-matrix encode.)
#pragma unroll
  for (int r = 0; r < RT; ++r) {
    const uint32_t sel = uint32_t(int32_t(m << (31 - r)) >> 31);  // 0 or ~0, wave-uniform (SALU)
    acc[r][0] = __builtin_amdgcn_bitop3_b32(acc[r][0], x.x, sel, 0x78);  // a ^ (b & c): 0xF0 ^ (0xCC & 0xAA)
    acc[r][1] = __builtin_amdgcn_bitop3_b32(acc[r][1], x.y, sel, 0x78);
  }
  // keep each source's row selectors local: hoisted over several sources they
  // exceed the SGPR file and spill to VGPR lanes (v_writelane / v_readlane,
  // VALU work as large as the XORs themselves at RT = 32)
  __builtin_amdgcn_sched_barrier(0);
}

template <int RT>
__global__ __launch_bounds__(kBlock) void gf_xor_packets(PacketArgs a) {
  const int64_t g = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (g >= a.ncols) return;
  int64_t sp, col;
  packet_coords(a, g, &sp, &col);
  const int64_t soff = sp * a.sstride + col * 8, doff = sp * a.dstride + col * 8;
  uint8_t* dp[RT];
#pragma unroll
  for (int r = 0; r < RT; ++r) dp[r] = r < a.R ? a.dst[r] : nullptr;
  uint32_t acc[RT][2];
#pragma unroll
  for (int r = 0; r < RT; ++r) acc[r][0] = acc[r][1] = 0u;
  int j = 0;
  for (; j + 4 <= a.nsrc; j += 4) {  // four loads in flight before the first use
    u32x2 x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) x[u] = *(const gu32x2*)(a.src[j + u] + soff);
#pragma unroll
    for (int u = 0; u < 4; ++u) xor_masked<RT>(acc, x[u], a.mask[j + u]);
  }
  for (; j < a.nsrc; ++j) {
    const u32x2 x = *(const gu32x2*)(a.src[j] + soff);
    xor_masked<RT>(acc, x, a.mask[j]);
  }
#pragma unroll
  for (int r = 0; r < RT; ++r)
    if (r < a.R) *(gu32x2*)(dp[r] + doff) = u32x2{acc[r][0], acc[r][1]};
}

// 16-byte form (packet sizes, strides and bases 16-B aligned): lane g owns
// 16 bytes of one packet column, so every SALU row-mask extract serves four
// dwords instead of two and a wave moves 1 KiB per load; CHUNK source rows
// are loaded before the first use.  Non-temporal loads and stores, as the
// matrix kernels.
template <int RT, int CHUNK>
__device__ __forceinline__ void xor_masked16(uint32_t (&acc)[RT][4], const u32x4& x, uint32_t m) {
#pragma unroll
  for (int r = 0; r < RT; ++r) {
    const uint32_t sel = uint32_t(int32_t(m << (31 - r)) >> 31);  // 0 or ~0, wave-uniform (SALU)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[r][c] = __builtin_amdgcn_bitop3_b32(acc[r][c], x[c], sel, 0x78);
  }
  __builtin_amdgcn_sched_barrier(0);  // selectors stay per source (see xor_masked)
}

template <int RT, int CHUNK>
__global__ __launch_bounds__(kBlock) void gf_xor_packets16(PacketArgs a) {
  const int64_t g = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (g >= a.ncols) return;
  int64_t sp, col;
  packet_coords(a, g, &sp, &col);
  const int64_t soff = sp * a.sstride + col * 16, doff = sp * a.dstride + col * 16;
  uint32_t acc[RT][4];
#pragma unroll
  for (int r = 0; r < RT; ++r) acc[r][0] = acc[r][1] = acc[r][2] = acc[r][3] = 0u;
  int j = 0;
  for (; j + CHUNK <= a.nsrc; j += CHUNK) {
    u32x4 x[CHUNK];
#pragma unroll
    for (int u = 0; u < CHUNK; ++u) x[u] = load16t<1>(a.src[j + u] + soff, 0);
#pragma unroll
    for (int u = 0; u < CHUNK; ++u) xor_masked16<RT, CHUNK>(acc, x[u], a.mask[j + u]);
  }
  for (; j < a.nsrc; ++j) xor_masked16<RT, CHUNK>(acc, load16t<1>(a.src[j] + soff, 0), a.mask[j]);
  // output pointers only now: held across the loop they would take RT SGPR
  // pairs from the row selectors (no store precedes these scalar loads)
#pragma unroll
  for (int r = 0; r < RT; ++r)
    if (r < a.R) store16t<1>(a.dst[r] + doff, 0, u32x4{acc[r][0], acc[r][1], acc[r][2], acc[r][3]});
}

// Production 16-B form (packets, strides and bases 16-B aligned): source
// rows in chunks of four, double-buffered -- chunk c + 1's loads (and its
// four row masks) are issued before chunk c is applied, so a wave always has
// four 1 KiB loads in flight while it XORs (RS(10,4) w = 8 64 MiB bit-matrix
// encode 187 -> 180.5 us against gf_xor_packets16's load-eight-then-apply).
// Loads past the last full chunk re-read that chunk (clamped index, no
// branch) so the wait counts stay the same on every path.
template <int RT>
__global__ __launch_bounds__(kBlock) void gf_xor_packets16p(PacketArgs a) {
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

// Unit form of the 16-B kernel for the map of every w = 8 Vandermonde
// bit-matrix encode (jerasure_matrix_to_bitmatrix of reed_sol's matrix,
// whose row 0 and column 0 are all ones, reed_sol.cpp:324-349): 32 output
// rows (4 coding devices x 8), sources device-major (j = 8 * device + bit),
// and the identity blocks of coefficient 1 -- output row b of coding device 0
// is fed by bit b of every data device, and data device 0's bit b feeds row b
// of every coding device -- checked exactly on the masks by the host per
// launch (packets.hip unit_packet_map).  Those terms become plain XORs into a
// compile-time row: 4 VALU per source row instead of 32 for rows 0..7, and 16
// instead of 128 for device 0's rows (RS(10,4): 7,328 instead of 10,240 VALU
// per lane; the 32-row kernel is VALU-bound, profiles/r04_pmc_packets.json).
// A chunk of four source rows holds bits 0..3 (even chunks) or 4..7 (odd),
// so the double-buffered loop keeps every bit compile-time.
// Data device 0's four source rows of bits B0..B0+3: identity blocks, one XOR
// into row 8g + b of every coding device g.
template <int B0>
__device__ __forceinline__ void xor_dev0_4(uint32_t (&acc)[32][4], const u32x4 (&x)[4]) {
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[8 * g + B0 + u][c] ^= x[u][c];
}

// Any other device's rows of bits B0..B0+3: row b of coding device 0 by XOR,
// rows 8..31 by their masks.
template <int B0>
__device__ __forceinline__ void xor_unit4(uint32_t (&acc)[32][4], const u32x4 (&x)[4], const uint32_t (&m)[4]) {
#pragma unroll
  for (int u = 0; u < 4; ++u) {
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[B0 + u][c] ^= x[u][c];
#pragma unroll
    for (int r = 8; r < 32; ++r) {
      const uint32_t sel = uint32_t(int32_t(m[u] << (31 - r)) >> 31);
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[r][c] = __builtin_amdgcn_bitop3_b32(acc[r][c], x[u][c], sel, 0x78);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// WPE: minimum waves per SIMD asked of the register allocator (3: 168 VGPRs
// with a 12-B spill, as the general kernel's 166; 1: 170 VGPRs, 2 waves).
template <int RT = 32, int WPE = 3>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(WPE))) void gf_xor_packets16u(PacketArgs a) {
  static_assert(RT == 32, "the unit form is the 4 x 8-row map of an RS(k, 4) w = 8 encode");
  const int64_t g = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (g >= a.ncols) return;
  int64_t sp, col;
  packet_coords(a, g, &sp, &col);
  const int64_t soff = sp * a.sstride + col * 16, doff = sp * a.dstride + col * 16;
  uint32_t acc[32][4];
#pragma unroll
  for (int r = 0; r < 32; ++r) acc[r][0] = acc[r][1] = acc[r][2] = acc[r][3] = 0u;
  const int nc = a.nsrc >> 2;  // even: 8 source rows per data device
  u32x4 xa[4], xb[4];
  uint32_t ma[4], mb[4];
  auto load4 = [&](u32x4 (&x)[4], uint32_t (&m)[4], int c) {
    const int b = (c < nc ? c : nc - 1) * 4;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      m[u] = kload(a.mask, b + u);
      x[u] = load16t<1>(kload(a.src, b + u) + soff, 0);
    }
  };
  // chunk 2d holds bits 0..3 of data device d, chunk 2d + 1 bits 4..7;
  // device 0 first (its rows need no masks), then the double-buffered loop
  load4(xa, ma, 0);
  load4(xb, mb, 1);
  xor_dev0_4<0>(acc, xa);
  load4(xa, ma, 2);
  xor_dev0_4<4>(acc, xb);
  for (int c = 2; c < nc; c += 2) {
    load4(xb, mb, c + 1);
    xor_unit4<0>(acc, xa, ma);
    load4(xa, ma, c + 2);
    xor_unit4<4>(acc, xb, mb);
  }
#pragma unroll
  for (int r = 0; r < 32; ++r)
    store16t<1>(kload(a.dst, r) + doff, 0, u32x4{acc[r][0], acc[r][1], acc[r][2], acc[r][3]});
}

// Byte form for packet sizes / bases that are not 8-byte aligned.
[[maybe_unused]] static __global__ __launch_bounds__(kBlock) void gf_xor_packets_bytes(PacketArgs a) {
  const int64_t g = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (g >= a.ncols) return;
  int64_t sp, col;
  packet_coords(a, g, &sp, &col);
  const int64_t soff = sp * a.sstride + col, doff = sp * a.dstride + col;
  uint8_t out[32];
  for (int r = 0; r < 32; ++r) out[r] = 0;
  for (int j = 0; j < a.nsrc; ++j) {
    const uint8_t x = a.src[j][soff];
    const uint32_t m = a.mask[j];
    for (int r = 0; r < a.R; ++r)
      if ((m >> r) & 1u) out[r] ^= x;
  }
  for (int r = 0; r < a.R; ++r) a.dst[r][doff] = out[r];
}

}  // namespace dev
}  // namespace ecgpu
