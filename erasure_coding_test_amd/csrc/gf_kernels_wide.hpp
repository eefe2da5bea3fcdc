// gf_kernels_wide.hpp -- w = 16 / 32 kernels: the v_perm form generalised to
// wider words, the LDS nibble-table kernels (32-bit entries, packed w = 16 pairs)
// and the pipelined-load form.  Included through gf_kernels.hpp.
#pragma once
#include "gf_kernels_w8.hpp"

namespace ecgpu {
namespace dev {

// ------------------------------------------- wide words (w = 16 and 32) ----
// jerasure.h's w = 16 / 32 surface (galois.cpp:469-729).  c*x in GF(2^16) or
// GF(2^32) is GF(2)-linear in x, so output byte o of c*x is the XOR over
// input bytes b of a byte->byte linear map L_{b->o}, and every such map
// splits into four 2-bit-slice lookups exactly as at w = 8.  Rotating the
// word by d bytes puts input byte b = (o + d) mod W under output lane o, so
// ONE v_perm per (rotation, slice) serves every lane whose table differs only
// by lane class:
//   w = 16 (W = 2): lane classes even / odd -> table A in the low dword of
//     the v_perm pool (selectors 0..3), B in the high dword (4..7):
//     2 rotations x 4 slices = 8 v_perm per coefficient-dword;
//   w = 32 (W = 4): four lane classes -> two v_perm per (rotation, slice),
//     each zeroing the other lane pair with selector 0x0C:
//     4 x 4 x 2 = 32 v_perm per coefficient-dword.
// Table word pairs per v_perm: [2i] = pool high dword (B), [2i+1] = low (A).
template <int W>
struct Wide;
template <>
struct Wide<2> {
  static constexpr int kPerms = 8;
};
template <>
struct Wide<4> {
  static constexpr int kPerms = 32;
};

template <int W>
__device__ __forceinline__ void wide_sel(uint32_t x, uint32_t (&sel)[Wide<W>::kPerms]) {
  if constexpr (W == 2) {
    const uint32_t xs = __builtin_amdgcn_perm(x, x, 0x02030001u);  // swap the bytes of each 16-bit word
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      sel[p] = ((x >> (2 * p)) & kLo2) | 0x04000400u;
      sel[4 + p] = ((xs >> (2 * p)) & kLo2) | 0x04000400u;
    }
  } else {
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const uint32_t xr = d == 0 ? x : __builtin_amdgcn_alignbit(x, x, 8 * d);  // rotr(x, 8d)
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const uint32_t t = (xr >> (2 * p)) & kLo2;
        sel[(d * 4 + p) * 2 + 0] = (t & 0x00000303u) | 0x0C0C0400u;
        sel[(d * 4 + p) * 2 + 1] = (t & 0x03030000u) | 0x04000C0Cu;
      }
    }
  }
}

template <int W, typename TP>
__device__ __forceinline__ uint32_t wide_mac(uint32_t acc, const TP* __restrict__ t,
                                             const uint32_t (&sel)[Wide<W>::kPerms]) {
#pragma unroll
  for (int i = 0; i < Wide<W>::kPerms; i += 2)
    acc = xor3(acc, __builtin_amdgcn_perm(t[2 * i], t[2 * i + 1], sel[i]),
               __builtin_amdgcn_perm(t[2 * i + 2], t[2 * i + 3], sel[i + 1]));
  return acc;
}

// 16-byte columns: lane l of block b handles column b*256 + l of every shard
// of stripe blockIdx.y; runtime K (the w = 16/32 surface is not the hot path).
template <int W, int R>
__global__ __launch_bounds__(kBlock) void gf_apply_wide(ApplyArgs a) {
  const int64_t col = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (col >= a.nvec) return;
  const int s = blockIdx.y;
  const uint8_t* const* sp = a.src + int64_t(s) * a.src_stride;
  uint8_t* dp[R];
#pragma unroll
  for (int r = 0; r < R; ++r) dp[r] = a.dst[int64_t(s) * a.dst_stride + a.row0 + r];
  constexpr int kWords = 2 * Wide<W>::kPerms;
  // sources in chunks of kWideChunk: every load of a chunk is in flight
  // before its first use (a load-use loop over runtime K keeps one 16-B load
  // per lane in flight and is latency-bound)
  constexpr int kWideChunk = 8;
  u32x4 acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = u32x4{0u, 0u, 0u, 0u};
  for (int j0 = 0; j0 < a.K; j0 += kWideChunk) {
    u32x4 xs[kWideChunk];
#pragma unroll
    for (int u = 0; u < kWideChunk; ++u)
      if (j0 + u < a.K) xs[u] = load16t<1>(sp[j0 + u], col);
#pragma unroll
    for (int u = 0; u < kWideChunk; ++u) {
      const int j = j0 + u;
      if (j >= a.K) break;
      const u32x4 x = xs[u];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        uint32_t sel[Wide<W>::kPerms];
        wide_sel<W>(x[c], sel);
#pragma unroll
        for (int r = 0; r < R; ++r) {
          if constexpr (W == 2) {
            // branch-free at w = 16: a unit or zero coefficient's tables are
            // the identity / zero map, so every term goes through wide_mac and
            // the chunk body is straight-line (352 vs 410 us per 64 MiB
            // RS(10,4) encode).  At w = 32 (32 v_perm per term) skipping the
            // 13 unit terms wins instead (1.18 vs 2.72 ms).
            acc[r][c] = wide_mac<W>(acc[r][c], (const kconst_u32*)a.wtab + size_t(r * a.K + j) * kWords, sel);
          } else {
            const uint8_t cls = a.wcls[r * a.K + j];
            if (cls == 2) continue;
            if (cls == 1) {
              acc[r][c] ^= x[c];
              continue;
            }
            acc[r][c] = wide_mac<W>(acc[r][c], a.wtab + size_t(r * a.K + j) * kWords, sel);
          }
        }
      }
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) store16t<1>(dp[r], col, acc[r]);
}

// Words from byte0 to size (tails, or whole regions whose pointers are not
// 16-B aligned): one W-byte word per lane, byte loads and stores.
template <int W>
__global__ __launch_bounds__(kBlock) void gf_apply_wide_words(ApplyArgs a) {
  const int64_t x0 = a.byte0 + (int64_t(blockIdx.x) * kBlock + threadIdx.x) * W;
  if (x0 + W > a.size) return;
  const int s = blockIdx.y;
  const uint8_t* const* sp = a.src + int64_t(s) * a.src_stride;
  constexpr int kWords = 2 * Wide<W>::kPerms;
  uint32_t acc[kMaxRows] = {0u, 0u, 0u, 0u};
  for (int j = 0; j < a.K; ++j) {
    const uint8_t* q = sp[j] + x0;
    uint32_t x = 0;
#pragma unroll
    for (int b = 0; b < W; ++b) x |= uint32_t(q[b]) << (8 * b);
    uint32_t sel[Wide<W>::kPerms];
    wide_sel<W>(x, sel);
    for (int r = 0; r < a.R; ++r) {
      const uint8_t cls = a.wcls[r * a.K + j];
      if (cls == 2) continue;
      acc[r] = cls == 1 ? (acc[r] ^ x) : wide_mac<W>(acc[r], a.wtab + size_t(r * a.K + j) * kWords, sel);
    }
  }
  for (int r = 0; r < a.R; ++r) {
    uint8_t* d = a.dst[int64_t(s) * a.dst_stride + a.row0 + r] + x0;
#pragma unroll
    for (int b = 0; b < W; ++b) d[b] = uint8_t(acc[r] >> (8 * b));
  }
}

// ------------------------------------- wide words, LDS nibble tables ----
// Second engine for w = 16 / 32 (production when the tables fit, below).
// c*x is GF(2)-linear, so for any dword x of a w = 16 / 32 region
//     c*x = XOR_t T_t[nibble t of x],   t = 0..7,
// with eight 16-entry dword tables per coefficient: w = 32: T_t[v] =
// c*(v << 4t); w = 16 (two words per dword): T_t[v] = c*(v << 4t) for t < 4
// (low word, entries in bits 0..15) and (c*(v << 4(t-4))) << 16 for t >= 4
// (high word).  Unit and zero coefficients are the identity / zero tables,
// so the body is branch-free.  The launch's rows share one LDS entry per
// (source, t, v): 8 B for R <= 2 (ds_read_b64), 16 B for R = 3, 4
// (ds_read_b128): one read does every row's lookup at the LDS array's full
// 256 B/clk (MI355X_MICROARCH.md §LDS; two ds_read_b64 at a 1 KiB distance
// would be merged by the compiler into ds_read2_b64, which runs at half that
// rate), and a 16-entry table of 8- or 16-B entries never puts two distinct
// addresses of one lane group on a bank.  Per source dword: 16 VALU for the
// eight lookup addresses (shared by every row), 8 LDS reads and 4 XOR3 per
// row -- against 32 v_perm per coefficient at w = 32 for gf_apply_wide.
// Workgroups loop over column blocks so the table staging (K * 1 or 2 KiB
// from L2) is amortised.
constexpr int kNibWords = 128;  // dwords of one coefficient's 8 tables
constexpr int kNibMaxLds = 64 * 1024;

__host__ __device__ constexpr int nib_entry_words(int R) { return R <= 2 ? 2 : 4; }
// LDS bytes of one source's tables for a launch of R rows
__host__ __device__ constexpr int nib_source_bytes(int R) { return kNibWords * 4 * nib_entry_words(R); }
// ... and of the whole launch: U = 1 (row 0 and column 0 all ones, below)
// keeps rows 1..R-1 of sources 1..K-1 only
__host__ __device__ constexpr int nib_lds_bytes(int K, int R, int U) {
  return (K - U) * nib_source_bytes(R - U);
}

typedef __attribute__((address_space(3))) const u32x2 lds_u32x2;

// U = 1: the launch's row 0 and column 0 are all ones -- every
// reed_sol_vandermonde_coding_matrix encode (reed_sol.cpp:324-349), checked
// exactly by the host per launch.  Row 0 is then the XOR of the sources and
// source 0 is XORed into every row: no lookups for either, and the LDS holds
// the L = R - 1 other rows of sources 1..K-1 (RS(10,4) w = 32: 72 instead of
// 80 ds_read_b128 per lane-column).  With fewer registers live (four source
// loads in flight, the eight lookups folded in two groups of four) the kernel
// runs 7 waves per SIMD instead of 5 (68 VGPRs).  RS(10,4) w = 32 64 MiB,
// tools/wide_lab.hip, 15 interleaved rounds: 191-195 us against 204-209 for
// the U = 0 form (profiles/r03_wide_lab.jsonl).
template <int R, int U = 0>
__global__ __launch_bounds__(kBlock) void gf_apply_wide_nib(ApplyArgs a) {
  static_assert(U == 0 || R >= 2, "U = 1 needs a row besides the unit row");
  constexpr int L = R - U;  // rows looked up in LDS
  constexpr int EW = nib_entry_words(L), EB = 4 * EW;
  constexpr int kChunk = U ? 4 : 8;   // source loads in flight before the first use
  constexpr int kGroups = U ? 2 : 1;  // lookups issued and folded in kGroups groups
  extern __shared__ __attribute__((aligned(16))) uint8_t nib_lds[];
  const int K = a.K;
  // LDS dword (((j - U) * 128 + t * 16 + v) * EW + l) = T[l + U][j][t][v] (0 for l >= L);
  // a.wtab is [R][K][kNibWords] for this launch's rows
  const int n = (K - U) * kNibWords * EW;
  for (int i = threadIdx.x; i < n; i += kBlock) {
    const int l = i % EW, e = (i / EW) % kNibWords, j = i / (EW * kNibWords) + U;
    reinterpret_cast<uint32_t*>(nib_lds)[i] = l < L ? a.wtab[size_t((l + U) * K + j) * kNibWords + e] : 0u;
  }
  __syncthreads();

  const int s = blockIdx.y;
  const uint8_t* const* sp = a.src + int64_t(s) * a.src_stride;
  uint8_t* dp[R];
#pragma unroll
  for (int r = 0; r < R; ++r) dp[r] = a.dst[int64_t(s) * a.dst_stride + a.row0 + r];
  const uint32_t lds_base = uint32_t(reinterpret_cast<uintptr_t>(static_cast<void*>(nib_lds)));
  const int64_t nblk = (a.nvec + kBlock - 1) / kBlock;
  for (int64_t b = blockIdx.x; b < nblk; b += gridDim.x) {
    const int64_t col = b * kBlock + threadIdx.x;
    if (col >= a.nvec) continue;
    u32x4 acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = u32x4{0u, 0u, 0u, 0u};
    for (int j0 = 0; j0 < K; j0 += kChunk) {
      u32x4 xs[kChunk];
#pragma unroll
      for (int u = 0; u < kChunk; ++u)
        if (j0 + u < K) xs[u] = load16t<1>(kload(sp, j0 + u), col);
#pragma unroll
      for (int u = 0; u < kChunk; ++u) {
        const int j = j0 + u;
        if (j >= K) break;
        if (U == 1) {
          if (j == 0) {  // column 0: a unit in every row
#pragma unroll
            for (int r = 0; r < R; ++r) acc[r] ^= xs[u];
            continue;
          }
          acc[0] ^= xs[u];  // row 0: units
        }
        // LDS byte address of source j's tables; the kernel has no static LDS,
        // so the dynamic allocation starts at 0 and jbase < 64 KiB (K <= 32)
        const uint32_t jbase = lds_base + uint32_t(j - U) * uint32_t(nib_source_bytes(L));
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const uint32_t x = xs[u][c];
          // lookup addresses, one v_perm each: nibble t = 2b (+1) of x, scaled
          // by EB, sits in byte b of ns[0] (ns[1]); v_perm takes that byte and
          // bytes 1, 2 of jbase (< 64 KiB, byte 0 zero); t's table offset is
          // the ds_read immediate
          constexpr int kSh = EB == 16 ? 4 : 3;
          constexpr uint32_t kNibMask = 0x0F0F0F0Fu << kSh;
          const uint32_t ns[2] = {(x << kSh) & kNibMask, (x >> (4 - kSh)) & kNibMask};
#pragma unroll
          for (int g = 0; g < kGroups; ++g) {
            constexpr int TN = 8 / kGroups;
            uint32_t v[TN][EW];
#pragma unroll
            for (int tt = 0; tt < TN; ++tt) {
              const int t = g * TN + tt;
              const uint32_t ad = __builtin_amdgcn_perm(jbase, ns[t & 1], 0x0C060500u | uint32_t(t >> 1)) +
                                  uint32_t(t * 16 * EB);
              if constexpr (EW == 2) {
                const u32x2 q = *(lds_u32x2*)(size_t(ad));
                v[tt][0] = q.x;
                v[tt][1] = q.y;
              } else {
                const u32x4 q = *(lds_u32x4*)(size_t(ad));
#pragma unroll
                for (int l = 0; l < 4; ++l) v[tt][l] = q[l];
              }
            }
#pragma unroll
            for (int l = 0; l < L; ++l) {
              uint32_t e = acc[l + U][c];
#pragma unroll
              for (int tt = 0; tt < TN; tt += 2) e = xor3(e, v[tt][l], v[tt + 1][l]);
              acc[l + U][c] = e;
            }
          }
        }
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) store16t<1>(dp[r], col, acc[r]);
  }
}

// w = 16 variant with two rows per LDS dword.  w = 16 products are 16-bit,
// so one dword entry packs rows 2p and 2p+1: (j, t, v) -> [row 2p | row 2p+1]
// of c*(v << 4t') for the word that nibble t belongs to (t < 4: low word,
// t >= 4: high word, t' = t mod 4).  An entry is 4 B for R <= 2 and 8 B for
// R = 3, 4 -- half of gf_apply_wide_nib's LDS bytes per lookup (that kernel
// is LDS-bound) -- and the folding works on packed row pairs: per pair one
// accumulator for the low-word tables, one for the high-word tables (2 XOR3
// each per source dword, half of the per-row form), and at the end one
// v_perm per row interleaves them: row 2p = [lo.lo16 | hi.lo16], row 2p+1 =
// [lo.hi16 | hi.hi16].  The entries are derived in the staging loop from the
// same per-coefficient tables (a.wtab, [R][K][kNibWords]).
__host__ __device__ constexpr int nib16_entry_words(int R) { return R <= 2 ? 1 : 2; }
__host__ __device__ constexpr int nib16_source_bytes(int R) { return kNibWords * 4 * nib16_entry_words(R); }

// U = 1: the unit structure of gf_apply_wide_nib<R, 1> (the launch's row 0
// and column 0 all ones, as in every Vandermonde encode): row 0 is the XOR of
// the sources and source 0 is XORed into every row, so the LDS holds the
// packed pairs of rows 1..R-1 (pair p = rows 1 + 2p, 2 + 2p) for sources
// 1..K-1 only -- 1/K fewer lookups, and for R = 3 one dword entry instead of
// two.  Production for such launches since round 4 (the wide16_units knob,
// ECGPU_WIDE16_UNITS; RS(10,4) 64 MiB through jerasure_matrix_encode 176.0 ->
// 174.7 us on separate shards, 174.1 -> 171.1 on the slab, lab 171.0 -> 168.9,
// profiles/r04_ab_wide16_units.json, r04_wide_lab_w16.jsonl).
template <int R, int U = 0>
__global__ __launch_bounds__(kBlock) void gf_apply_wide_nib16(ApplyArgs a) {
  static_assert(U == 0 || R >= 2, "the unit form needs a row besides the unit row");
  constexpr int L = R - U;  // rows looked up, packed in pairs
  constexpr int EW = nib16_entry_words(L), EB = 4 * EW;
  extern __shared__ __attribute__((aligned(16))) uint8_t nib_lds[];
  const int K = a.K;
  const int n = (K - U) * kNibWords * EW;
  for (int i = threadIdx.x; i < n; i += kBlock) {
    const int pr = i % EW, e = (i / EW) % kNibWords, j = i / (EW * kNibWords) + U;
    const bool high = (e >> 4) >= 4;  // tables 4..7 hold the high word's products in bits 16..31
    auto word = [&](int r) -> uint32_t {
      if (r >= R) return 0u;
      const uint32_t v = a.wtab[size_t(r * K + j) * kNibWords + e];
      return high ? (v >> 16) : (v & 0xFFFFu);
    };
    reinterpret_cast<uint32_t*>(nib_lds)[i] = word(U + 2 * pr) | (word(U + 2 * pr + 1) << 16);
  }
  __syncthreads();

  const int s = blockIdx.y;
  const uint8_t* const* sp = a.src + int64_t(s) * a.src_stride;
  uint8_t* dp[R];
#pragma unroll
  for (int r = 0; r < R; ++r) dp[r] = a.dst[int64_t(s) * a.dst_stride + a.row0 + r];
  const uint32_t lds_base = uint32_t(reinterpret_cast<uintptr_t>(static_cast<void*>(nib_lds)));
  constexpr int kChunk = 8;  // source loads in flight before the first use
  const int64_t nblk = (a.nvec + kBlock - 1) / kBlock;
  for (int64_t b = blockIdx.x; b < nblk; b += gridDim.x) {
    const int64_t col = b * kBlock + threadIdx.x;
    if (col >= a.nvec) continue;
    uint32_t lo[4][EW], hi[4][EW];  // [dword c][row pair]
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int q = 0; q < EW; ++q) lo[c][q] = hi[c][q] = 0u;
    u32x4 x0 = u32x4{0u, 0u, 0u, 0u}, row0 = u32x4{0u, 0u, 0u, 0u};
    if constexpr (U == 1) {
      x0 = load16t<1>(kload(sp, 0), col);  // column 0: into every row
      row0 = x0;                            // row 0: the XOR of the sources
    }
    for (int j0 = U; j0 < K; j0 += kChunk) {
      u32x4 xs[kChunk];
#pragma unroll
      for (int u = 0; u < kChunk; ++u)
        if (j0 + u < K) xs[u] = load16t<1>(kload(sp, j0 + u), col);
#pragma unroll
      for (int u = 0; u < kChunk; ++u) {
        const int j = j0 + u;
        if (j >= K) break;
        if constexpr (U == 1) row0 ^= xs[u];
        const uint32_t jbase = lds_base + uint32_t(j - U) * uint32_t(nib16_source_bytes(L));
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const uint32_t x = xs[u][c];
          // nibble t of x scaled by EB in byte t/2 of ns[t & 1] (see gf_apply_wide_nib)
          constexpr int kSh = EB == 8 ? 3 : 2;
          constexpr uint32_t kNibMask = 0x0F0F0F0Fu << kSh;
          const uint32_t ns[2] = {(x << kSh) & kNibMask, (x >> (4 - kSh)) & kNibMask};
          uint32_t v[8][EW];
#pragma unroll
          for (int t = 0; t < 8; ++t) {
            const uint32_t ad = __builtin_amdgcn_perm(jbase, ns[t & 1], 0x0C060500u | uint32_t(t >> 1)) +
                                uint32_t(t * 16 * EB);
            if constexpr (EW == 1) {
              v[t][0] = *(lds_u32*)(size_t(ad));
            } else {
              const u32x2 q = *(lds_u32x2*)(size_t(ad));
              v[t][0] = q.x;
              v[t][1] = q.y;
            }
          }
#pragma unroll
          for (int q = 0; q < EW; ++q) {
            lo[c][q] = xor3(xor3(lo[c][q], v[0][q], v[1][q]), v[2][q], v[3][q]);
            hi[c][q] = xor3(xor3(hi[c][q], v[4][q], v[5][q]), v[6][q], v[7][q]);
          }
        }
      }
    }
    if constexpr (U == 1) store16t<1>(dp[0], col, row0);
#pragma unroll
    for (int r = U; r < R; ++r) {
      const int l = r - U;  // looked-up row: pair l / 2, half l % 2
      u32x4 o;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        o[c] = __builtin_amdgcn_perm(hi[c][l >> 1], lo[c][l >> 1], (l & 1) ? 0x07060302u : 0x05040100u);
        if constexpr (U == 1) o[c] ^= x0[c];
      }
      store16t<1>(dp[r], col, o);
    }
  }
}

// ------------------------------------- wide words, pipelined loads ----
// The two nibble kernels above with compile-time K and software-pipelined
// shard loads.  Production where it measured faster: launches of whole
// 256-column blocks in the w = 32 unit form with 7-10 sources
// (ecgpu_runtime.hip plan_launch_wide; ECGPU_WIDE_PIPE=2 takes it for every
// whole-block launch of every mode, for tests and A/B).  The K
// sources of a column are NCH (even) chunks of CH, and the chunk sequence is
// double-buffered across the workgroup's column blocks: chunk c + 1's loads
// (after the last chunk, the next block's chunk 0) are issued before chunk
// c's lookups.  Every load and store is unconditional -- the last prefetch
// re-reads the workgroup's own block and the launch covers whole column
// blocks -- so the compiler's wait counts are static and a wave waits only
// for the chunk it is about to look up.  The runtime-K kernels load a chunk
// and wait for it before any lookup, leaving the wait to other waves to
// hide (a first pipelined form with conditional loads got vmcnt(0) before
// every chunk and ran slower).  RS(K,4) 64 MiB, tools/wide_lab.hip in one
// process, unit form: K = 7 148 -> 139 us, K = 8 162 -> 149, K = 10 195 ->
// 184-191; K = 5, 11, 12, the general w = 32 form and w = 16 within +-3 %
// (profiles/r03_wide_lab.jsonl, runs "r03 pipe ...").
enum WidePipeMode : int { kPipeW32 = 0, kPipeW32Unit = 1, kPipeW16 = 2 };

template <int K, int MODE, int NCHO = 0>
struct WidePipeShape {
  // chunks per column: w = 32 four for K = 7..12 (RS(10,4): 3 + 3 + 3 + 1,
  // 101 VGPRs, 4 workgroups per CU) except the unit form at K = 12: six
  // chunks of 2 hold 128 VGPRs (4 workgroups per CU) where four hold 131 (3
  // per CU) -- RS(12,4) w = 32 64 MiB 235.3 -> 216.8 us, and 4.7 % under the
  // unpipelined unit kernel's 227.6 (tools/wide_lab.hip, round 4); w = 16
  // two (5 + 5); NCHO > 0 overrides (even)
  static constexpr int NCH = NCHO > 0                             ? NCHO
                             : MODE == kPipeW16                   ? 2
                             : (MODE == kPipeW32Unit && K == 12) ? 6
                                                                  : 2 * ((K + 5) / 6);
  static constexpr int CH = (K + NCH - 1) / NCH;
};

template <int K, int R, int MODE, int WPE = 1, int NCHO = 0, int FG = 4>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(WPE))) void gf_apply_wide_pipe(ApplyArgs a) {
  static_assert(FG == 4 || FG == 2, "lookups folded four or two at a time");
  constexpr bool W16 = MODE == kPipeW16;
  constexpr int U = MODE == kPipeW32Unit ? 1 : 0;
  static_assert(U == 0 || R >= 2, "the unit form needs a row besides the unit row");
  constexpr int L = R - U;  // rows looked up (w = 32)
  constexpr int EW = W16 ? nib16_entry_words(R) : nib_entry_words(L), EB = 4 * EW;
  constexpr uint32_t kSrcBytes = uint32_t(W16 ? nib16_source_bytes(R) : nib_source_bytes(L));
  constexpr int NCH = WidePipeShape<K, MODE, NCHO>::NCH, CH = WidePipeShape<K, MODE, NCHO>::CH;
  static_assert(NCH % 2 == 0, "buffer parity repeats per column");
  extern __shared__ __attribute__((aligned(16))) uint8_t nib_lds[];
  {
    // the LDS images of gf_apply_wide_nib<R, U> / gf_apply_wide_nib16<R>
    const int n = (K - U) * kNibWords * EW;
    for (int i = threadIdx.x; i < n; i += kBlock) {
      const int l = i % EW, e = (i / EW) % kNibWords, j = i / (EW * kNibWords) + U;
      uint32_t v;
      if constexpr (W16) {
        const bool high = (e >> 4) >= 4;
        auto word = [&](int r) -> uint32_t {
          if (r >= R) return 0u;
          const uint32_t t = a.wtab[size_t(r * K + j) * kNibWords + e];
          return high ? (t >> 16) : (t & 0xFFFFu);
        };
        v = word(2 * l) | (word(2 * l + 1) << 16);
      } else {
        v = l < L ? a.wtab[size_t((l + U) * K + j) * kNibWords + e] : 0u;
      }
      reinterpret_cast<uint32_t*>(nib_lds)[i] = v;
    }
  }
  __syncthreads();

  const int s = blockIdx.y;
  const uint8_t* const* sp = a.src + int64_t(s) * a.src_stride;
  uint8_t* dp[R];
#pragma unroll
  for (int r = 0; r < R; ++r) dp[r] = a.dst[int64_t(s) * a.dst_stride + a.row0 + r];
  const uint32_t lds_base = uint32_t(reinterpret_cast<uintptr_t>(static_cast<void*>(nib_lds)));
  const int64_t nblk = a.nvec / kBlock;  // whole column blocks (host-checked)
  const int64_t g = gridDim.x;
  int64_t b = blockIdx.x;
  if (b >= nblk) return;

  auto load = [&](u32x4 (&x)[CH], int64_t bb, int c) {
    const int64_t col = bb * kBlock + threadIdx.x;
#pragma unroll
    for (int u = 0; u < CH; ++u)
      if (c * CH + u < K) x[u] = load16t<1>(kload(sp, c * CH + u), col);  // compile-time test
  };
  u32x4 acc[R];            // w = 32: rows
  uint32_t lo[4][EW], hi[4][EW];  // w = 16: [dword][row pair], low / high word tables
  auto apply = [&](const u32x4 (&x)[CH], int c) {
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      const int j = c * CH + u;
      if (j >= K) break;
      if (U == 1) {
        if (j == 0) {  // column 0: a unit in every row
#pragma unroll
          for (int r = 0; r < R; ++r) acc[r] ^= x[u];
          continue;
        }
        acc[0] ^= x[u];  // row 0: units
      }
      const uint32_t jbase = lds_base + uint32_t(j - U) * kSrcBytes;
#pragma unroll
      for (int cc = 0; cc < 4; ++cc) {
        // nibble t of x scaled by EB in byte t/2 of ns[t & 1] (see gf_apply_wide_nib)
        constexpr int kSh = EB == 16 ? 4 : EB == 8 ? 3 : 2;
        constexpr uint32_t kNibMask = 0x0F0F0F0Fu << kSh;
        const uint32_t xv = x[u][cc];
        const uint32_t ns[2] = {(xv << kSh) & kNibMask, (xv >> (4 - kSh)) & kNibMask};
#pragma unroll
        for (int h = 0; h < 8 / FG; ++h) {  // lookups in groups of FG, each folded before the next
          uint32_t v[4][EW];
#pragma unroll
          for (int tt = 0; tt < FG; ++tt) {
            const int t = h * FG + tt;
            const uint32_t ad = __builtin_amdgcn_perm(jbase, ns[t & 1], 0x0C060500u | uint32_t(t >> 1)) +
                                uint32_t(t * 16 * EB);
            if constexpr (EW == 1) {
              v[tt][0] = *(lds_u32*)(size_t(ad));
            } else if constexpr (EW == 2) {
              const u32x2 q = *(lds_u32x2*)(size_t(ad));
              v[tt][0] = q.x;
              v[tt][1] = q.y;
            } else {
              const u32x4 q = *(lds_u32x4*)(size_t(ad));
#pragma unroll
              for (int l = 0; l < 4; ++l) v[tt][l] = q[l];
            }
          }
          if constexpr (W16) {
#pragma unroll
            for (int q = 0; q < EW; ++q) {
              uint32_t& e = h * FG < 4 ? lo[cc][q] : hi[cc][q];  // tables 0-3 low word, 4-7 high word
              e = FG == 4 ? xor3(xor3(e, v[0][q], v[1][q]), v[2][q], v[3][q]) : xor3(e, v[0][q], v[1][q]);
            }
          } else {
#pragma unroll
            for (int l = 0; l < L; ++l)
              acc[l + U][cc] = FG == 4 ? xor3(xor3(acc[l + U][cc], v[0][l], v[1][l]), v[2][l], v[3][l])
                                       : xor3(acc[l + U][cc], v[0][l], v[1][l]);
          }
        }
      }
    }
  };

  u32x4 buf[2][CH];
  load(buf[0], b, 0);
  for (;;) {
    const int64_t bn = b + g < nblk ? b + g : b;  // the last prefetch re-reads this block
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
    for (int cc = 0; cc < 4; ++cc)
#pragma unroll
      for (int q = 0; q < EW; ++q) lo[cc][q] = hi[cc][q] = 0u;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      if (c + 1 < NCH)
        load(buf[(c + 1) & 1], b, c + 1);
      else
        load(buf[0], bn, 0);
      apply(buf[c & 1], c);
    }
    const int64_t col = b * kBlock + threadIdx.x;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if constexpr (W16) {
        u32x4 o;
#pragma unroll
        for (int cc = 0; cc < 4; ++cc)
          o[cc] = __builtin_amdgcn_perm(hi[cc][r >> 1], lo[cc][r >> 1], (r & 1) ? 0x07060302u : 0x05040100u);
        store16t<1>(dp[r], col, o);
      } else {
        store16t<1>(dp[r], col, acc[r]);
      }
    }
    if (bn == b) break;
    b = bn;
  }
}

}  // namespace dev
}  // namespace ecgpu
