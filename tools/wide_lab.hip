// wide_lab.hip -- A/B lab for the w = 32 (and w = 16) LDS nibble-table
// column kernels: RS(k,m) encode of one stripe of S-byte device shards laid
// out at the library's skewed stride, every variant checked bit-exact against
// the production kernel (and that one against a host GF(2^w) multiply on
// sample columns), then timed in interleaved rounds with HIP events.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include -I erasure_coding_test_amd/csrc \
//     tools/wide_lab.hip erasure_coding_test_amd/csrc/gf_host.cpp erasure_coding_test_amd/csrc/matrix_host.cpp -o tools/wide_lab.bin
//   tools/wide_lab.bin [--w 32] [--k 10] [--m 4] [--mib 64] [--rounds 7] [--reps 10] [--only name,name] [--skew-kib N]
//
// Prints one JSON line per variant: median / min us and GB/s of (k+m)*S.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
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

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                      \
    }                                                                                    \
  } while (0)

namespace lab {

typedef __attribute__((address_space(3))) const uint32_t lds_u32c;
typedef __attribute__((address_space(3))) const u32x2 lds_u32x2c;
typedef __attribute__((address_space(3))) const u32x4 lds_u32x4c;
typedef const uint8_t* gptr;
typedef __attribute__((address_space(4))) const gptr kptr;  // a pointer-table entry in constant memory

// Split-entry nibble kernel.  U = 1: row 0 and column 0 of the launch are all
// ones (a Vandermonde encode), so row 0 is the XOR of the sources, source 0
// is XORed into every row, and the LDS holds rows 1..R-1 of sources 1..K-1
// only.  The L = R - U LDS rows are stored as NP = ceil(L/2) pair tables of
// 8-B entries per (source, nibble t) (the last one a single row read with
// ds_read_b32 when L is odd), or, with B128 and L = 4, one 16-B entry.
template <int R, int U, bool B128, int CHUNK = 8, int HALVES = 1, int WPE = 1>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(WPE))) void nib_split(ApplyArgs a) {
  constexpr int L = R - U;
  constexpr bool kWide = B128 && L >= 3;
  constexpr int NP = kWide ? 1 : (L + 1) / 2;        // LDS blocks per (source, t)
  constexpr int kBlkBytes = kWide ? 256 : 128;       // bytes of one block (16 entries)
  constexpr int kTBytes = NP * kBlkBytes;            // bytes per (source, t)
  constexpr int kSrcBytes = 8 * kTBytes;
  constexpr int kEntry = kWide ? 16 : 8;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int K = a.K, KL = K - U;
  // staging: dword index i of the LDS image
  {
    uint32_t* w = reinterpret_cast<uint32_t*>(lds);
    const int n = KL * kSrcBytes / 4;
    for (int i = threadIdx.x; i < n; i += kBlock) {
      const int jj = i / (kSrcBytes / 4), rem = i % (kSrcBytes / 4);
      const int t = rem / (kTBytes / 4), r2 = rem % (kTBytes / 4);
      const int blk = r2 / (kBlkBytes / 4), r3 = r2 % (kBlkBytes / 4);
      const int v = r3 / (kEntry / 4), word = r3 % (kEntry / 4);
      const int lr = kWide ? word : 2 * blk + word;  // LDS row
      const int row = lr + U, j = jj + U;
      w[i] = lr < L ? a.wtab[size_t(row * K + j) * kNibWords + t * 16 + v] : 0u;
    }
  }
  __syncthreads();
  // the pointer table through the constant address space: scalar loads, even
  // inside the column loop after stores (a generic load there is a vector
  // load whose vmcnt(0) wait serialises every shard load issued before it)
  const kptr* sp = (const kptr*)a.src;
  uint8_t* dp[R];
#pragma unroll
  for (int r = 0; r < R; ++r) dp[r] = a.dst[a.row0 + r];
  const uint32_t lds_base = uint32_t(reinterpret_cast<uintptr_t>(static_cast<void*>(lds)));
  constexpr int kChunk = CHUNK;
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
        if (j0 + u < K) xs[u] = load16t<1>(sp[j0 + u], col);
#pragma unroll
      for (int u = 0; u < kChunk; ++u) {
        const int j = j0 + u;
        if (j >= K) break;
        if (U == 1 && j == 0) {
#pragma unroll
          for (int r = 0; r < R; ++r) acc[r] ^= xs[u];
          continue;
        }
        if (U == 1) acc[0] ^= xs[u];
        const uint32_t jbase = lds_base + uint32_t(j - U) * uint32_t(kSrcBytes);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const uint32_t x = xs[u][c];
          constexpr int kSh = kEntry == 16 ? 4 : 3;
          constexpr uint32_t kNibMask = 0x0F0F0F0Fu << kSh;
          const uint32_t ns[2] = {(x << kSh) & kNibMask, (x >> (4 - kSh)) & kNibMask};
          // the eight lookups in HALVES groups, each folded before the next
          // group's reads are issued (fewer live registers)
#pragma unroll
          for (int h = 0; h < HALVES; ++h) {
            constexpr int TN = 8 / HALVES;
            uint32_t v[TN][4];
#pragma unroll
            for (int tt = 0; tt < TN; ++tt) {
              const int t = h * TN + tt;
              const uint32_t ad = __builtin_amdgcn_perm(jbase, ns[t & 1], 0x0C060500u | uint32_t(t >> 1)) +
                                  uint32_t(t * kTBytes);
              if constexpr (kWide) {
                const u32x4 q = *(lds_u32x4c*)(size_t(ad));
#pragma unroll
                for (int r = 0; r < 4; ++r) v[tt][r] = q[r];
              } else {
#pragma unroll
                for (int p = 0; p < NP; ++p) {
                  if (2 * p + 1 < L) {
                    const u32x2 q = *(lds_u32x2c*)(size_t(ad + p * kBlkBytes));
                    v[tt][2 * p] = q.x;
                    v[tt][2 * p + 1] = q.y;
                  } else {
                    v[tt][2 * p] = *(lds_u32c*)(size_t(ad + p * kBlkBytes));
                  }
                }
              }
            }
#pragma unroll
            for (int lr = 0; lr < L; ++lr) {
              uint32_t e = acc[lr + U][c];
#pragma unroll
              for (int tt = 0; tt < TN; tt += 2) e = xor3(e, v[tt][lr], v[tt + 1][lr]);
              acc[lr + U][c] = e;
            }
          }
        }
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) store16t<1>(dp[r], col, acc[r]);
  }
}


// w = 16 packed-pair kernel (gf_apply_wide_nib16) with the source chunk and
// the lookup grouping as parameters.
template <int R, int CHUNK, int GROUPS, int WPE = 1>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(WPE))) void nib16v(ApplyArgs a) {
  constexpr int EW = nib16_entry_words(R), EB = 4 * EW;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int K = a.K;
  const int n = K * kNibWords * EW;
  for (int i = threadIdx.x; i < n; i += kBlock) {
    const int pr = i % EW, e = (i / EW) % kNibWords, j = i / (EW * kNibWords);
    const bool high = (e >> 4) >= 4;
    auto word = [&](int r) -> uint32_t {
      if (r >= R) return 0u;
      const uint32_t v = a.wtab[size_t(r * K + j) * kNibWords + e];
      return high ? (v >> 16) : (v & 0xFFFFu);
    };
    reinterpret_cast<uint32_t*>(lds)[i] = word(2 * pr) | (word(2 * pr + 1) << 16);
  }
  __syncthreads();
  const kptr* sp = (const kptr*)a.src;
  uint8_t* dp[R];
#pragma unroll
  for (int r = 0; r < R; ++r) dp[r] = a.dst[a.row0 + r];
  const uint32_t lds_base = uint32_t(reinterpret_cast<uintptr_t>(static_cast<void*>(lds)));
  const int64_t nblk = (a.nvec + kBlock - 1) / kBlock;
  for (int64_t b = blockIdx.x; b < nblk; b += gridDim.x) {
    const int64_t col = b * kBlock + threadIdx.x;
    if (col >= a.nvec) continue;
    uint32_t lo[4][EW], hi[4][EW];
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int q = 0; q < EW; ++q) lo[c][q] = hi[c][q] = 0u;
    for (int j0 = 0; j0 < K; j0 += CHUNK) {
      u32x4 xs[CHUNK];
#pragma unroll
      for (int u = 0; u < CHUNK; ++u)
        if (j0 + u < K) xs[u] = load16t<1>(sp[j0 + u], col);
#pragma unroll
      for (int u = 0; u < CHUNK; ++u) {
        const int j = j0 + u;
        if (j >= K) break;
        const uint32_t jbase = lds_base + uint32_t(j) * uint32_t(nib16_source_bytes(R));
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const uint32_t x = xs[u][c];
          constexpr int kSh = EB == 8 ? 3 : 2;
          constexpr uint32_t kNibMask = 0x0F0F0F0Fu << kSh;
          const uint32_t ns[2] = {(x << kSh) & kNibMask, (x >> (4 - kSh)) & kNibMask};
#pragma unroll
          for (int g = 0; g < GROUPS; ++g) {
            constexpr int TN = 8 / GROUPS;
            uint32_t v[TN][EW];
#pragma unroll
            for (int tt = 0; tt < TN; ++tt) {
              const int t = g * TN + tt;
              const uint32_t ad = __builtin_amdgcn_perm(jbase, ns[t & 1], 0x0C060500u | uint32_t(t >> 1)) +
                                  uint32_t(t * 16 * EB);
              if constexpr (EW == 1) {
                v[tt][0] = *(lds_u32c*)(size_t(ad));
              } else {
                const u32x2 q = *(lds_u32x2c*)(size_t(ad));
                v[tt][0] = q.x;
                v[tt][1] = q.y;
              }
            }
#pragma unroll
            for (int q = 0; q < EW; ++q) {
#pragma unroll
              for (int tt = 0; tt < TN; tt += 2) {
                const int t = g * TN + tt;
                if (t < 4) lo[c][q] = xor3(lo[c][q], v[tt][q], v[tt + 1][q]);
                else hi[c][q] = xor3(hi[c][q], v[tt][q], v[tt + 1][q]);
              }
            }
          }
        }
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      u32x4 o;
#pragma unroll
      for (int c = 0; c < 4; ++c)
        o[c] = __builtin_amdgcn_perm(hi[c][r >> 1], lo[c][r >> 1], (r & 1) ? 0x07060302u : 0x05040100u);
      store16t<1>(dp[r], col, o);
    }
  }
}

// w = 16 with the unit structure of gf_apply_wide_nib<R, 1>: the launch's row
// 0 and column 0 are all ones, so row 0 is the XOR of the sources and source
// 0 is XORed into every row; the LDS holds the packed pairs of rows
// 1..R-1 (pair p = rows 1 + 2p, 2 + 2p) for sources 1..K-1 only.
template <int R, int CHUNK, int GROUPS>
__global__ __launch_bounds__(kBlock) void nib16u(ApplyArgs a) {
  constexpr int L = R - 1;
  constexpr int EW = nib16_entry_words(L), EB = 4 * EW;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int K = a.K;
  const int n = (K - 1) * kNibWords * EW;
  for (int i = threadIdx.x; i < n; i += kBlock) {
    const int pr = i % EW, e = (i / EW) % kNibWords, j = i / (EW * kNibWords) + 1;
    const bool high = (e >> 4) >= 4;
    auto word = [&](int r) -> uint32_t {
      if (r >= R) return 0u;
      const uint32_t v = a.wtab[size_t(r * K + j) * kNibWords + e];
      return high ? (v >> 16) : (v & 0xFFFFu);
    };
    reinterpret_cast<uint32_t*>(lds)[i] = word(1 + 2 * pr) | (word(2 + 2 * pr) << 16);
  }
  __syncthreads();
  const kptr* sp = (const kptr*)a.src;
  uint8_t* dp[R];
#pragma unroll
  for (int r = 0; r < R; ++r) dp[r] = a.dst[a.row0 + r];
  const uint32_t lds_base = uint32_t(reinterpret_cast<uintptr_t>(static_cast<void*>(lds)));
  const int64_t nblk = (a.nvec + kBlock - 1) / kBlock;
  for (int64_t b = blockIdx.x; b < nblk; b += gridDim.x) {
    const int64_t col = b * kBlock + threadIdx.x;
    if (col >= a.nvec) continue;
    uint32_t lo[4][EW], hi[4][EW];
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int q = 0; q < EW; ++q) lo[c][q] = hi[c][q] = 0u;
    u32x4 x0 = load16t<1>(sp[0], col);  // column 0: into every row
    u32x4 row0 = x0;                     // row 0: XOR of the sources
    for (int j0 = 1; j0 < K; j0 += CHUNK) {
      u32x4 xs[CHUNK];
#pragma unroll
      for (int u = 0; u < CHUNK; ++u)
        if (j0 + u < K) xs[u] = load16t<1>(sp[j0 + u], col);
#pragma unroll
      for (int u = 0; u < CHUNK; ++u) {
        const int j = j0 + u;
        if (j >= K) break;
        row0 ^= xs[u];
        const uint32_t jbase = lds_base + uint32_t(j - 1) * uint32_t(nib16_source_bytes(L));
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const uint32_t x = xs[u][c];
          constexpr int kSh = EB == 8 ? 3 : 2;
          constexpr uint32_t kNibMask = 0x0F0F0F0Fu << kSh;
          const uint32_t ns[2] = {(x << kSh) & kNibMask, (x >> (4 - kSh)) & kNibMask};
#pragma unroll
          for (int g = 0; g < GROUPS; ++g) {
            constexpr int TN = 8 / GROUPS;
            uint32_t v[TN][EW];
#pragma unroll
            for (int tt = 0; tt < TN; ++tt) {
              const int t = g * TN + tt;
              const uint32_t ad = __builtin_amdgcn_perm(jbase, ns[t & 1], 0x0C060500u | uint32_t(t >> 1)) +
                                  uint32_t(t * 16 * EB);
              if constexpr (EW == 1) {
                v[tt][0] = *(lds_u32c*)(size_t(ad));
              } else {
                const u32x2 q = *(lds_u32x2c*)(size_t(ad));
                v[tt][0] = q.x;
                v[tt][1] = q.y;
              }
            }
#pragma unroll
            for (int q = 0; q < EW; ++q) {
#pragma unroll
              for (int tt = 0; tt < TN; tt += 2) {
                const int t = g * TN + tt;
                if (t < 4) lo[c][q] = xor3(lo[c][q], v[tt][q], v[tt + 1][q]);
                else hi[c][q] = xor3(hi[c][q], v[tt][q], v[tt + 1][q]);
              }
            }
          }
        }
      }
    }
    store16t<1>(dp[0], col, row0);
#pragma unroll
    for (int r = 1; r < R; ++r) {
      u32x4 o;
#pragma unroll
      for (int c = 0; c < 4; ++c)
        o[c] = __builtin_amdgcn_perm(hi[c][(r - 1) >> 1], lo[c][(r - 1) >> 1], ((r - 1) & 1) ? 0x07060302u : 0x05040100u) ^
               x0[c];
      store16t<1>(dp[r], col, o);
    }
  }
}

template <int R, int U, bool B128>
constexpr unsigned split_lds(int K) {
  constexpr int L = R - U;
  constexpr bool kWide = B128 && L >= 3;
  constexpr int NP = kWide ? 1 : (L + 1) / 2;
  return unsigned(K - U) * 8u * unsigned(NP * (kWide ? 256 : 128));
}


// w = 16 RS(K,4) unit form without the persistent loop (round 4): one (or
// BPW) column block(s) per workgroup, compile-time K, the column's K source
// loads issued first, then the LDS image copied in from a packed global image
// (a.ptab: the staging loop's output, built once on the host) and the
// barrier -- the shape that put the w = 8 LDS engine at the v_perm engine's
// rate.  BPW > 1: the next block's loads go out before this block's lookups.
template <int K, int BPW>
__global__ __launch_bounds__(kBlock) void nib16_flat(ApplyArgs a) {
  constexpr int L = 3, EW = 2, EB = 8;  // rows 1..3 in two packed pairs per entry
  extern __shared__ __attribute__((aligned(16))) uint8_t nib_lds[];
  const uint8_t* const* sp = a.src;
  uint8_t* dp[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) dp[r] = a.dst[a.row0 + r];
  int64_t col = int64_t(blockIdx.x) * BPW * kBlock + threadIdx.x;
  u32x4 x[K];
#pragma unroll
  for (int j = 0; j < K; ++j) x[j] = col < a.nvec ? load16t<1>(kload(sp, j), col) : u32x4{0u, 0u, 0u, 0u};
  {
    const u32x4* img = reinterpret_cast<const u32x4*>(a.ptab);
    constexpr int n4 = (K - 1) * kNibWords * EW / 4;
    for (int i = threadIdx.x; i < n4; i += kBlock) reinterpret_cast<u32x4*>(nib_lds)[i] = img[i];
  }
  __syncthreads();
  const uint32_t lds_base = uint32_t(reinterpret_cast<uintptr_t>(static_cast<void*>(nib_lds)));
#pragma unroll
  for (int q = 0; q < BPW; ++q) {
    u32x4 xn[K];
    const int64_t ncol = col + kBlock;
    if (q + 1 < BPW) {
#pragma unroll
      for (int j = 0; j < K; ++j) xn[j] = ncol < a.nvec ? load16t<1>(kload(sp, j), ncol) : u32x4{0u, 0u, 0u, 0u};
    }
    uint32_t lo[4][EW], hi[4][EW];
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int e = 0; e < EW; ++e) lo[c][e] = hi[c][e] = 0u;
    u32x4 row0 = x[0];
#pragma unroll
    for (int j = 1; j < K; ++j) {
      row0 ^= x[j];
      const uint32_t jbase = lds_base + uint32_t(j - 1) * uint32_t(nib16_source_bytes(L));
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const uint32_t xv = x[j][c];
        constexpr int kSh = 3;
        constexpr uint32_t kNibMask = 0x0F0F0F0Fu << kSh;
        const uint32_t ns[2] = {(xv << kSh) & kNibMask, (xv >> (4 - kSh)) & kNibMask};
        uint32_t v[8][EW];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          const uint32_t ad = __builtin_amdgcn_perm(jbase, ns[t & 1], 0x0C060500u | uint32_t(t >> 1)) +
                              uint32_t(t * 16 * EB);
          const u32x2 qv = *(lds_u32x2*)(size_t(ad));
          v[t][0] = qv.x;
          v[t][1] = qv.y;
        }
#pragma unroll
        for (int e = 0; e < EW; ++e) {
          lo[c][e] = xor3(xor3(lo[c][e], v[0][e], v[1][e]), v[2][e], v[3][e]);
          hi[c][e] = xor3(xor3(hi[c][e], v[4][e], v[5][e]), v[6][e], v[7][e]);
        }
      }
    }
    if (col < a.nvec) {
      store16t<1>(dp[0], col, row0);
#pragma unroll
      for (int r = 1; r < 4; ++r) {
        const int l = r - 1;
        u32x4 o;
#pragma unroll
        for (int c = 0; c < 4; ++c)
          o[c] = __builtin_amdgcn_perm(hi[c][l >> 1], lo[c][l >> 1], (l & 1) ? 0x07060302u : 0x05040100u) ^ x[0][c];
        store16t<1>(dp[r], col, o);
      }
    }
    if (q + 1 < BPW) {
#pragma unroll
      for (int j = 0; j < K; ++j) x[j] = xn[j];
    }
    col = ncol;
  }
}
}  // namespace lab

// production's pipelined wide kernel (gf_apply_wide_pipe<K, 4, mode>) for the
// lab's K: 5, 7, 8, 10, 11, 12
const void* pipe_fn(int K, int mode) {
  auto pick = [&](auto k) -> const void* {
    constexpr int kK = decltype(k)::value;
    return mode == kPipeW16      ? reinterpret_cast<const void*>(&gf_apply_wide_pipe<kK, 4, kPipeW16>)
           : mode == kPipeW32Unit ? reinterpret_cast<const void*>(&gf_apply_wide_pipe<kK, 4, kPipeW32Unit>)
                                  : reinterpret_cast<const void*>(&gf_apply_wide_pipe<kK, 4, kPipeW32>);
  };
  switch (K) {
    case 5: return pick(std::integral_constant<int, 5>{});
    case 7: return pick(std::integral_constant<int, 7>{});
    case 8: return pick(std::integral_constant<int, 8>{});
    case 9: return pick(std::integral_constant<int, 9>{});
    case 10: return pick(std::integral_constant<int, 10>{});
    case 11: return pick(std::integral_constant<int, 11>{});
    case 12: return pick(std::integral_constant<int, 12>{});
    default: return nullptr;
  }
}

struct Variant {
  std::string name;
  const void* fn;
  unsigned lds;
  int bpcu = 0;  // > 0: grid of bpcu workgroups per CU (fewer resident than the occupancy allows)
  int flat = 0;  // > 0: a non-persistent grid of one workgroup per `flat` column blocks
};

int main(int argc, char** argv) {
  int w = 32, k = 10, m = 4, mib = 64, rounds = 7, reps = 10, skew_kib = -1;
  std::string only;
  for (int i = 1; i + 1 < argc; i += 2) {
    const std::string f = argv[i];
    if (f == "--w") w = std::atoi(argv[i + 1]);
    else if (f == "--k") k = std::atoi(argv[i + 1]);
    else if (f == "--m") m = std::atoi(argv[i + 1]);
    else if (f == "--mib") mib = std::atoi(argv[i + 1]);
    else if (f == "--rounds") rounds = std::atoi(argv[i + 1]);
    else if (f == "--reps") reps = std::atoi(argv[i + 1]);
    else if (f == "--only") only = argv[i + 1];
    else if (f == "--skew-kib") skew_kib = std::atoi(argv[i + 1]);
  }
  if (m != 4 || k < 2 || k > 16 || (w != 32 && w != 16)) {
    std::fprintf(stderr, "lab covers m = 4, 2 <= k <= 16, w = 16 / 32\n");
    return 2;
  }
  // the library's stride (shard_stride.hpp: +8 KiB at 64 MiB), or --skew-kib
  const size_t S = size_t(mib) << 20;
  const size_t stride = skew_kib >= 0 ? S + size_t(skew_kib) * 1024 : size_t(shard_stride(int64_t(S)));
  const int R = m, K = k;
  // Vandermonde coding matrix of the reference (reed_sol.cpp:63-84)
  int* M = vandermonde_coding_matrix(k, m, w);
  // per-coefficient nibble tables (ecgpu_runtime.hip build_wide_nib_tables)
  std::vector<uint32_t> wtab(size_t(R) * K * kNibWords);
  for (int r = 0; r < R; ++r)
    for (int j = 0; j < K; ++j) {
      const uint32_t c = uint32_t(M[r * k + j]);
      uint32_t* t = &wtab[(size_t(r) * K + j) * kNibWords];
      for (int tt = 0; tt < 8; ++tt)
        for (uint32_t v = 0; v < 16; ++v)
          t[tt * 16 + int(v)] = w == 32  ? gf_mul_poly(v << (4 * tt), c, 32)
                                : tt < 4 ? gf_mul_poly(v << (4 * tt), c, 16)
                                         : gf_mul_poly(v << (4 * (tt - 4)), c, 16) << 16;
    }
  bool unit_rc = true;
  for (int j = 0; j < k; ++j) unit_rc = unit_rc && M[j] == 1;
  for (int r = 0; r < m; ++r) unit_rc = unit_rc && M[r * k] == 1;

  uint8_t* slab = nullptr;
  CK(hipMalloc(&slab, stride * size_t(K + R) + 2 * stride));  // + a second output set for the checks
  {
    std::vector<uint8_t> h(S);
    std::mt19937_64 g(1234);
    for (int j = 0; j < K; ++j) {
      for (size_t i = 0; i < S; i += 8) {
        const uint64_t x = g();
        std::memcpy(&h[i], &x, std::min<size_t>(8, S - i));
      }
      CK(hipMemcpy(slab + stride * j, h.data(), S, hipMemcpyHostToDevice));
    }
  }
  std::vector<uint8_t*> hp(size_t(K + R));
  for (int i = 0; i < K + R; ++i) hp[i] = slab + stride * size_t(i);
  uint8_t** d_ptrs = nullptr;
  CK(hipMalloc(&d_ptrs, sizeof(void*) * (K + R)));
  CK(hipMemcpy(d_ptrs, hp.data(), sizeof(void*) * (K + R), hipMemcpyHostToDevice));
  uint32_t* d_wtab = nullptr;
  CK(hipMalloc(&d_wtab, wtab.size() * 4));
  CK(hipMemcpy(d_wtab, wtab.data(), wtab.size() * 4, hipMemcpyHostToDevice));

  // the w = 16 unit form's LDS image (gf_apply_wide_nib16<4, 1>'s staging
  // loop, done once here): dword ((j - 1) * kNibWords + e) * 2 + pr = rows
  // 1 + 2pr | 2 + 2pr of source j's table entry e, low or high word
  std::vector<uint32_t> img16(size_t(K > 1 ? K - 1 : 0) * kNibWords * 2);
  for (int j = 1; j < K && w == 16; ++j)
    for (int e = 0; e < kNibWords; ++e)
      for (int pr = 0; pr < 2; ++pr) {
        const bool high = (e >> 4) >= 4;
        auto word = [&](int r) -> uint32_t {
          if (r >= R) return 0u;
          const uint32_t v = wtab[size_t(r * K + j) * kNibWords + e];
          return high ? (v >> 16) : (v & 0xFFFFu);
        };
        img16[(size_t(j - 1) * kNibWords + e) * 2 + pr] = word(1 + 2 * pr) | (word(2 + 2 * pr) << 16);
      }
  uint32_t* d_img16 = nullptr;
  CK(hipMalloc(&d_img16, std::max<size_t>(16, img16.size() * 4)));
  if (!img16.empty()) CK(hipMemcpy(d_img16, img16.data(), img16.size() * 4, hipMemcpyHostToDevice));

  ApplyArgs a{};
  a.ptab = d_img16;
  a.src = d_ptrs;
  a.dst = d_ptrs + K;
  a.nvec = int64_t(S / 16);
  a.size = int64_t(S);
  a.byte0 = a.nvec * 16;
  a.src_stride = K;
  a.dst_stride = R;
  a.row0 = 0;
  a.K = K;
  a.R = R;
  a.nt = 1;
  a.wtab = d_wtab;

  std::vector<Variant> vs;
#define V(name, ...) \
  vs.push_back({name, reinterpret_cast<const void*>(&lab::nib_split<__VA_ARGS__>), lab::split_lds<4, 0, true>(K)})
#define VU(name, ...) \
  vs.push_back({name, reinterpret_cast<const void*>(&lab::nib_split<__VA_ARGS__>), lab::split_lds<4, 1, true>(K)})
  if (w == 32) {
    vs.push_back({"prod_u0", reinterpret_cast<const void*>(&gf_apply_wide_nib<4>), unsigned(nib_lds_bytes(K, 4, 0))});
    if (const void* f = pipe_fn(K, kPipeW32); f && (S / 16) % kBlock == 0)
      vs.push_back({"prod_pipe_u0", f, unsigned(nib_lds_bytes(K, 4, 0))});
    V("u0_c8", 4, 0, true, 8, 1, 1);
    V("u0_c4_h4", 4, 0, true, 4, 4, 1);
    V("u0_c4_h2", 4, 0, true, 4, 2, 1);
    if (unit_rc) {
      vs.push_back({"prod_u1", reinterpret_cast<const void*>(&gf_apply_wide_nib<4, 1>), unsigned(nib_lds_bytes(K, 4, 1))});
      for (int b : {2, 3, 4, 5})
        vs.push_back({"prod_u1_grid" + std::to_string(b), reinterpret_cast<const void*>(&gf_apply_wide_nib<4, 1>),
                      unsigned(nib_lds_bytes(K, 4, 1)), b});
      VU("u1_c10_h2", 4, 1, true, 10, 2, 1);
      VU("u1_c4_h1", 4, 1, true, 4, 1, 1);
      VU("u1_c4_h2", 4, 1, true, 4, 2, 1);
      VU("u1_c4_h4", 4, 1, true, 4, 4, 1);
      VU("u1_c5_h2_w6", 4, 1, true, 5, 2, 6);
      VU("u1_c5_h4", 4, 1, true, 5, 4, 1);
      VU("u1_c3_h2", 4, 1, true, 3, 2, 1);
      VU("u1_c2_h4", 4, 1, true, 2, 4, 1);
      if (const void* f = pipe_fn(K, kPipeW32Unit); f && (S / 16) % kBlock == 0) {
        vs.push_back({"prod_pipe", f, unsigned(nib_lds_bytes(K, 4, 1))});
        if (K == 10) {
          vs.push_back({"pipe_wpe5", reinterpret_cast<const void*>(&gf_apply_wide_pipe<10, 4, kPipeW32Unit, 5>),
                        unsigned(nib_lds_bytes(K, 4, 1))});
          vs.push_back({"pipe_wpe6", reinterpret_cast<const void*>(&gf_apply_wide_pipe<10, 4, kPipeW32Unit, 6>),
                        unsigned(nib_lds_bytes(K, 4, 1))});
        }
        // round 4: chunkings that fit 128 VGPRs (4 workgroups per CU) at K = 12
        // (6 or 8 chunks: 128 VGPRs; production's 4 chunks: 131, 3 per CU)
        if (K == 12) {
          vs.push_back({"pipe_nch6", reinterpret_cast<const void*>(&gf_apply_wide_pipe<12, 4, kPipeW32Unit, 1, 6>),
                        unsigned(nib_lds_bytes(K, 4, 1))});
          vs.push_back({"pipe_nch8", reinterpret_cast<const void*>(&gf_apply_wide_pipe<12, 4, kPipeW32Unit, 1, 8>),
                        unsigned(nib_lds_bytes(K, 4, 1))});
        }
        if (K == 11) {
          vs.push_back({"pipe_nch2", reinterpret_cast<const void*>(&gf_apply_wide_pipe<11, 4, kPipeW32Unit, 1, 2>),
                        unsigned(nib_lds_bytes(K, 4, 1))});
          vs.push_back({"pipe_nch6", reinterpret_cast<const void*>(&gf_apply_wide_pipe<11, 4, kPipeW32Unit, 1, 6>),
                        unsigned(nib_lds_bytes(K, 4, 1))});
        }
      }
    }
  } else {
    const unsigned l16 = unsigned(K * nib16_source_bytes(4));
    vs.push_back({"prod_nib16_4", reinterpret_cast<const void*>(&gf_apply_wide_nib16<4>), l16});
    vs.push_back({"n16_c8_g1", reinterpret_cast<const void*>(&lab::nib16v<4, 8, 1>), l16});
    vs.push_back({"n16_c4_g1", reinterpret_cast<const void*>(&lab::nib16v<4, 4, 1>), l16});
    vs.push_back({"n16_c4_g2", reinterpret_cast<const void*>(&lab::nib16v<4, 4, 2>), l16});
    vs.push_back({"n16_c2_g2", reinterpret_cast<const void*>(&lab::nib16v<4, 2, 2>), l16});
    vs.push_back({"n16_c5_g2", reinterpret_cast<const void*>(&lab::nib16v<4, 5, 2>), l16});
    vs.push_back({"n16_c10_g2", reinterpret_cast<const void*>(&lab::nib16v<4, 10, 2>), l16});
    vs.push_back({"n16_c4_g2_w8", reinterpret_cast<const void*>(&lab::nib16v<4, 4, 2, 8>), l16});
    for (int b : {2, 3, 4, 5})
      vs.push_back({"prod_nib16_4_grid" + std::to_string(b), reinterpret_cast<const void*>(&gf_apply_wide_nib16<4>), l16, b});
    for (int b : {2, 3, 4})
      vs.push_back({"n16_c2_g2_grid" + std::to_string(b), reinterpret_cast<const void*>(&lab::nib16v<4, 2, 2>), l16, b});
    if (const void* f = pipe_fn(K, kPipeW16); f && (S / 16) % kBlock == 0)
      for (int b : {0, 3, 4})
        vs.push_back({b ? "prod_pipe16_grid" + std::to_string(b) : "prod_pipe16", f, l16, b});
    if (unit_rc) {
      const unsigned lu = unsigned((K - 1) * nib16_source_bytes(3));
      // round 4: the unit form in production (gf_apply_wide_nib16<4, 1>, the wide16_units knob)
      for (int b : {0, 3})
        vs.push_back({std::string("prod_nib16u") + (b ? "_grid3" : ""),
                      reinterpret_cast<const void*>(&gf_apply_wide_nib16<4, 1>), lu, b});
      // round 4: non-persistent forms (lab::nib16_flat), dynamic LDS sized for 2 / 3 / 4 workgroups per CU
      if (K == 10) {
        for (int per_cu : {2, 3, 4}) {
          const unsigned dyn = std::max(lu, (unsigned(163840 / per_cu) & ~4095u) - 4096u);
          const std::string ps = "_cu" + std::to_string(per_cu);
          vs.push_back({"flat1" + ps, reinterpret_cast<const void*>(&lab::nib16_flat<10, 1>), dyn, 0, 1});
          vs.push_back({"flat2" + ps, reinterpret_cast<const void*>(&lab::nib16_flat<10, 2>), dyn, 0, 2});
        }
      }
      for (int b : {0, 2, 3, 4}) {
        const std::string gs = b ? "_grid" + std::to_string(b) : "";
        vs.push_back({"n16u_c8_g1" + gs, reinterpret_cast<const void*>(&lab::nib16u<4, 8, 1>), lu, b});
        vs.push_back({"n16u_c4_g2" + gs, reinterpret_cast<const void*>(&lab::nib16u<4, 4, 2>), lu, b});
        vs.push_back({"n16u_c3_g1" + gs, reinterpret_cast<const void*>(&lab::nib16u<4, 3, 1>), lu, b});
      }
    }
  }
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  auto grid_of = [&](const Variant& v) {
    int n = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, v.fn, kBlock, v.lds));
    if (v.bpcu > 0) n = std::min(n, v.bpcu);
    return std::max(1, n) * cus;
  };
  auto launch = [&](const Variant& v, ApplyArgs args) {
    void* kargs[] = {&args};
    const int64_t nblk = (args.nvec + kBlock - 1) / kBlock;
    const unsigned grid = v.flat > 0 ? unsigned((nblk + v.flat - 1) / v.flat) : unsigned(grid_of(v));
    CK(hipLaunchKernel(v.fn, dim3(grid, 1), dim3(kBlock), kargs, v.lds, nullptr));
  };
  // reference outputs from the production kernel, then a host spot check
  launch(vs[0], a);
  CK(hipDeviceSynchronize());
  std::vector<std::vector<uint8_t>> want(static_cast<size_t>(R), std::vector<uint8_t>(S));
  for (int r = 0; r < R; ++r) CK(hipMemcpy(want[r].data(), hp[size_t(K + r)], S, hipMemcpyDeviceToHost));
  {
    std::vector<uint32_t> col(static_cast<size_t>(K));
    std::mt19937_64 g(99);
    for (int n = 0; n < 2000; ++n) {
      const size_t off = (g() % (S / 4)) * 4;
      for (int j = 0; j < K; ++j) CK(hipMemcpy(&col[j], hp[j] + off, 4, hipMemcpyDeviceToHost));
      for (int r = 0; r < R; ++r) {
        uint32_t e = 0;
        for (int j = 0; j < K; ++j) {
          if (w == 32) {
            e ^= gf_mul_poly(col[j], uint32_t(M[r * k + j]), 32);
          } else {
            e ^= gf_mul_poly(col[j] & 0xFFFF, uint32_t(M[r * k + j]), 16) |
                 (gf_mul_poly(col[j] >> 16, uint32_t(M[r * k + j]), 16) << 16);
          }
        }
        uint32_t got;
        std::memcpy(&got, &want[r][off], 4);
        if (got != e) {
          std::fprintf(stderr, "production kernel disagrees with the host at row %d offset %zu\n", r, off);
          return 1;
        }
      }
    }
  }
  for (size_t i = 1; i < vs.size(); ++i) {
    CK(hipMemset(slab + stride * size_t(K), 0, stride * size_t(R)));
    launch(vs[i], a);
    CK(hipDeviceSynchronize());
    std::vector<uint8_t> got(S);
    for (int r = 0; r < R; ++r) {
      CK(hipMemcpy(got.data(), hp[size_t(K + r)], S, hipMemcpyDeviceToHost));
      if (got != want[r]) {
        std::fprintf(stderr, "variant %s differs at row %d\n", vs[i].name.c_str(), r);
        return 1;
      }
    }
  }
  // timing: interleaved rounds, reps launches each, median per launch
  std::vector<std::vector<float>> t(vs.size());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int rd = 0; rd < rounds; ++rd)
    for (size_t i = 0; i < vs.size(); ++i) {
      if (!only.empty() && i != 0) {  // --only a,b,c: names containing any of them
        bool hit = false;
        for (size_t p0 = 0; p0 <= only.size();) {
          const size_t p1 = std::min(only.find(',', p0), only.size());
          hit = hit || vs[i].name.find(only.substr(p0, p1 - p0)) != std::string::npos;
          p0 = p1 + 1;
        }
        if (!hit) continue;
      }
      for (int q = 0; q < 2; ++q) launch(vs[i], a);  // warm
      for (int q = 0; q < reps; ++q) {
        CK(hipEventRecord(e0, nullptr));
        launch(vs[i], a);
        CK(hipEventRecord(e1, nullptr));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        t[i].push_back(ms * 1000.f);
      }
    }
  const double bytes = double(K + R) * double(S);
  for (size_t i = 0; i < vs.size(); ++i) {
    if (t[i].empty()) continue;
    std::sort(t[i].begin(), t[i].end());
    const double med = t[i][t[i].size() / 2], mn = t[i][0];
    int n = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, vs[i].fn, kBlock, vs[i].lds));
    if (vs[i].bpcu > 0) n = std::min(n, vs[i].bpcu);
    std::printf("{\"w\": %d, \"k\": %d, \"m\": %d, \"shard_mib\": %d, \"variant\": \"%s\", \"lds\": %u, "
                "\"blocks_per_cu\": %d, \"median_us\": %.1f, \"min_us\": %.1f, \"GBps\": %.0f, \"samples\": %zu}\n",
                w, k, m, mib, vs[i].name.c_str(), vs[i].lds, n, med, mn, bytes / med / 1e3, t[i].size());
  }
  return 0;
}
