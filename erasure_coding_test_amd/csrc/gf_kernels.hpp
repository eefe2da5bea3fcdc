// gf_kernels.hpp -- CDNA4 (gfx950) kernels for the fused GF(2^8) matrix apply
//
//     dst[s][r][x] = XOR_j  coef[r][j] * src[s][j][x]      (GF(2^8), poly 0x11D)
//
// for every stripe s, output row r < R (<= 4 per launch) and byte x.  This
// one primitive carries jerasure_matrix_encode, _decode, _dotprod and the
// galois region ops (see planner.hpp).  It is HBM-bound integer byte work:
// no MFMA; 16-byte coalesced loads/stores; all K source columns of a lane
// are loaded before any arithmetic so a wave has K*16 B per lane in flight.
//
// Multiply engines:
//  * gf_apply<K,R,UNITS> (production, w = 8): c*x is GF(2)-linear in x, so a
//    byte splits into bit slices [0:2], [3:5], [6:7] and
//    c*x = T0[x&7] ^ T1[(x>>3)&7] ^ T2[x>>6] with Tp[e] = c*(e << 3p); one
//    v_perm_b32 looks up four bytes at once from tables held in scalar
//    registers (3 v_perm per coefficient-dword), terms fold three at a time
//    with v_bitop3 (XOR3), and unit coefficients are plain XORs from a
//    compile-time structure the host checks per launch.  K and R are
//    compile-time; gf_apply_perm_generic covers K > 16 and gf_apply_bytes
//    shard tails and misaligned pointers.
//  * gf_apply_lds<K,R> (w = 8, selectable; the bench's independent
//    self-check engine): the north star's nibble tables T_lo[x] = c*x,
//    T_hi[x] = c*(x<<4) staged in LDS, one 4-byte entry serving all R rows
//    of a nibble (2 ds_read_b32 per source byte for every row together).
//  * gf_apply_wide_nib<R> / gf_apply_wide<W,R> (w = 16 / 32) and
//    gf_xor_packets16 / gf_xor_packets (GF(2) bit-matrix / schedule coding):
//    see their sections below.
// gf_apply_perm (2-bit slices, runtime coefficient classes) and the LDS-DMA
// form are kept for the A/B probes of the diagnostic library.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ecgpu {
namespace dev {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kBlock = 256;              // 4 waves
constexpr int kMaxRows = 4;              // rows per launch
constexpr int kMaxSpecK = 16;            // K specialised at compile time
constexpr uint32_t kQ0Unit = 0x03020100u;  // PERM table word 0 of coefficient 1
constexpr uint32_t kLo2 = 0x03030303u;

struct ApplyArgs {
  const u32x4* qtab;              // [R][K] PERM tables (16 B each)
  const uint32_t* ptab;           // [R][K][kP3Words] 3-bit-slice PERM tables (production kernel)
  const uint8_t* ntab;            // [R][K][32] nibble tables (LDS engine)
  const uint8_t* const* src;      // [stripes][src_stride] device pointers
  uint8_t* const* dst;            // [stripes][dst_stride] device pointers
  int64_t nvec;                   // 16-B columns per shard in the vector part
  int64_t size;                   // bytes per shard
  int64_t byte0;                  // first byte handled by the byte kernel
  uint64_t unit_mask;             // bit r*K+j: coefficient == 1 (this launch's rows)
  uint64_t zero_mask;             // bit r*K+j: coefficient == 0
  int src_stride, dst_stride, row0;  // row0 = first dst column of this launch
  int K, R;                       // runtime copies (generic / byte kernels)
  int nt;                         // 1: non-temporal loads/stores
  int stripe_fast;                // 1: blockIdx.x = stripe, blockIdx.y = column block
  const uint32_t* wtab;           // [R][K][2 * Wide<W>::kPerms] wide-word tables (w = 16 / 32)
  const uint8_t* wcls;            // [R][K] wide coefficient class: 0 general, 1 unit, 2 zero
};

// How a launch treats coefficients 0 and 1.
enum CoefMode : int {
  kClassFromTable = 0,  // test the (s_load'ed) table word: 0 -> skip, unit -> XOR
  kClassFromMask = 1,   // test kernarg bit masks (no load on the branch path)
  kAllPerm = 2,         // no test: every coefficient through v_perm
  kXorOnly = 3,         // DIAGNOSTIC: XOR all sources, ignore coefficients
};

__device__ __forceinline__ uint32_t perm_lookup(uint32_t table, uint32_t sel) {
  // v_perm_b32: selector bytes 0..3 pick bytes of the second operand.
  return __builtin_amdgcn_perm(table, table, sel);
}

__device__ __forceinline__ uint32_t gf_mul_perm(const u32x4& q, uint32_t s0, uint32_t s1, uint32_t s2, uint32_t s3) {
  return perm_lookup(q.x, s0) ^ perm_lookup(q.y, s1) ^ perm_lookup(q.z, s2) ^ perm_lookup(q.w, s3);
}

// Shards live in global memory: address space 1 makes these global_load /
// global_store (not flat_*, which also arbitrates the LDS aperture).
typedef __attribute__((address_space(1))) u32x4 gu32x4;

__device__ __forceinline__ u32x4 load16(const uint8_t* p, int64_t col, int nt) {
  const gu32x4* a = (const gu32x4*)p + col;  // C cast: generic -> global address space
  return nt ? __builtin_nontemporal_load(a) : *a;
}

// Compile-time cache policy.  A runtime `nt ? nontemporal : plain` pair is
// merged by the compiler into ONE plain access (the two loads differ only in
// metadata), so the production kernels take the policy as a template
// argument: NT = 1 emits the `nt` bit on the global_load / global_store.
template <int NT>
__device__ __forceinline__ u32x4 load16t(const uint8_t* p, int64_t col) {
  const gu32x4* a = (const gu32x4*)p + col;
  if constexpr (NT != 0) return __builtin_nontemporal_load(a);
  else return *a;
}

// A kernel-invariant table entry (pointer tables, row masks) read through the
// constant address space: always a scalar load.  A generic load issued after
// the kernel's own vector stores must be a VECTOR load (the scalar cache is
// not coherent with vector stores), and waiting for it (vmcnt(0)) waits for
// every shard load issued before it -- in a column loop that serialised the
// K source loads of each iteration.  Valid because no table is written while
// a kernel runs.
template <class T>
__device__ __forceinline__ T kload(const T* p, int64_t i) {
  typedef __attribute__((address_space(4))) const T kT;
  return ((const kT*)p)[i];  // C cast: generic -> constant
}

// Store cache policy POL: 0 plain, 1 non-temporal (`nt`).  (Stores that
// bypass the XCD's L2 -- `sc1`, `sc0 sc1`, inline asm -- were probed in round
// 1 and were equal or slower in the bench's back-to-back launches, DESIGN.md
// §5; they live only in the diagnostic library.)
template <int POL>
__device__ __forceinline__ void store16t(uint8_t* p, int64_t col, const u32x4& v) {
  gu32x4* a = (gu32x4*)p + col;
  if constexpr (POL == 1) {
    __builtin_nontemporal_store(v, a);
  } else {
    *a = v;
  }
}

__device__ __forceinline__ void store16(uint8_t* p, int64_t col, const u32x4& v, int nt) {
  gu32x4* a = (gu32x4*)p + col;
  if (nt)
    __builtin_nontemporal_store(v, a);
  else
    *a = v;
}

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

typedef __attribute__((address_space(3))) const u32x4 lds_u32x4;

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

// ------------------------------------------------- PERM, production ----
// Unit-coefficient structure known at compile time (host checks it exactly):
//   kUnitCol0 -- coefficient (r, 0) == 1 for every row of the launch
//   kUnitRow0 -- coefficient (0, j) == 1 for every source (launch row 0)
//   kUnitAll  -- every coefficient == 1 (pure XOR, e.g. decode of one data
//                shard with the all-ones parity row)
// reed_sol_vandermonde_coding_matrix always has row 0 and column 0 all ones
// (reed_sol.cpp:324-349), so RS encode launches take kUnitCol0|kUnitRow0.
// A unit term costs one XOR and no selectors; every other term is 4 v_perm
// + 2 v_bitop3 (XOR3) per dword.
enum UnitMask : int { kUnitNone = 0, kUnitCol0 = 1, kUnitRow0 = 2, kUnitAll = 4 };

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

template <int UNITS>
__device__ __forceinline__ constexpr bool is_unit(int r, int j) {
  return (UNITS & kUnitAll) || ((UNITS & kUnitCol0) && j == 0) || ((UNITS & kUnitRow0) && r == 0);
}

__device__ __forceinline__ uint32_t mac_word(uint32_t acc, const u32x4& q, uint32_t x) {
  const uint32_t s0 = x & kLo2, s1 = (x >> 2) & kLo2, s2 = (x >> 4) & kLo2, s3 = (x >> 6) & kLo2;
  return xor3(acc, xor3(perm_lookup(q.x, s0), perm_lookup(q.y, s1), perm_lookup(q.z, s2)), perm_lookup(q.w, s3));
}

// 3-bit slices (production): v_perm picks from EIGHT bytes -- the pair
// {hi, lo} -- so a byte splits into slices [0:2], [3:5], [6:7] and
//   c*x = T0[x & 7] ^ T1[(x >> 3) & 7] ^ T2[x >> 6],  Tp[e] = c*(e << 3p),
// T0 and T1 each a dword pair, T2 one dword: 3 v_perm per coefficient-dword
// instead of 4, and 5 selector ops per source dword instead of 7.  Table
// layout per coefficient (kP3Words dwords): T0lo T0hi T1lo T1hi T2 (pad).
constexpr int kP3Words = 8;
constexpr uint32_t kLo3 = 0x07070707u;

struct Sel3 {
  uint32_t s0, s1, s2;
};

__device__ __forceinline__ Sel3 sel3(uint32_t x) { return Sel3{x & kLo3, (x >> 3) & kLo3, (x >> 6) & kLo2}; }

// c*x for one dword, from the coefficient's table t and x's selectors.
__device__ __forceinline__ uint32_t mul3(const uint32_t* __restrict__ t, const Sel3& s) {
  return xor3(__builtin_amdgcn_perm(t[1], t[0], s.s0), __builtin_amdgcn_perm(t[3], t[2], s.s1),
              __builtin_amdgcn_perm(t[4], t[4], s.s2));
}

// XOR accumulator that folds terms three at a time: v_bitop3 (XOR3) takes
// the running value plus TWO new terms, so one odd term is parked until its
// partner arrives.  N terms cost ceil(N/2) instead of N XORs (the compiler
// does not reassociate the chain itself).  `has` is a compile-time constant
// after full unrolling.
struct Xacc {
  uint32_t acc = 0u, pend = 0u;
  bool has = false;
  __device__ __forceinline__ void add(uint32_t v) {
    if (has) {
      acc = xor3(acc, pend, v);
      has = false;
    } else {
      pend = v;
      has = true;
    }
  }
  __device__ __forceinline__ uint32_t value() const { return has ? (acc ^ pend) : acc; }
};

typedef __attribute__((address_space(4))) const uint32_t kconst_u32;

__device__ __forceinline__ void mac3(Xacc& x, const kconst_u32* __restrict__ t, const Sel3& s) {
  x.add(__builtin_amdgcn_perm(t[1], t[0], s.s0));
  x.add(__builtin_amdgcn_perm(t[3], t[2], s.s1));
  x.add(__builtin_amdgcn_perm(t[4], t[4], s.s2));
}

// R output columns from the K source columns of one lane with the
// 3-bit-slice tables at `ptab` ([R][K][kP3Words], constant address space: a
// device table or the launch's own kernel arguments, see gf_apply_inl).
template <int K, int R, int UNITS>
__device__ __forceinline__ void combine3(const kconst_u32* __restrict__ ptab, const u32x4 (&x)[K], u32x4 (&acc)[R]) {
  Xacc xa[R][4];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    Sel3 sl[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) sl[c] = sel3(x[j][c]);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (is_unit<UNITS>(r, j)) {
#pragma unroll
        for (int c = 0; c < 4; ++c) xa[r][c].add(x[j][c]);
      } else {
        const kconst_u32* t = ptab + (r * K + j) * kP3Words;
#pragma unroll
        for (int c = 0; c < 4; ++c) mac3(xa[r][c], t, sl[c]);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[r][c] = xa[r][c].value();
}

// R output columns from the K source columns of one lane (combine_store:
// then R stores).  SLICES = 3: production 3-bit-slice tables (ptab); 2: the round-1 2-bit
// form (qtab), kept for A/B timing in the diagnostic library.
template <int K, int R, int UNITS, int SLICES>
__device__ __forceinline__ void combine(const ApplyArgs& a, const u32x4 (&x)[K], u32x4 (&acc)[R]) {
  if constexpr (SLICES == 3) {
    // constant address space: always a scalar load, even after an LDS-DMA
    // (which the compiler otherwise treats as a clobber)
    combine3<K, R, UNITS>((const kconst_u32*)a.ptab, x, acc);  // C cast: generic -> constant
  } else {
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
    for (int j = 0; j < K; ++j) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (is_unit<UNITS>(r, j)) {
          acc[r] ^= x[j];
        } else {
          const u32x4 q = a.qtab[r * K + j];
#pragma unroll
          for (int c = 0; c < 4; ++c) acc[r][c] = mac_word(acc[r][c], q, x[j][c]);
        }
      }
    }
  }
}

template <int K, int R, int UNITS, int SLICES, int NTS>
__device__ __forceinline__ void combine_store(const ApplyArgs& a, const u32x4 (&x)[K], uint8_t* const (&dp)[R],
                                              int64_t col) {
  u32x4 acc[R];
  combine<K, R, UNITS, SLICES>(a, x, acc);
#pragma unroll
  for (int r = 0; r < R; ++r) store16t<NTS>(dp[r], col, acc[r]);
}

// Lane l of block b handles the 16-byte columns (b*VEC + v)*256 + l, v < VEC,
// of every shard of stripe s: all K*VEC loads are issued before any
// arithmetic, then R*VEC stores.  NT: bit 0 = non-temporal loads, NT >> 1 =
// store policy of store16t (VEC == 1; the VEC > 1 probe form follows a.nt).
template <int K, int R, int UNITS, int VEC, int SLICES = 3, int NT = 3>
__device__ __forceinline__ void gf_apply_body(const ApplyArgs& a) {
  const unsigned cblk = a.stripe_fast ? blockIdx.y : blockIdx.x;
  const int s = a.stripe_fast ? blockIdx.x : blockIdx.y;
  const int64_t col0 = int64_t(cblk) * (VEC * kBlock) + threadIdx.x;
  if (col0 >= a.nvec) return;
  const uint8_t* const* sp = a.src + int64_t(s) * a.src_stride;
  // Fetch ALL pointers before the first store: a pointer read after a store
  // cannot use the scalar cache (not coherent with vector stores), and the
  // compiler then chains one dependent global load per output row.
  uint8_t* dp[R];
#pragma unroll
  for (int r = 0; r < R; ++r) dp[r] = a.dst[int64_t(s) * a.dst_stride + a.row0 + r];

  if constexpr (VEC == 1) {
    // Single column per lane (production): straight-line form, which keeps
    // the register allocation low (69 VGPRs for RS(10,4)).
    u32x4 x[K];
#pragma unroll
    for (int j = 0; j < K; ++j) x[j] = load16t<NT & 1>(sp[j], col0);
    combine_store<K, R, UNITS, SLICES, (NT >> 1)>(a, x, dp, col0);
    return;
  }

  bool live[VEC];
#pragma unroll
  for (int v = 0; v < VEC; ++v) live[v] = col0 + v * kBlock < a.nvec;
  u32x4 x[VEC][K];
#pragma unroll
  for (int v = 0; v < VEC; ++v) {
    if (!live[v]) continue;
    if (a.nt) {
#pragma unroll
      for (int j = 0; j < K; ++j) x[v][j] = load16(sp[j], col0 + v * kBlock, 1);
    } else {
#pragma unroll
      for (int j = 0; j < K; ++j) x[v][j] = load16(sp[j], col0 + v * kBlock, 0);
    }
  }

  u32x4 acc[VEC][R];
#pragma unroll
  for (int v = 0; v < VEC; ++v)
#pragma unroll
    for (int r = 0; r < R; ++r) acc[v][r] = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
  for (int j = 0; j < K; ++j) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (is_unit<UNITS>(r, j)) {
#pragma unroll
        for (int v = 0; v < VEC; ++v) acc[v][r] ^= x[v][j];
      } else {
        static_assert(SLICES == 3 || VEC == 1, "VEC > 1 uses the 3-bit-slice tables");
        const uint32_t* t = a.ptab + (r * K + j) * kP3Words;
#pragma unroll
        for (int v = 0; v < VEC; ++v)
#pragma unroll
          for (int c = 0; c < 4; ++c) acc[v][r][c] ^= mul3(t, sel3(x[v][j][c]));
      }
    }
  }

#pragma unroll
  for (int v = 0; v < VEC; ++v) {
    if (!live[v]) continue;
    if (a.nt) {
#pragma unroll
      for (int r = 0; r < R; ++r) store16(dp[r], col0 + v * kBlock, acc[v][r], 1);
    } else {
#pragma unroll
      for (int r = 0; r < R; ++r) store16(dp[r], col0 + v * kBlock, acc[v][r], 0);
    }
  }
}

// Cache policy: NT bit 0 = non-temporal loads, NT >> 1 = store policy
// (store16t: 0 plain, 1 nt).  The production
// instantiations (gf_spec.hip) all load `nt` and select the store policy per
// launch.
template <int K, int R, int UNITS, int VEC = 1, int SLICES = 3, int NT = 3>
__global__ __launch_bounds__(kBlock) void gf_apply(ApplyArgs a) {
  gf_apply_body<K, R, UNITS, VEC, SLICES, NT>(a);
}

// ---------------------------------------------- one-stripe inline form ----
// A synchronous one-stripe call (the drop-in jerasure_* / galois_* names)
// is latency-bound: uploading its pointer table and coefficient tables cost
// two to five small DMAs (~10 us each on MI355X, tools/hip_overheads.cpp)
// before the kernel could start.  Here the launch carries everything in its
// kernel arguments (< 4 KiB): the K source and R destination pointers and
// the rows' 3-bit-slice tables, read with scalar loads straight from the
// kernarg segment.  One launch covers the whole shard: blocks below
// nblk_vec do 16-B columns (the production combine, unit structure UNITS),
// the blocks after them one byte per lane for the tail [byte0, size) -- or
// every byte when a pointer is not 16-B aligned (nvec = 0).
struct InlineArgs {
  const uint8_t* src[kMaxSpecK];
  uint8_t* dst[kMaxRows];
  int64_t nvec, size, byte0;
  int nblk_vec;
  int pad_;
  uint32_t ptab[kMaxRows * kMaxSpecK * kP3Words];  // [R][K][kP3Words], this launch's rows
};
static_assert(sizeof(InlineArgs) <= 4096, "kernel arguments are limited to 4 KiB");

template <int K, int R, int UNITS>
__device__ __forceinline__ void inl_column(const uint8_t* const (&sp)[K], uint8_t* const (&dp)[R],
                                           const kconst_u32* t, int64_t col) {
  u32x4 x[K];
#pragma unroll
  for (int j = 0; j < K; ++j) x[j] = load16t<1>(sp[j], col);
  u32x4 acc[R];
  combine3<K, R, UNITS>(t, x, acc);
#pragma unroll
  for (int r = 0; r < R; ++r) store16t<1>(dp[r], col, acc[r]);
}

// ZC = false (device buffers): one 16-B column per lane, straight-line like
// gf_apply -- in a loop the compiler hoists every table load out of it,
// which overflows the SGPR file into VGPR lanes (RS(10,4): 180 v_readlane,
// 132 VGPRs; a 64 MiB encode took 271 us against gf_apply's 157).
// ZC = true (host memory read and written in place over PCIe): grid-stride
// over a capped grid -- fewer PCIe requests in flight read faster
// (tools/zero_copy_probe.cpp); PCIe-bound, so the spills do not matter there.
template <int K, int R, int UNITS, bool ZC>
__global__ __launch_bounds__(kBlock) void gf_apply_inl(InlineArgs a) {
  const kconst_u32* ptab = (const kconst_u32*)a.ptab;  // kernarg segment: scalar loads
  if (int(blockIdx.x) < a.nblk_vec) {
    // (pointers copied out by value: a reference to the kernarg struct would
    // copy all 2.2 KiB of it to scratch)
    const uint8_t* sp[K];
#pragma unroll
    for (int j = 0; j < K; ++j) sp[j] = a.src[j];
    uint8_t* dp[R];
#pragma unroll
    for (int r = 0; r < R; ++r) dp[r] = a.dst[r];
    int64_t col = int64_t(blockIdx.x) * kBlock + threadIdx.x;
    if constexpr (!ZC) {
      if (col < a.nvec) inl_column<K, R, UNITS>(sp, dp, ptab, col);
    } else {
      const int64_t step = int64_t(a.nblk_vec) * kBlock;
      for (; col < a.nvec; col += step) inl_column<K, R, UNITS>(sp, dp, ptab, col);
    }
    return;
  }
  const int64_t x = a.byte0 + int64_t(int(blockIdx.x) - a.nblk_vec) * kBlock + threadIdx.x;
  if (x >= a.size) return;
  Xacc xa[R];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const uint32_t v = a.src[j][x];
    const Sel3 sl = sel3(v);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (is_unit<UNITS>(r, j))
        xa[r].add(v);
      else
        mac3(xa[r], ptab + (r * K + j) * kP3Words, sl);
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) a.dst[r][x] = uint8_t(xa[r].value());
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

// ----------------------------------------------------------------- LDS ----
// The north star's LDS nibble-table kernel.  c*x = T_lo[x & 15] ^ T_hi[x >> 4]
// with T_lo[v] = c*v, T_hi[v] = c*(v << 4) (galois.h's multiplication
// restricted to one nibble), staged once per workgroup in LDS.  One LDS
// entry per (source j, nibble half h, nibble value v) packs the products of
// ALL R <= 4 output rows -- byte r = coef[r][j] * (v << 4h) -- so a single
// ds_read_b32 serves every row of a byte's nibble: 8 reads per source dword
// for all rows together (the round-1 form read one byte per row per nibble:
// 8 * R ds_read_u8, LDS-issue-bound at 3.7 TB/s).  Zero and unit
// coefficients are just table contents (branch-free).  The lookup address is
// the nibble times 4 extracted by one v_perm from a pre-shifted copy of the
// source dword (the table offset j*128 + 64h is the ds_read immediate); the
// lo/hi entries fold into per-byte-position accumulators with XOR3, and
// only at the end does a 4x4 byte transpose (8 v_perm per dword for R = 4)
// turn "byte position b holds all rows" into "row r holds all positions".
// A 16-entry table of 4-B entries spans 16 distinct banks: no conflicts.
typedef __attribute__((address_space(3))) const uint8_t lds_u8;
typedef __attribute__((address_space(3))) const uint32_t lds_u32;

__device__ __forceinline__ uint32_t lds_word(lds_u8* base, uint32_t byte_off) {
  return *(lds_u32*)(base + byte_off);  // C cast: byte address -> dword load (ds_read_b32)
}

template <int K, int R>
__global__ __launch_bounds__(kBlock) void gf_apply_lds(ApplyArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t lut[K * 32];  // [j][h][v]
  // The column's K loads go out before the table staging and its barrier, so
  // their HBM latency overlaps the staging (RS(10,4) encode at 3 workgroups
  // per CU 918 -> 902 us, tools/encode_lab.hip --lds).
  const int64_t col = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  const bool live = col < a.nvec;
  const int s = blockIdx.y;
  const uint8_t* const* sp = a.src + int64_t(s) * a.src_stride;
  u32x4 x[K];
#pragma unroll
  for (int j = 0; j < K; ++j) x[j] = live ? load16t<1>(sp[j], col) : u32x4{0u, 0u, 0u, 0u};
  // entry (j, h, v): byte r = coef[r][j] * (v << 4h), from the per-coefficient
  // nibble tables ntab[r][j] = {c*v (16 B), c*(v << 4) (16 B)}
  for (int i = threadIdx.x; i < K * 32; i += kBlock) {
    const int j = i >> 5, hv = i & 31;
    uint32_t e = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) e |= uint32_t(a.ntab[(r * K + j) * 32 + hv]) << (8 * r);
    lut[i] = e;
  }
  __syncthreads();
  if (!live) return;
  uint8_t* dp[R];  // all pointers before the first store (see gf_apply_body)
#pragma unroll
  for (int r = 0; r < R; ++r) dp[r] = a.dst[int64_t(s) * a.dst_stride + a.row0 + r];

  lds_u8* lb = (lds_u8*)lut;  // C cast: generic -> LDS address space
  uint32_t e[4][4];  // [dword c][byte position b]: byte r = row r's product byte
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int b = 0; b < 4; ++b) e[c][b] = 0u;
  u32x4 ux = u32x4{0u, 0u, 0u, 0u};  // XOR of the sources whose every row coefficient is 1
#pragma unroll
  for (int j = 0; j < K; ++j) {
    // a source that is a unit (or zero) in every row of the launch needs no
    // lookup: wave-uniform branches on the host's masks (decode{0} is all
    // XOR; every Vandermonde encode has column 0 all ones)
    uint64_t colbits = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) colbits |= uint64_t(1) << (r * K + j);
    if ((a.zero_mask & colbits) == colbits) continue;
    if ((a.unit_mask & colbits) == colbits) {
      ux ^= x[j];
      continue;
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const uint32_t xl = (x[j][c] & 0x0F0F0F0Fu) << 2;  // lo nibble * 4 per byte
      const uint32_t xh = (x[j][c] >> 2) & 0x3C3C3C3Cu;  // hi nibble * 4 per byte
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        // byte b alone into byte 0 (selector 0x0C = zero byte): one v_perm per address
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
    // 4x4 byte transpose: row r of dword c = byte r of e[c][0..3]
    const uint32_t p01l = __builtin_amdgcn_perm(e[c][1], e[c][0], 0x05010400u);  // E0.0 E1.0 E0.1 E1.1
    const uint32_t p23l = __builtin_amdgcn_perm(e[c][3], e[c][2], 0x05010400u);
    const uint32_t p01h = __builtin_amdgcn_perm(e[c][1], e[c][0], 0x07030602u);  // E0.2 E1.2 E0.3 E1.3
    const uint32_t p23h = __builtin_amdgcn_perm(e[c][3], e[c][2], 0x07030602u);
    acc[0][c] = __builtin_amdgcn_perm(p23l, p01l, 0x05040100u);
    if constexpr (R > 1) acc[1][c] = __builtin_amdgcn_perm(p23l, p01l, 0x07060302u);
    if constexpr (R > 2) acc[2][c] = __builtin_amdgcn_perm(p23h, p01h, 0x05040100u);
    if constexpr (R > 3) acc[3][c] = __builtin_amdgcn_perm(p23h, p01h, 0x07060302u);
  }
#pragma unroll
  for (int r = 0; r < R; ++r) store16t<1>(dp[r], col, acc[r] ^ ux);
}

// ------------------------------------------- generic K (> kMaxSpecK) ----
template <int R>
__global__ __launch_bounds__(kBlock) void gf_apply_perm_generic(ApplyArgs a) {
  const int64_t col = int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (col >= a.nvec) return;
  const int s = blockIdx.y;
  const uint8_t* const* sp = a.src + int64_t(s) * a.src_stride;
  uint8_t* dp[R];  // all pointers before the first store (see gf_apply_body)
#pragma unroll
  for (int r = 0; r < R; ++r) dp[r] = a.dst[int64_t(s) * a.dst_stride + a.row0 + r];
  u32x4 acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = u32x4{0u, 0u, 0u, 0u};
  const int K = a.K;
  int j = 0;
  for (; j + 4 <= K; j += 4) {
    u32x4 x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) x[u] = load16t<1>(sp[j + u], col);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const u32x4 v = x[u];
      const u32x4 s0 = v & kLo2, s1 = (v >> 2) & kLo2, s2 = (v >> 4) & kLo2, s3 = (v >> 6) & kLo2;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const u32x4 q = a.qtab[r * K + j + u];
        if (q.x == 0u) continue;
        if (q.x == kQ0Unit) {
          acc[r] ^= v;
          continue;
        }
        acc[r].x ^= gf_mul_perm(q, s0.x, s1.x, s2.x, s3.x);
        acc[r].y ^= gf_mul_perm(q, s0.y, s1.y, s2.y, s3.y);
        acc[r].z ^= gf_mul_perm(q, s0.z, s1.z, s2.z, s3.z);
        acc[r].w ^= gf_mul_perm(q, s0.w, s1.w, s2.w, s3.w);
      }
    }
  }
  for (; j < K; ++j) {
    const u32x4 v = load16t<1>(sp[j], col);
    const u32x4 s0 = v & kLo2, s1 = (v >> 2) & kLo2, s2 = (v >> 4) & kLo2, s3 = (v >> 6) & kLo2;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const u32x4 q = a.qtab[r * K + j];
      acc[r].x ^= gf_mul_perm(q, s0.x, s1.x, s2.x, s3.x);
      acc[r].y ^= gf_mul_perm(q, s0.y, s1.y, s2.y, s3.y);
      acc[r].z ^= gf_mul_perm(q, s0.z, s1.z, s2.z, s3.z);
      acc[r].w ^= gf_mul_perm(q, s0.w, s1.w, s2.w, s3.w);
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) store16t<1>(dp[r], col, acc[r]);
}

// --------------------------------------- bytes: tails, misaligned shards ----
// One lane per byte in [byte0, size); any K, R <= kMaxRows, any alignment.
[[maybe_unused]] static __global__ __launch_bounds__(kBlock) void gf_apply_bytes(ApplyArgs a) {
  const int64_t x = a.byte0 + int64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (x >= a.size) return;
  const int s = blockIdx.y;
  const uint8_t* const* sp = a.src + int64_t(s) * a.src_stride;
  uint8_t* const* dp = a.dst + int64_t(s) * a.dst_stride + a.row0;
  uint32_t acc[kMaxRows] = {0u, 0u, 0u, 0u};
  for (int j = 0; j < a.K; ++j) {
    const uint32_t v = sp[j][x];
    const uint32_t s0 = v & 3u, s1 = (v >> 2) & 3u, s2 = (v >> 4) & 3u, s3 = v >> 6;
    for (int r = 0; r < a.R; ++r) acc[r] ^= gf_mul_perm(a.qtab[r * a.K + j], s0, s1, s2, s3);
  }
  for (int r = 0; r < a.R; ++r) dp[r][x] = uint8_t(acc[r]);
}


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

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) u32x2 gu32x2;

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
