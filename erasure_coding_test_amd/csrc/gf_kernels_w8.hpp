// gf_kernels_w8.hpp -- the shared kernel vocabulary (argument blocks, cache-policy
// loads / stores, constant-address table reads) and the w = 8 kernels of the
// library: the production v_perm engine gf_apply, the one-stripe inline form,
// the LDS nibble-table engine, the generic-K and byte-tail kernels.  Included
// through gf_kernels.hpp (the overview).  The measurement-only forms (2-bit
// PERM, LDS-DMA, occupancy-8, streaming, copy) live in diag_kernels_w8.hpp,
// compiled into libecgpu_diag.so only.
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
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) u32x2 gu32x2;

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

typedef __attribute__((address_space(3))) const u32x4 lds_u32x4;

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


}  // namespace dev
}  // namespace ecgpu
