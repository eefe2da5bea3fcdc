// cpu_exec.cpp -- see cpu_exec.hpp.  Host-only (g++ -O2): the SIMD paths are
// per-function target attributes chosen at run time, so the library still
// loads on a host without AVX-512 or GFNI.
#include "cpu_exec.hpp"

#include <immintrin.h>

#include <algorithm>
#include <cstring>

#include "gf_host.hpp"
#include "knobs.hpp"

#define ECGPU_TARGET_GFNI __attribute__((target("avx512f,avx512bw,gfni")))
#define ECGPU_TARGET_AVX2 __attribute__((target("avx2")))

namespace ecgpu {
namespace __attribute__((visibility("hidden"))) rt {

namespace {

// Output rows computed together per pass over the sources (4 x B
// accumulators stay in the 32 zmm registers at w = 32).
constexpr int kRows = 4;

// Bytes of every buffer per step where outputs go through temporaries (more
// than kRows rows with an output that is also a source; the per-term paths --
// w = 16 / 32 without GFNI, scalar -- always): every source block is read
// before any output block is written.
// 32 KiB: 14 RS(10,4) buffers stay in a core's L2.  A multiple of 64.
constexpr int64_t kChunk = int64_t(32) << 10;

int detected_level() {
  static const int level = [] {
    if (__builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") && __builtin_cpu_supports("gfni"))
      return 2;
    return __builtin_cpu_supports("avx2") ? 1 : 0;
  }();
  return level;
}

// GF(2^8): c*x = lo[x & 15] ^ hi[x >> 4] (the north star's nibble split)
struct Nib8 {
  uint8_t lo[16], hi[16];
};

Nib8 nib8(uint32_t c) {
  Nib8 t;
  const auto& T = gf8().mul[c & 0xFFu];
  for (int v = 0; v < 16; ++v) {
    t.lo[v] = T[v];
    t.hi[v] = T[v << 4];
  }
  return t;
}

// Per-coefficient tables of GF(2^8), built once: the affine matrix of
// y -> c * y (vgf2p8affineqb) and the nibble tables -- a call's setup then
// costs lookups, not 64-step bit scatters per coefficient (the whole fixed
// cost of a small call's execution).
struct W8Tables {
  uint64_t affine[256];
  Nib8 nib[256];
};

const W8Tables& w8_tables() {
  static const W8Tables t = [] {
    W8Tables x{};
    for (uint32_t c = 0; c < 256; ++c) {
      x.affine[c] = gf_affine_block(c, 8, 0, 0);
      x.nib[c] = nib8(c);
    }
    return x;
  }();
  return t;
}

// ================================================ AVX-512 + GFNI ====
inline __mmask64 tail_mask(int64_t n) { return n >= 64 ? ~__mmask64(0) : (__mmask64(1) << n) - 1; }

// R <= kRows rows of a w = 8 map over n bytes: K sources, A[j * R + r] the
// affine matrix of coefficient (r, j).  Each 64-byte column: every source
// loaded once, R accumulators, stores after the last source.
template <int R>
ECGPU_TARGET_GFNI void gfni8_group(const uint8_t* const* src, int K, uint8_t* const* dst, const uint64_t* A,
                                   int64_t n) {
  int64_t i = 0;
  for (; i + 64 <= n; i += 64) {
    __m512i acc[R];
#pragma GCC unroll 4
    for (int r = 0; r < R; ++r) acc[r] = _mm512_setzero_si512();
    for (int j = 0; j < K; ++j) {
      const __m512i x = _mm512_loadu_si512(src[j] + i);
      const uint64_t* a = A + size_t(j) * R;
#pragma GCC unroll 4
      for (int r = 0; r < R; ++r)
        acc[r] = _mm512_xor_si512(acc[r], _mm512_gf2p8affine_epi64_epi8(x, _mm512_set1_epi64(int64_t(a[r])), 0));
    }
#pragma GCC unroll 4
    for (int r = 0; r < R; ++r) _mm512_storeu_si512(dst[r] + i, acc[r]);
  }
  if (i < n) {
    const __mmask64 m = tail_mask(n - i);
    __m512i acc[R];
#pragma GCC unroll 4
    for (int r = 0; r < R; ++r) acc[r] = _mm512_setzero_si512();
    for (int j = 0; j < K; ++j) {
      const __m512i x = _mm512_maskz_loadu_epi8(m, src[j] + i);
      const uint64_t* a = A + size_t(j) * R;
#pragma GCC unroll 4
      for (int r = 0; r < R; ++r)
        acc[r] = _mm512_xor_si512(acc[r], _mm512_gf2p8affine_epi64_epi8(x, _mm512_set1_epi64(int64_t(a[r])), 0));
    }
#pragma GCC unroll 4
    for (int r = 0; r < R; ++r) _mm512_mask_storeu_epi8(dst[r] + i, m, acc[r]);
  }
}

// w = 16 / 32 (B = 2 / 4 bytes per word, little-endian like the reference's
// casts): output byte a of a word is XOR_b A_ab * (input byte b).  x_s = x
// with every word's bytes rotated by s puts input byte (a + s) % B at
// position a, so acc[r][a] ^= A_{a,(a+s)%B} * x_s over s, and the output
// takes acc[r][a] at the positions p % B == a.  A[((j * R + r) * B + s) * B + a].
template <int R, int B>
ECGPU_TARGET_GFNI __attribute__((always_inline)) inline void gfniw_column(const uint8_t* const* src, int K,
                                                                          uint8_t* const* dst, const uint64_t* A,
                                                                          int64_t i, __mmask64 m, const __m512i* rot,
                                                                          const uint64_t* pos) {
  __m512i acc[R][B];
#pragma GCC unroll 16
  for (int q = 0; q < R * B; ++q) acc[q / B][q % B] = _mm512_setzero_si512();
  for (int j = 0; j < K; ++j) {
    __m512i xs[B];
    xs[0] = _mm512_maskz_loadu_epi8(m, src[j] + i);
#pragma GCC unroll 4
    for (int s = 1; s < B; ++s) xs[s] = _mm512_shuffle_epi8(xs[0], rot[s]);
    const uint64_t* a = A + size_t(j) * R * B * B;
#pragma GCC unroll 64
    for (int q = 0; q < R * B * B; ++q) {
      const int r = q / (B * B), s = (q / B) % B, o = q % B;
      acc[r][o] =
          _mm512_xor_si512(acc[r][o], _mm512_gf2p8affine_epi64_epi8(xs[s], _mm512_set1_epi64(int64_t(a[q])), 0));
    }
  }
#pragma GCC unroll 4
  for (int r = 0; r < R; ++r) {
    __m512i out = acc[r][0];
#pragma GCC unroll 4
    for (int o = 1; o < B; ++o) out = _mm512_mask_blend_epi8(__mmask64(pos[o]), out, acc[r][o]);
    _mm512_mask_storeu_epi8(dst[r] + i, m, out);
  }
}

template <int R, int B>
ECGPU_TARGET_GFNI void gfniw_group(const uint8_t* const* src, int K, uint8_t* const* dst, const uint64_t* A,
                                   int64_t n) {
  alignas(64) uint8_t idx[B][64];
  uint64_t pos[B] = {};
  for (int p = 0; p < 64; ++p) {
    const int a = p % B, lane = p % 16;
    for (int s = 0; s < B; ++s) idx[s][p] = uint8_t(lane - a + (a + s) % B);
    pos[a] |= uint64_t(1) << p;
  }
  __m512i rot[B];
  for (int s = 0; s < B; ++s) rot[s] = _mm512_load_si512(idx[s]);
  int64_t i = 0;
  for (; i + 64 <= n; i += 64) gfniw_column<R, B>(src, K, dst, A, i, ~__mmask64(0), rot, pos);
  if (i < n) gfniw_column<R, B>(src, K, dst, A, i, tail_mask(n - i), rot, pos);
}

ECGPU_TARGET_GFNI void xor_into_gfni(uint8_t* acc, const uint8_t* src, int64_t n) {
  int64_t i = 0;
  for (; i + 64 <= n; i += 64)
    _mm512_storeu_si512(acc + i, _mm512_xor_si512(_mm512_loadu_si512(acc + i), _mm512_loadu_si512(src + i)));
  if (i < n) {
    const __mmask64 m = tail_mask(n - i);
    _mm512_mask_storeu_epi8(acc + i, m,
                            _mm512_xor_si512(_mm512_maskz_loadu_epi8(m, acc + i), _mm512_maskz_loadu_epi8(m, src + i)));
  }
}

using GroupFn = void (*)(const uint8_t* const*, int, uint8_t* const*, const uint64_t*, int64_t);

GroupFn gfni_group(int R, int w) {
  static const GroupFn t8[kRows] = {gfni8_group<1>, gfni8_group<2>, gfni8_group<3>, gfni8_group<4>};
  static const GroupFn t16[kRows] = {gfniw_group<1, 2>, gfniw_group<2, 2>, gfniw_group<3, 2>, gfniw_group<4, 2>};
  static const GroupFn t32[kRows] = {gfniw_group<1, 4>, gfniw_group<2, 4>, gfniw_group<3, 4>, gfniw_group<4, 4>};
  return (w == 8 ? t8 : w == 16 ? t16 : t32)[R - 1];
}

// ====================================== AVX2 / scalar (no GFNI) ====
void mul_add8_scalar(uint8_t* acc, const uint8_t* src, int64_t n, const Nib8& t) {
  for (int64_t i = 0; i < n; ++i) acc[i] ^= uint8_t(t.lo[src[i] & 15] ^ t.hi[src[i] >> 4]);
}

// R <= kRows rows of a w = 8 map on AVX2, gfni8_group's shape: per 32-byte
// column every source is loaded and split into nibbles once, R accumulators
// stay in registers, one store per row.  T[j * R + r] are coefficient (r, j)'s
// nibble tables (c = 1 and c = 0 are ordinary tables: identity and zero).
template <int R>
ECGPU_TARGET_AVX2 void avx2_group8(const uint8_t* const* src, int K, uint8_t* const* dst, const Nib8* T, int64_t n) {
  const __m256i low4 = _mm256_set1_epi8(0x0f);
  int64_t i = 0;
  for (; i + 32 <= n; i += 32) {
    __m256i acc[R];
#pragma GCC unroll 4
    for (int r = 0; r < R; ++r) acc[r] = _mm256_setzero_si256();
    for (int j = 0; j < K; ++j) {
      const __m256i x = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src[j] + i));
      const __m256i l = _mm256_and_si256(x, low4);
      const __m256i h = _mm256_and_si256(_mm256_srli_epi64(x, 4), low4);
      const Nib8* t = T + size_t(j) * R;
#pragma GCC unroll 4
      for (int r = 0; r < R; ++r) {
        const __m256i tlo = _mm256_broadcastsi128_si256(_mm_loadu_si128(reinterpret_cast<const __m128i*>(t[r].lo)));
        const __m256i thi = _mm256_broadcastsi128_si256(_mm_loadu_si128(reinterpret_cast<const __m128i*>(t[r].hi)));
        acc[r] = _mm256_xor_si256(acc[r], _mm256_xor_si256(_mm256_shuffle_epi8(tlo, l), _mm256_shuffle_epi8(thi, h)));
      }
    }
#pragma GCC unroll 4
    for (int r = 0; r < R; ++r) _mm256_storeu_si256(reinterpret_cast<__m256i*>(dst[r] + i), acc[r]);
  }
  for (; i < n; ++i) {  // the last < 32 bytes: every row's byte before any store (an output may be a source)
    uint8_t a[R] = {};
    for (int j = 0; j < K; ++j) {
      const uint8_t x = src[j][i];
      for (int r = 0; r < R; ++r) {
        const Nib8& t = T[size_t(j) * R + size_t(r)];
        a[r] ^= uint8_t(t.lo[x & 15] ^ t.hi[x >> 4]);
      }
    }
    for (int r = 0; r < R; ++r) dst[r][i] = a[r];
  }
}

using Avx2GroupFn = void (*)(const uint8_t* const*, int, uint8_t* const*, const Nib8*, int64_t);

// ================================= row groups (GFNI; AVX2 at w = 8) ====
// One group's sources (those with a non-zero coefficient in its rows) and
// their coefficients in gfni*_group's (A) or avx2_group8's (T) layout.
struct Group {
  int r0 = 0, R = 0;
  std::vector<int> js;
  std::vector<uint64_t> A;
  std::vector<Nib8> T;
};

// level 2: affine matrices; level 1 (w = 8 only): nibble tables.
std::vector<Group> plan_groups(const FusedOp& op, int level) {
  const int rows = int(op.dsts.size()), nsrc = int(op.srcs.size()), B = op.w / 8;
  const uint32_t mask = op.w == 32 ? 0xFFFFFFFFu : (uint32_t(1) << op.w) - 1u;
  std::vector<Group> groups;
  for (int r0 = 0; r0 < rows; r0 += kRows) {
    Group g;
    g.r0 = r0;
    g.R = std::min(kRows, rows - r0);
    for (int j = 0; j < nsrc; ++j) {
      bool any = false;
      for (int r = 0; r < g.R; ++r) any |= (op.coef[size_t(r0 + r) * nsrc + j] & mask) != 0;
      if (!any) continue;
      g.js.push_back(j);
      for (int r = 0; r < g.R; ++r) {
        const uint32_t c = op.coef[size_t(r0 + r) * nsrc + j] & mask;
        if (level < 2) {
          g.T.push_back(w8_tables().nib[c & 0xFFu]);
          continue;
        }
        if (op.w == 8) {
          g.A.push_back(w8_tables().affine[c]);
          continue;
        }
        for (int s = 0; s < B; ++s)
          for (int a = 0; a < B; ++a) g.A.push_back(gf_affine_block(c, op.w, a, (a + s) % B));
      }
    }
    groups.push_back(std::move(g));
  }
  return groups;
}

// Runs `g` over [off, off + n) of the sources into `dst` (R pointers, already
// offset).
void run_group(const FusedOp& op, const Group& g, int64_t off, uint8_t* const* dst, int64_t n, int level) {
  if (g.js.empty()) {
    for (int r = 0; r < g.R; ++r) std::memset(dst[r], 0, size_t(n));
    return;
  }
  const uint8_t* small[32];  // no allocation for the usual source counts
  std::vector<const uint8_t*> big;
  const uint8_t** src = small;
  if (g.js.size() > 32) {
    big.resize(g.js.size());
    src = big.data();
  }
  for (size_t i = 0; i < g.js.size(); ++i) src[i] = static_cast<const uint8_t*>(op.srcs[size_t(g.js[i])]) + off;
  const int K = int(g.js.size());
  if (level >= 2) return gfni_group(g.R, op.w)(src, K, dst, g.A.data(), n);
  static const Avx2GroupFn t8[kRows] = {avx2_group8<1>, avx2_group8<2>, avx2_group8<3>, avx2_group8<4>};
  t8[g.R - 1](src, K, dst, g.T.data(), n);
}

// Row groups of <= kRows outputs, each one pass over its sources (level 2:
// any w; level 1: w = 8).
void apply_groups(const FusedOp& op, int64_t size, int level) {
  const int rows = int(op.dsts.size());
  const std::vector<Group> groups = plan_groups(op, level);
  if (!(op.dst_is_src && rows > kRows)) {
    // direct: a group's outputs are read by no later group
    for (const Group& g : groups) {
      uint8_t* dst[kRows];
      for (int r = 0; r < g.R; ++r) dst[r] = static_cast<uint8_t*>(op.dsts[size_t(g.r0 + r)]);
      run_group(op, g, 0, dst, size, level);
    }
    return;
  }
  const int64_t chunk = std::min(size, kChunk);
  std::vector<uint8_t> tmp(size_t(rows) * size_t(chunk));
  for (int64_t a = 0; a < size; a += chunk) {
    const int64_t n = std::min(chunk, size - a);
    for (const Group& g : groups) {
      uint8_t* dst[kRows];
      for (int r = 0; r < g.R; ++r) dst[r] = tmp.data() + size_t(g.r0 + r) * size_t(chunk);
      run_group(op, g, a, dst, n, level);
    }
    for (int r = 0; r < rows; ++r)
      std::memcpy(static_cast<uint8_t*>(op.dsts[size_t(r)]) + a, tmp.data() + size_t(r) * size_t(chunk), size_t(n));
  }
}

// GF(2^16) / GF(2^32) words: c*x = XOR_t T_t[nibble t of x]
template <typename Word>
struct NibW {
  Word t[sizeof(Word) * 2][16];
};

template <typename Word>
NibW<Word> nibw(uint32_t c) {
  constexpr int w = int(sizeof(Word)) * 8;
  NibW<Word> n;
  for (int tt = 0; tt < w / 4; ++tt)
    for (uint32_t v = 0; v < 16; ++v) n.t[tt][v] = Word(gf_mul_poly(v << (4 * tt), c, w));
  return n;
}

template <typename Word>
void mul_addw(uint8_t* acc, const uint8_t* src, int64_t n, const NibW<Word>& t) {
  constexpr int nt = int(sizeof(Word)) * 2;
  for (int64_t i = 0; i + int64_t(sizeof(Word)) <= n; i += sizeof(Word)) {
    Word x, a;
    std::memcpy(&x, src + i, sizeof(Word));  // unaligned, little-endian words like the reference's casts
    std::memcpy(&a, acc + i, sizeof(Word));
    Word p = 0;
    for (int tt = 0; tt < nt; ++tt) p ^= t.t[tt][(x >> (4 * tt)) & 15u];
    a ^= p;
    std::memcpy(acc + i, &a, sizeof(Word));
  }
}

void xor_into_scalar(uint8_t* acc, const uint8_t* src, int64_t n) {
  int64_t i = 0;
  for (; i + 8 <= n; i += 8) {  // 8-byte words (the library builds at -O2, which does not vectorise)
    uint64_t a, b;
    std::memcpy(&a, acc + i, 8);
    std::memcpy(&b, src + i, 8);
    a ^= b;
    std::memcpy(acc + i, &a, 8);
  }
  for (; i < n; ++i) acc[i] ^= src[i];
}

ECGPU_TARGET_AVX2 void xor_into_avx2(uint8_t* acc, const uint8_t* src, int64_t n) {
  int64_t i = 0;
  for (; i + 32 <= n; i += 32) {
    const __m256i x = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i));
    const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(acc + i));
    _mm256_storeu_si256(reinterpret_cast<__m256i*>(acc + i), _mm256_xor_si256(a, x));
  }
  xor_into_scalar(acc + i, src + i, n - i);
}

void xor_into(uint8_t* acc, const uint8_t* src, int64_t n, int level) {
  if (level >= 2) xor_into_gfni(acc, src, n);
  else if (level == 1) xor_into_avx2(acc, src, n);
  else xor_into_scalar(acc, src, n);
}

// Per-term table of one call (coefficients 0 and 1 need none).
struct Term {
  uint32_t c = 0;
  Nib8 t8{};
  NibW<uint16_t> t16{};
  NibW<uint32_t> t32{};
};

void apply_term(uint8_t* acc, const uint8_t* src, int64_t n, const Term& t, int w, int level) {
  if (t.c == 0) return;
  if (t.c == 1) return xor_into(acc, src, n, level);
  if (w == 8) return mul_add8_scalar(acc, src, n, t.t8);  // level 0 (levels 1-2 take apply_groups)
  if (w == 16) return mul_addw<uint16_t>(acc, src, n, t.t16);
  mul_addw<uint32_t>(acc, src, n, t.t32);
}

void apply_nibbles(const FusedOp& op, int64_t size, int level) {
  const int rows = int(op.dsts.size()), nsrc = int(op.srcs.size());
  const uint32_t mask = op.w == 32 ? 0xFFFFFFFFu : (uint32_t(1) << op.w) - 1u;
  std::vector<Term> terms(op.coef.size());
  for (size_t i = 0; i < op.coef.size(); ++i) {
    Term& t = terms[i];
    t.c = op.coef[i] & mask;
    if (t.c <= 1) continue;
    if (op.w == 8) t.t8 = w8_tables().nib[t.c & 0xFFu];
    else if (op.w == 16) t.t16 = nibw<uint16_t>(t.c);
    else t.t32 = nibw<uint32_t>(t.c);
  }
  const int64_t chunk = std::min(size, kChunk);
  std::vector<uint8_t> tmp(size_t(rows) * size_t(chunk));
  for (int64_t a = 0; a < size; a += chunk) {
    const int64_t n = std::min(chunk, size - a);
    for (int r = 0; r < rows; ++r) {
      uint8_t* acc = tmp.data() + size_t(r) * size_t(chunk);
      std::memset(acc, 0, size_t(n));
      for (int j = 0; j < nsrc; ++j)
        apply_term(acc, static_cast<const uint8_t*>(op.srcs[size_t(j)]) + a, n, terms[size_t(r) * nsrc + j], op.w,
                   level);
    }
    for (int r = 0; r < rows; ++r)
      std::memcpy(static_cast<uint8_t*>(op.dsts[size_t(r)]) + a, tmp.data() + size_t(r) * size_t(chunk), size_t(n));
  }
}

}  // namespace

int cpu_simd_level() {
  const int want = knob(Knob::kCpuSimd);
  return want < 0 ? detected_level() : std::min(want, detected_level());
}

uint64_t gf_affine_block(uint32_t c, int w, int a, int b) {
  // col[j] = c * x^(8b + j): the image of input bit 8b + j
  const uint32_t mask = w == 32 ? 0xFFFFFFFFu : (uint32_t(1) << w) - 1u;
  uint32_t col = c & mask;
  for (int q = 0; q < 8 * b; ++q) col = ((col << 1) ^ ((col >> (w - 1)) & 1u ? prim_poly(w) : 0u)) & mask;
  uint64_t A = 0;
  for (int j = 0; j < 8; ++j) {
    const uint32_t out = (col >> (8 * a)) & 0xFFu;  // output byte a
    for (int i = 0; i < 8; ++i)
      if ((out >> i) & 1u) A |= uint64_t(1) << (8 * (7 - i) + j);
    col = ((col << 1) ^ ((col >> (w - 1)) & 1u ? prim_poly(w) : 0u)) & mask;
  }
  return A;
}

void cpu_apply(const FusedOp& op, int64_t size) { cpu_apply(op, size, cpu_simd_level()); }

void cpu_apply(const FusedOp& op, int64_t size, int level) {
  if (op.dsts.empty() || size <= 0) return;
  level = std::max(0, std::min(level, detected_level()));
  if (level >= 2 || (level == 1 && op.w == 8)) return apply_groups(op, size, level);
  apply_nibbles(op, size, level);
}

void cpu_apply_packets(const FusedOp& op, const std::vector<char*>& ptrs, int64_t nsp, int64_t spstride, int64_t ps) {
  cpu_apply_packets(op, ptrs, nsp, spstride, ps, cpu_simd_level());
}

void cpu_apply_packets(const FusedOp& op, const std::vector<char*>& ptrs, int64_t nsp, int64_t spstride, int64_t ps,
                       int level) {
  const int rows = int(op.dsts.size()), nsrc = int(op.srcs.size());
  if (rows == 0 || nsp <= 0 || ps <= 0) return;
  level = std::max(0, std::min(level, detected_level()));
  auto addr = [&](const void* key, int64_t sp) {
    return ptrs[size_t(PacketTracker::key_slot(key))] + sp * spstride + int64_t(PacketTracker::key_row(key)) * ps;
  };
  const int64_t chunk = std::min(ps, kChunk);
  std::vector<uint8_t> tmp(size_t(rows) * size_t(chunk));
  for (int64_t sp = 0; sp < nsp; ++sp)
    for (int64_t a = 0; a < ps; a += chunk) {
      const int64_t n = std::min(chunk, ps - a);
      for (int r = 0; r < rows; ++r) {
        uint8_t* acc = tmp.data() + size_t(r) * size_t(chunk);
        std::memset(acc, 0, size_t(n));
        for (int j = 0; j < nsrc; ++j)
          if (op.coef[size_t(r) * nsrc + j] & 1u)
            xor_into(acc, reinterpret_cast<const uint8_t*>(addr(op.srcs[size_t(j)], sp)) + a, n, level);
      }
      for (int r = 0; r < rows; ++r)
        std::memcpy(addr(op.dsts[size_t(r)], sp) + a, tmp.data() + size_t(r) * size_t(chunk), size_t(n));
    }
}

}  // namespace rt
}  // namespace ecgpu
