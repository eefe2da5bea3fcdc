// cpu_fallback.cpp -- see cpu_fallback.hpp.  Host-only (g++): the CPU
// executor of a fused map and the fallback bookkeeping.
#include "cpu_fallback.hpp"

#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <mutex>

#include "ecgpu.h"
#include "gf_host.hpp"
#include "knobs.hpp"

namespace ecgpu {
namespace __attribute__((visibility("hidden"))) rt {

int fail(int code, const std::string& msg);  // capi_host.cpp

namespace {

// Bytes of every buffer processed per step (32 KiB: 14 RS(10,4) buffers stay in
// a core's L2): all sources of the step are read
// into the outputs' temporaries before any output is written, the kernel's
// per-column order.  A multiple of 4 (whole w = 16 / 32 words).
constexpr int64_t kChunk = int64_t(32) << 10;

// ---- GF(2^8): c*x = lo[x & 15] ^ hi[x >> 4] (the north star's nibble split)
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

void mul_add8_scalar(uint8_t* acc, const uint8_t* src, int64_t n, const Nib8& t) {
  for (int64_t i = 0; i < n; ++i) acc[i] ^= uint8_t(t.lo[src[i] & 15] ^ t.hi[src[i] >> 4]);
}

// 32 bytes per step: two vpshufb lookups (16-entry tables in each 128-bit
// lane) and the XORs.
__attribute__((target("avx2"))) void mul_add8_avx2(uint8_t* acc, const uint8_t* src, int64_t n, const Nib8& t) {
  const __m256i tlo = _mm256_broadcastsi128_si256(_mm_loadu_si128(reinterpret_cast<const __m128i*>(t.lo)));
  const __m256i thi = _mm256_broadcastsi128_si256(_mm_loadu_si128(reinterpret_cast<const __m128i*>(t.hi)));
  const __m256i low4 = _mm256_set1_epi8(0x0f);
  int64_t i = 0;
  for (; i + 32 <= n; i += 32) {
    const __m256i x = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i));
    const __m256i l = _mm256_and_si256(x, low4);
    const __m256i h = _mm256_and_si256(_mm256_srli_epi64(x, 4), low4);
    const __m256i p = _mm256_xor_si256(_mm256_shuffle_epi8(tlo, l), _mm256_shuffle_epi8(thi, h));
    const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(acc + i));
    _mm256_storeu_si256(reinterpret_cast<__m256i*>(acc + i), _mm256_xor_si256(a, p));
  }
  mul_add8_scalar(acc + i, src + i, n - i, t);
}

bool have_avx2() {
  static const bool yes = __builtin_cpu_supports("avx2");
  return yes;
}

// ---- GF(2^16) / GF(2^32) words: c*x = XOR_t T_t[nibble t of x]
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

__attribute__((target("avx2"))) void xor_into_avx2(uint8_t* acc, const uint8_t* src, int64_t n) {
  int64_t i = 0;
  for (; i + 32 <= n; i += 32) {
    const __m256i x = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i));
    const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(acc + i));
    _mm256_storeu_si256(reinterpret_cast<__m256i*>(acc + i), _mm256_xor_si256(a, x));
  }
  xor_into_scalar(acc + i, src + i, n - i);
}

void xor_into(uint8_t* acc, const uint8_t* src, int64_t n) {
  if (have_avx2()) xor_into_avx2(acc, src, n);
  else xor_into_scalar(acc, src, n);
}

// Per-term table of one call (coefficients 0 and 1 need none).
struct Term {
  uint32_t c = 0;
  Nib8 t8{};
  NibW<uint16_t> t16{};
  NibW<uint32_t> t32{};
};

void apply_term(uint8_t* acc, const uint8_t* src, int64_t n, const Term& t, int w) {
  if (t.c == 0) return;
  if (t.c == 1) return xor_into(acc, src, n);
  if (w == 8) return have_avx2() ? mul_add8_avx2(acc, src, n, t.t8) : mul_add8_scalar(acc, src, n, t.t8);
  if (w == 16) return mul_addw<uint16_t>(acc, src, n, t.t16);
  mul_addw<uint32_t>(acc, src, n, t.t32);
}

thread_local bool t_written = false;
std::atomic<uint64_t> g_lost{0};
std::atomic<int64_t> g_fallbacks{0};
std::once_flag g_log_once;

uint64_t device_bit(int device) { return uint64_t(1) << std::min(63, std::max(0, device)); }

}  // namespace

void cpu_apply(const FusedOp& op, int64_t size) {
  const int rows = int(op.dsts.size()), nsrc = int(op.srcs.size());
  if (rows == 0 || size <= 0) return;
  const uint32_t mask = op.w == 32 ? 0xFFFFFFFFu : (uint32_t(1) << op.w) - 1u;
  std::vector<Term> terms(op.coef.size());
  for (size_t i = 0; i < op.coef.size(); ++i) {
    Term& t = terms[i];
    t.c = op.coef[i] & mask;
    if (t.c <= 1) continue;
    if (op.w == 8) t.t8 = nib8(t.c);
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
        apply_term(acc, static_cast<const uint8_t*>(op.srcs[size_t(j)]) + a, n, terms[size_t(r) * nsrc + j], op.w);
    }
    for (int r = 0; r < rows; ++r)
      std::memcpy(static_cast<uint8_t*>(op.dsts[size_t(r)]) + a, tmp.data() + size_t(r) * size_t(chunk), size_t(n));
  }
}

void cpu_apply_packets(const FusedOp& op, const std::vector<char*>& ptrs, int64_t nsp, int64_t spstride, int64_t ps) {
  const int rows = int(op.dsts.size()), nsrc = int(op.srcs.size());
  if (rows == 0 || nsp <= 0 || ps <= 0) return;
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
            xor_into(acc, reinterpret_cast<const uint8_t*>(addr(op.srcs[size_t(j)], sp)) + a, n);
      }
      for (int r = 0; r < rows; ++r)
        std::memcpy(addr(op.dsts[size_t(r)], sp) + a, tmp.data() + size_t(r) * size_t(chunk), size_t(n));
    }
}

void trace_begin() { t_written = false; }
void note_caller_write() { t_written = true; }
bool caller_written() { return t_written; }

void mark_device_lost(int device) { g_lost.fetch_or(device_bit(device), std::memory_order_relaxed); }
bool device_lost(int device) { return (g_lost.load(std::memory_order_relaxed) & device_bit(device)) != 0; }

bool fallback_enabled() { return knob(Knob::kCpuFallback) != 0; }

int injected_failure(int device, int stage) {
  const int v = knob(Knob::kTestInjectHip);
  if (v <= 0) return ECGPU_OK;
  if ((v == 1 || v == 2) && stage == 0) {
    if (v == 2) mark_device_lost(device);
    return fail(ECGPU_ERR_HIP, "injected HIP failure before the first launch (ECGPU_TEST_INJECT_HIP=" +
                                   std::to_string(v) + ")");
  }
  if (v == 3 && stage == 1)
    return fail(ECGPU_ERR_HIP, "injected HIP failure after caller memory was written (ECGPU_TEST_INJECT_HIP=3)");
  return ECGPU_OK;
}

void record_fallback(const char* call, const std::string& why) {
  g_fallbacks.fetch_add(1, std::memory_order_relaxed);
  std::call_once(g_log_once, [&] {
    std::fprintf(stderr,
                 "libecgpu: %s: %s -- completed on the CPU (ECGPU_CPU_FALLBACK=1); later fallbacks are counted "
                 "(ecgpu_fallback_count), not printed\n",
                 call ? call : "ecgpu", why.c_str());
  });
}

int64_t fallback_count() { return g_fallbacks.load(std::memory_order_relaxed); }

}  // namespace rt
}  // namespace ecgpu

extern "C" {
ECGPU_API int64_t ecgpu_fallback_count(void) { return ecgpu::rt::fallback_count(); }
ECGPU_API int ecgpu_device_lost(int device) { return ecgpu::rt::device_lost(device) ? 1 : 0; }
}
