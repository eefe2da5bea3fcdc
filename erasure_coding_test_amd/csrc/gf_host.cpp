// gf_host.cpp -- host GF(2^w) arithmetic; see gf_host.hpp.
#include "gf_host.hpp"

#include <cstdio>
#include <cstdlib>
#include <atomic>
#include <mutex>
#include <new>
#include <vector>

namespace ecgpu {

namespace {

// Primitive polynomials, low bits (the x^w term is implicit for reduction).
// Field definitions identical to galois.cpp:48-81.
constexpr uint32_t kPoly[33] = {
    0x0,       0x1,       0x7,       0xb,        0x13,       0x25,       0x43,       0x89,      0x11d,
    0x211,     0x409,     0x805,     0x1053,     0x201b,     0x4443,     0x8003,     0x1100b,   0x20009,
    0x40081,   0x80027,   0x100009,  0x200005,   0x400003,   0x800021,   0x1000087,  0x2000009, 0x4000047,
    0x8000027, 0x10000009, 0x20000005, 0x40800007, 0x80000009, 0x400007};

inline uint32_t field_mask(int w) { return w >= 32 ? 0xFFFFFFFFu : ((1u << w) - 1u); }

Gf8Tables* g_gf8 = nullptr;
std::once_flag g_gf8_once;

void build_gf8() {
  auto* t = new Gf8Tables();
  uint32_t b = 1;
  for (int j = 0; j < 256; ++j) t->log[j] = 255;
  for (int j = 0; j < 255; ++j) {
    t->exp[j] = static_cast<uint8_t>(b);
    t->log[b] = static_cast<int16_t>(j);
    b = gf_mul_poly(b, 2, 8);
  }
  for (int a = 0; a < 256; ++a)
    for (int c = 0; c < 256; ++c)
      t->mul[a][c] = (a && c) ? t->exp[(t->log[a] + t->log[c]) % 255] : 0;
  t->inv[0] = 0;
  for (int a = 1; a < 256; ++a) t->inv[a] = t->exp[(255 - t->log[a]) % 255];
  g_gf8 = t;
}

// Lazily built reference-layout tables, one set per w.  Never freed: the
// reference hands out raw pointers with process lifetime (galois.h:53-56).
struct WTables {
  int* log = nullptr;
  int* ilog = nullptr;  // offset pointer
  int* mult = nullptr;
  int* div = nullptr;
};
WTables g_wt[33];
std::mutex g_wt_mu;

int build_log_locked(int w) {
  if (w < 1 || w > 30) return -1;
  WTables& t = g_wt[w];
  if (t.log) return 0;
  const uint32_t nw = 1u << w, nwm1 = nw - 1;
  int* lg = static_cast<int*>(std::malloc(sizeof(int) * nw));
  int* il = static_cast<int*>(std::calloc(size_t(nw) * 3, sizeof(int)));
  if (!lg || !il) {
    std::free(lg);
    std::free(il);
    return -1;
  }
  for (uint32_t j = 0; j < nw; ++j) lg[j] = static_cast<int>(nwm1);
  uint32_t b = 1;
  for (uint32_t j = 0; j < nwm1; ++j) {
    lg[b] = static_cast<int>(j);
    il[j] = static_cast<int>(b);
    b = gf_mul_poly(b, 2, w);
  }
  for (uint32_t j = 0; j < nwm1; ++j) {
    il[j + nwm1] = il[j];
    il[j + 2 * nwm1] = il[j];
  }
  t.ilog = il + nwm1;
  t.log = lg;
  return 0;
}

int build_mult_locked(int w) {
  if (w < 1 || w >= 14) return -1;
  WTables& t = g_wt[w];
  if (t.mult) return 0;
  if (build_log_locked(w) < 0) return -1;
  const uint32_t nw = 1u << w;
  int* mu = static_cast<int*>(std::malloc(sizeof(int) * nw * nw));
  int* dv = static_cast<int*>(std::malloc(sizeof(int) * nw * nw));
  if (!mu || !dv) {
    std::free(mu);
    std::free(dv);
    return -1;
  }
  for (uint32_t x = 0; x < nw; ++x)
    for (uint32_t y = 0; y < nw; ++y) {
      const size_t idx = (size_t(x) << w) | y;
      if (x == 0 || y == 0) {
        mu[idx] = 0;
        dv[idx] = (y == 0) ? -1 : 0;
      } else {
        mu[idx] = t.ilog[t.log[x] + t.log[y]];
        dv[idx] = t.ilog[t.log[x] - t.log[y]];
      }
    }
  t.div = dv;
  t.mult = mu;
  return 0;
}

}  // namespace

uint32_t prim_poly(int w) { return (w >= 0 && w <= 32) ? kPoly[w] : 0; }

uint32_t gf_mul_poly(uint32_t a, uint32_t b, int w) {
  if (w <= 0 || w > 32) return 0;
  const uint32_t mask = field_mask(w);
  a &= mask;
  b &= mask;
  // Shift-and-add with reduction after each doubling: the product of b by
  // x^i is kept reduced, exactly the field multiply of galois.cpp:292-320.
  uint32_t acc = 0, cur = b;
  const uint32_t top = 1u << (w - 1);
  const uint32_t poly = kPoly[w] & mask;
  for (int i = 0; i < w; ++i) {
    if ((a >> i) & 1u) acc ^= cur;
    const bool carry = (cur & top) != 0;
    cur = (cur << 1) & mask;
    if (carry) cur ^= poly;
  }
  return acc;
}

const Gf8Tables& gf8() {
  std::call_once(g_gf8_once, build_gf8);
  return *g_gf8;
}

int single_multiply(int a, int b, int w) {
  if (a == 0 || b == 0) return 0;
  if (w == 8) return gf8().mul[a & 0xFF][b & 0xFF];
  return static_cast<int>(gf_mul_poly(static_cast<uint32_t>(a), static_cast<uint32_t>(b), w));
}

int shift_multiply(int a, int b, int w) {
  return static_cast<int>(gf_mul_poly(static_cast<uint32_t>(a), static_cast<uint32_t>(b), w));
}

int shift_inverse(int a, int w) {
  // a^(2^w - 2) by square-and-multiply.
  const uint32_t x = static_cast<uint32_t>(a) & field_mask(w);
  if (x == 0) return 0;
  uint32_t result = 1, base = x;
  uint64_t e = (w >= 32 ? 0xFFFFFFFFull : ((1ull << w) - 1)) - 1;
  while (e) {
    if (e & 1) result = gf_mul_poly(result, base, w);
    base = gf_mul_poly(base, base, w);
    e >>= 1;
  }
  return static_cast<int>(result);
}

int inverse(int a, int w) {
  if (a == 0) return -1;
  if (w == 8) return gf8().inv[a & 0xFF];
  return shift_inverse(a, w);
}

int single_divide(int a, int b, int w) {
  if (b == 0) return -1;
  if (a == 0) return 0;
  return single_multiply(a, inverse(b, w), w);
}

int create_log_tables(int w) {
  std::lock_guard<std::mutex> lk(g_wt_mu);
  return build_log_locked(w);
}

int create_mult_tables(int w) {
  std::lock_guard<std::mutex> lk(g_wt_mu);
  return build_mult_locked(w);
}

int* mult_table(int w) {
  std::lock_guard<std::mutex> lk(g_wt_mu);
  return build_mult_locked(w) < 0 ? nullptr : g_wt[w].mult;
}

int* div_table(int w) {
  std::lock_guard<std::mutex> lk(g_wt_mu);
  return build_mult_locked(w) < 0 ? nullptr : g_wt[w].div;
}

int* log_table(int w) {
  std::lock_guard<std::mutex> lk(g_wt_mu);
  return build_log_locked(w) < 0 ? nullptr : g_wt[w].log;
}

int* ilog_table(int w) {
  std::lock_guard<std::mutex> lk(g_wt_mu);
  return build_log_locked(w) < 0 ? nullptr : g_wt[w].ilog;
}

namespace {
// split_w8[i + j][(a << 8) | b] = (a << 8i) * (b << 8j) in GF(2^32), for the
// byte-position pairs the reference fills (i = 0: j = 0..3; i = 3: j = 1..3),
// galois.cpp:756-789.  One allocation, built once, read-only afterwards.
std::once_flag g_split_once;
std::vector<int> g_split;  // 7 x 65536
std::atomic<int> g_split_rc{-1};  // 0 once built (release), read with acquire
}  // namespace

int create_split_w8_tables() {
  std::call_once(g_split_once, [] {
    try {
      g_split.assign(size_t(7) << 16, 0);
    } catch (const std::bad_alloc&) {
      return;  // g_split_rc stays -1, like the reference's failed malloc
    }
    for (int i = 0; i < 4; i += 3)
      for (int j = i == 0 ? 0 : 1; j < 4; ++j) {
        int* t = &g_split[size_t(i + j) << 16];
        for (int a = 0; a < 256; ++a)
          for (int b = 0; b < 256; ++b) t[(a << 8) | b] =
              shift_multiply(int(uint32_t(a) << (8 * i)), int(uint32_t(b) << (8 * j)), 32);
      }
    g_split_rc.store(0, std::memory_order_release);
  });
  return g_split_rc.load(std::memory_order_acquire);
}

int split_w8_multiply(int x, int y) {
  // galois.cpp:791-809: byte i of x times byte j of y from table i + j
  if (g_split_rc.load(std::memory_order_acquire) != 0) return shift_multiply(x, y, 32);
  const uint32_t ux = uint32_t(x), uy = uint32_t(y);
  int acc = 0;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j)
      acc ^= g_split[(size_t(i + j) << 16) | (((ux >> (8 * i)) & 255u) << 8) | ((uy >> (8 * j)) & 255u)];
  return acc;
}

}  // namespace ecgpu
