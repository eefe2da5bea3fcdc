// host_harness.cpp -- drives the HOST-ONLY part of libecgpu (field tables,
// matrix construction / inversion, the decode planner, bit-matrix and
// schedule construction, the buffer contract, knobs, the CPU fallback's
// executor and bookkeeping; csrc/{gf_host,matrix_host,planner,schedule_host,
// capi_host,contract_host,knobs,cpu_fallback}.cpp) under AddressSanitizer +
// UBSan, or ThreadSanitizer with `threads` > 1 (first-use table
// initialisation races between callers).
// Built and run by tests/test_sanitizers.py.  No GPU code is linked: the one
// device entry point the host objects reference is stubbed and never called.
//
//   host_harness [threads]      exit 0 = every check passed, sanitizer clean
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "cpu_fallback.hpp"
#include "ecgpu.h"
#include "gf_host.hpp"
#include "planner.hpp"

extern "C" int ecgpu_schedule_run(int, char**, int**, int, int, int) {
  std::fprintf(stderr, "ecgpu_schedule_run: GPU entry point called from the host harness\n");
  std::abort();
}

namespace {

int failures = 0;

void expect(bool ok, const char* what, int a = 0, int b = 0) {
  if (!ok) {
    std::fprintf(stderr, "FAIL %s (%d, %d)\n", what, a, b);
    __atomic_add_fetch(&failures, 1, __ATOMIC_RELAXED);
  }
}

// Known answers from the reference.
void known_answers() {
  expect(ecgpu_galois_single_multiply(2, 0x80, 8) == 29, "mul(2,0x80)");
  expect(ecgpu_galois_single_multiply(3, 7, 8) == 9, "mul(3,7)");
  expect(ecgpu_galois_inverse(2, 8) == 142, "inverse(2)");
  expect(ecgpu_galois_single_divide(1, 147, 8) == 79, "div(1,147)");
  int* M = ecgpu_reed_sol_vandermonde_coding_matrix(10, 4, 8);
  const int row1[10] = {1, 147, 138, 73, 93, 161, 103, 58, 99, 178};
  expect(M && std::memcmp(M + 10, row1, sizeof(row1)) == 0, "RS(10,4) row 1");
  std::free(M);
}

void matrices() {
  for (int w : {8, 16, 32})
    for (int k = 2; k <= 16; ++k)
      for (int m = 1; m <= 8; ++m) {
        if (w == 8 && k + m > 256) continue;
        int* M = ecgpu_reed_sol_vandermonde_coding_matrix(k, m, w);
        expect(M != nullptr, "vandermonde", k, m);
        if (!M) continue;
        for (int j = 0; j < k; ++j) expect(M[j] == 1, "row 0 all ones", k, j);
        for (int i = 0; i < m; ++i) expect(M[i * k] == 1, "column 0 all ones", k, i);
        // the bit-matrix image and its two-erasure decoding bit-matrix
        if (w == 8 && m >= 2) {
          int* B = ecgpu_jerasure_matrix_to_bitmatrix(k, m, w, M);
          std::vector<int> erased(static_cast<size_t>(k + m), 0), dm(static_cast<size_t>(k * k * w * w)),
              ids(static_cast<size_t>(k));
          erased[0] = erased[1] = 1;
          expect(ecgpu_jerasure_make_decoding_bitmatrix(k, m, w, B, erased.data(), dm.data(), ids.data()) == 0,
                 "decoding bitmatrix", k, m);
          int** dumb = ecgpu_jerasure_dumb_bitmatrix_to_schedule(k, m, w, B);
          int** smart = ecgpu_jerasure_smart_bitmatrix_to_schedule(k, m, w, B);
          expect(dumb && smart, "schedules", k, m);
          ecgpu_jerasure_free_schedule(dumb);
          ecgpu_jerasure_free_schedule(smart);
          if (m == 2 && k <= 8) {
            int*** cache = ecgpu_jerasure_generate_schedule_cache(k, m, w, B, 1);
            expect(cache != nullptr, "schedule cache", k, m);
            expect(ecgpu_jerasure_free_schedule_cache(k, m, cache) == 0, "free schedule cache", k, m);
          }
          std::free(B);
        }
        std::free(M);
      }
}

// Every erasure pattern of RS(10,4) up to 5 erasures (5 = undecodable) and
// row_k_ones 0/1, through the fused decode planner; inversion round trips.
void decode_plans() {
  const int k = 10, m = 4, n = k + m;
  int* M = ecgpu_reed_sol_vandermonde_coding_matrix(k, m, 8);
  std::vector<int> out(static_cast<size_t>(n)), src(static_cast<size_t>(n)), coef(static_cast<size_t>(n * n));
  int patterns = 0;
  for (int mask = 1; mask < (1 << n); ++mask) {
    const int ne = __builtin_popcount(unsigned(mask));
    if (ne > m + 1) continue;
    std::vector<int> er;
    for (int i = 0; i < n; ++i)
      if (mask >> i & 1) er.push_back(i);
    er.push_back(-1);
    for (int rko = 0; rko < 2; ++rko) {
      int n_out = 0, n_src = 0;
      const int rc = ecgpu_decode_plan(k, m, 8, M, rko, er.data(), out.data(), &n_out, src.data(), &n_src,
                                       coef.data());
      expect(ne <= m ? rc == 0 : rc != 0, "decode plan rc", mask, rc);
      if (rc == 0) expect(n_out == ne && n_src <= k, "decode plan shape", n_out, n_src);
      ++patterns;
    }
  }
  expect(patterns > 2000, "pattern count", patterns);
  // inversion of every k x k survivor matrix of RS(6,3) with 3 erasures
  int* M63 = ecgpu_reed_sol_vandermonde_coding_matrix(6, 3, 8);
  std::vector<int> erased(9), dm(36), ids(6);
  for (int a = 0; a < 9; ++a)
    for (int b = a + 1; b < 9; ++b)
      for (int c = b + 1; c < 9; ++c) {
        std::fill(erased.begin(), erased.end(), 0);
        erased[size_t(a)] = erased[size_t(b)] = erased[size_t(c)] = 1;
        expect(ecgpu_jerasure_make_decoding_matrix(6, 3, 8, M63, erased.data(), dm.data(), ids.data()) == 0,
               "RS(6,3) decoding matrix", a * 100 + b * 10 + c);
      }
  std::free(M63);
  std::free(M);
}

// The buffer contract of the plan API (contract_host.cpp): random binds
// against the pairwise rule, so the sweep's sort / groups run under the
// sanitizers and concurrently.
void buffer_contract(unsigned seed) {
  for (int trial = 0; trial < 300; ++trial) {
    seed = seed * 1103515245u + 12345u;
    const int rows = 1 + int(seed >> 8) % 6, nsrc = 1 + int(seed >> 12) % 5, stripes = 1 + int(seed >> 16) % 4;
    const int64_t size = 1 + int64_t(seed >> 20) % 100;
    std::vector<uint8_t*> src(size_t(stripes * nsrc)), dst(size_t(stripes * rows));
    auto pick = [&]() {
      seed = seed * 1103515245u + 12345u;
      return reinterpret_cast<uint8_t*>(uintptr_t(1) << 20) + (seed >> 16) % 400;
    };
    for (auto& p : src) p = pick();
    for (auto& p : dst) p = pick();
    bool ok = true;  // the pairwise rule
    const int per = nsrc + rows;
    for (int i = 0; i < stripes * per && ok; ++i)
      for (int j = i + 1; j < stripes * per && ok; ++j) {
        const int si = i / per, sj = j / per, ii = i % per, jj = j % per;
        const bool wi = ii >= nsrc, wj = jj >= nsrc;
        if (!wi && !wj) continue;
        const uint8_t* p = wi ? dst[size_t(si * rows + ii - nsrc)] : src[size_t(si * nsrc + ii)];
        const uint8_t* q = wj ? dst[size_t(sj * rows + jj - nsrc)] : src[size_t(sj * nsrc + jj)];
        if (!(p < q + size && q < p + size)) continue;
        if (p == q && wi != wj && si == sj && rows <= 4) continue;
        ok = false;
      }
    const int rc = ecgpu_plan_check_buffers(rows, nsrc, stripes, const_cast<const uint8_t* const*>(src.data()),
                                            dst.data(), size);
    expect((rc == ECGPU_OK) == ok, "plan buffer contract", trial, rc);
    if (rc != ECGPU_OK) expect(std::strstr(ecgpu_last_error(), "overlap") != nullptr, "contract message", trial);
  }
}

// Knobs set and read from several threads; the split tables built once.
void knobs_and_split_tables() {
  int v = 0;
  expect(ecgpu_get_knob("ECGPU_CAP", &v) == ECGPU_OK, "get knob");
  expect(ecgpu_set_knob("ECGPU_NOT_A_KNOB", 1) == ECGPU_ERR_ARG, "unknown knob");
  expect(ecgpu_galois_create_split_w8_tables() == 0, "split tables");
  for (int x : {0, 1, 255, 0x12345678, -1})
    expect(ecgpu_galois_split_w8_multiply(x, 0x0BADF00D) == ecgpu_galois_single_multiply(x, 0x0BADF00D, 32),
           "split multiply", x);
}

// The CPU fallback's executor (cpu_fallback.cpp) against the reference's
// SEQUENTIAL semantics: random sequences of whole-region copy / XOR /
// multiply(-add) over a few buffers -- aliasing included (a destination that
// is also a source, r3 == r1) -- run op by op on one copy of the buffers, and
// planned into one fused map (LinearTracker) run by cpu_apply on another.
// Sizes straddle the executor's 64 KiB chunks and are whole w-bit words.
// Then the packet form (PacketTracker + cpu_apply_packets) the same way.
uint32_t word_at(const std::vector<uint8_t>& b, size_t i, int w) {
  uint32_t v = 0;
  std::memcpy(&v, b.data() + i * size_t(w / 8), size_t(w / 8));
  return v;
}

void set_word(std::vector<uint8_t>& b, size_t i, int w, uint32_t v) { std::memcpy(b.data() + i * size_t(w / 8), &v, size_t(w / 8)); }

void cpu_fallback_exec(unsigned seed) {
  using ecgpu::FusedOp;
  using ecgpu::LinearTracker;
  auto rnd = [&]() {
    seed = seed * 1103515245u + 12345u;
    return seed >> 8;
  };
  for (int trial = 0; trial < 72; ++trial) {
    const int w = trial % 3 == 0 ? 8 : trial % 3 == 1 ? 16 : 32;
    const int level = (trial / 3) % 3;  // scalar, AVX2, AVX-512 + GFNI (capped at the host's)
    const int nbuf = 2 + int(rnd() % 8);  // up to 9 buffers: > 4 output rows, aliased ones included
    const size_t n = size_t(w / 8) * (1 + rnd() % ((70u << 10) / unsigned(w / 8)));
    const uint32_t mask = w == 32 ? 0xFFFFFFFFu : (1u << w) - 1u;
    std::vector<std::vector<uint8_t>> seq(static_cast<size_t>(nbuf)), fused;
    for (auto& b : seq) {
      b.resize(n);
      for (auto& x : b) x = uint8_t(rnd());
    }
    fused = seq;
    LinearTracker t(w);
    std::vector<void*> id(static_cast<size_t>(nbuf));
    for (int i = 0; i < nbuf; ++i) id[size_t(i)] = fused[size_t(i)].data();
    const int nops = 1 + int(rnd() % 12);
    for (int o = 0; o < nops; ++o) {
      const int a = int(rnd() % unsigned(nbuf)), b = int(rnd() % unsigned(nbuf)), c = int(rnd() % unsigned(nbuf));
      const int kind = int(rnd() % 3);
      const size_t words = n / size_t(w / 8);
      if (kind == 0) {  // b = a
        seq[size_t(b)] = std::vector<uint8_t>(seq[size_t(a)]);
        t.copy(id[size_t(b)], id[size_t(a)]);
      } else if (kind == 1) {  // c = a ^ b
        std::vector<uint8_t> r(n);
        for (size_t i = 0; i < n; ++i) r[i] = seq[size_t(a)][i] ^ seq[size_t(b)][i];
        seq[size_t(c)] = r;
        t.xor3(id[size_t(a)], id[size_t(b)], id[size_t(c)]);
      } else {  // b (^)= k * a
        const uint32_t k = uint32_t(rnd()) & mask;
        const bool add = rnd() & 1;
        std::vector<uint8_t> r = seq[size_t(b)];
        for (size_t i = 0; i < words; ++i) {
          const uint32_t p = ecgpu::gf_mul_poly(word_at(seq[size_t(a)], i, w), k, w);
          set_word(r, i, w, add ? (word_at(r, i, w) ^ p) : p);
        }
        seq[size_t(b)] = r;
        t.mul(id[size_t(a)], int(k), id[size_t(b)], add);
      }
    }
    ecgpu::rt::cpu_apply(t.finish(), int64_t(n), level);
    for (int i = 0; i < nbuf; ++i) expect(fused[size_t(i)] == seq[size_t(i)], "cpu_apply vs sequential", trial, i);
  }
  // packets: slots x rows of ps bytes, super-packets nsp apart
  for (int trial = 0; trial < 12; ++trial) {
    const int nslots = 2 + int(rnd() % 3), nrows = 1 + int(rnd() % 4), nsp = 1 + int(rnd() % 3);
    const int64_t ps = 8 * (1 + int64_t(rnd() % 64)), spstride = ps * nrows;
    std::vector<std::vector<char>> seq(size_t(nslots), std::vector<char>(size_t(spstride * nsp)));
    for (auto& b : seq)
      for (auto& x : b) x = char(rnd());
    auto fused = seq;
    ecgpu::PacketTracker t(nslots, nrows);
    const int nops = 1 + int(rnd() % 8);
    for (int o = 0; o < nops; ++o) {
      const int ss = int(rnd() % unsigned(nslots)), sr = int(rnd() % unsigned(nrows));
      const int ds = int(rnd() % unsigned(nslots)), dr = int(rnd() % unsigned(nrows));
      const bool x = rnd() & 1;
      for (int sp = 0; sp < nsp; ++sp)
        for (int64_t i = 0; i < ps; ++i) {
          char& d = seq[size_t(ds)][size_t(sp * spstride + dr * ps + i)];
          const char s = seq[size_t(ss)][size_t(sp * spstride + sr * ps + i)];
          d = x ? char(d ^ s) : s;
        }
      if (x) t.xor_into(ds, dr, ss, sr);
      else t.copy(ds, dr, ss, sr);
    }
    std::vector<char*> ptrs;
    for (auto& b : fused) ptrs.push_back(b.data());
    ecgpu::rt::cpu_apply_packets(t.finish(), ptrs, nsp, spstride, ps, trial % 3);
    for (int i = 0; i < nslots; ++i) expect(fused[size_t(i)] == seq[size_t(i)], "cpu_apply_packets", trial, i);
  }
  // the bookkeeping, concurrently under TSan
  const int64_t before = ecgpu_fallback_count();
  ecgpu::rt::record_fallback("harness", "test");
  expect(ecgpu_fallback_count() >= before + 1, "fallback count");
  ecgpu::rt::trace_begin();
  expect(!ecgpu::rt::caller_written(), "trace begin");
  ecgpu::rt::note_caller_write();
  expect(ecgpu::rt::caller_written(), "caller write noted");
  ecgpu::rt::mark_device_lost(5);
  expect(ecgpu_device_lost(5) == 1 && ecgpu_device_lost(4) == 0, "device lost bits");
  // ordinals past 63 have their own flags; out-of-range ones are never lost
  ecgpu::rt::mark_device_lost(700);
  ecgpu::rt::mark_device_lost(-1);
  ecgpu::rt::mark_device_lost(5000);
  expect(ecgpu_device_lost(700) == 1 && ecgpu_device_lost(63) == 0 && ecgpu_device_lost(0) == 0 &&
             ecgpu_device_lost(-1) == 0 && ecgpu_device_lost(5000) == 0,
         "device lost flags per ordinal");
}

void run_all() {
  knobs_and_split_tables();
  cpu_fallback_exec(0xFA11u);
  known_answers();
  matrices();
  decode_plans();
  buffer_contract(0xEC5u);
}

}  // namespace

int main(int argc, char** argv) {
  const int threads = argc > 1 ? std::atoi(argv[1]) : 1;
  if (threads <= 1) {
    run_all();
  } else {
    // concurrent first use of the lazily built field tables and the planner
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; ++t) ts.emplace_back(run_all);
    for (auto& t : ts) t.join();
  }
  if (failures) {
    std::fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  std::printf("host harness ok (%d thread(s))\n", threads);
  return 0;
}
