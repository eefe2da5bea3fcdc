// host_overhead.cpp -- the fixed host cost of a synchronous call that the
// library routes to its CPU executor (below ECGPU_MIN_OFFLOAD_KIB), split
// into its parts, on tiny shards so the arithmetic is ~0: through the
// mangled names (the unchanged callers' view), RS(10,4) encode, decode{0}
// with one pattern, decode{0,1,2,3} cycling all 210 4-of-10 data patterns
// (the read path's worst case), an ECX region multiply-add; and HIP's
// hipPointerGetAttributes on a pageable pointer (the executor needs every
// buffer proven host memory before it may touch it).  Median ns per call.
//
// Built by tools/build_tools.sh; DESIGN.md §8.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <functional>
#include <vector>

#include "galois.h"
#include "jerasure.h"
#include "reed_sol.h"

extern "C" long ecgpu_cpu_call_count(void);
extern "C" int ecgpu_set_knob(const char* name, int value);

namespace {
double median_ns(const std::function<void()>& f, int reps) {
  std::vector<double> t;
  for (int r = 0; r < reps + 20; ++r) {
    const auto a = std::chrono::steady_clock::now();
    f();
    const auto b = std::chrono::steady_clock::now();
    if (r >= 20) t.push_back(std::chrono::duration<double, std::nano>(b - a).count());
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}
}  // namespace

int main() {
  ecgpu_set_knob("ECGPU_CPU_FALLBACK", 0);
  const int k = 10, m = 4;
  int* M = reed_sol_vandermonde_coding_matrix(k, m, 8);
  for (int S : {64, 4096}) {
    std::vector<std::vector<char>> buf(k + m, std::vector<char>(size_t(S)));
    for (int i = 0; i < k; ++i)
      for (int j = 0; j < S; ++j) buf[size_t(i)][size_t(j)] = char(i * 31 + j);
    std::vector<char*> d(k), c(m);
    for (int i = 0; i < k; ++i) d[size_t(i)] = buf[size_t(i)].data();
    for (int i = 0; i < m; ++i) c[size_t(i)] = buf[size_t(k + i)].data();
    jerasure_matrix_encode(k, m, 8, M, d.data(), c.data(), S);
    std::vector<std::vector<int>> pats;
    for (int a = 0; a < 10; ++a)
      for (int b = a + 1; b < 10; ++b)
        for (int x = b + 1; x < 10; ++x)
          for (int y = x + 1; y < 10; ++y) pats.push_back({a, b, x, y, -1});
    int e0[] = {0, -1};
    size_t next = 0;
    const long calls0 = ecgpu_cpu_call_count();
    const double enc = median_ns([&] { jerasure_matrix_encode(k, m, 8, M, d.data(), c.data(), S); }, 2000);
    const double dec0 = median_ns([&] { jerasure_matrix_decode(k, m, 8, M, 0, e0, d.data(), c.data(), S); }, 2000);
    const double dec4 = median_ns(
        [&] { jerasure_matrix_decode(k, m, 8, M, 0, pats[next++ % pats.size()].data(), d.data(), c.data(), S); }, 2100);
    const double dec4_same =
        median_ns([&] { jerasure_matrix_decode(k, m, 8, M, 0, pats[7].data(), d.data(), c.data(), S); }, 2000);
    const double ecx = median_ns([&] { galois_w08_region_multiply(d[0], 0x8E, S, c[0], 1); }, 2000);
    hipPointerAttribute_t attr;
    const double attr_ns = median_ns([&] {
      (void)hipPointerGetAttributes(&attr, d[3]);
      (void)hipGetLastError();
    }, 2000);
    std::printf("{\"shard_bytes\": %d, \"encode_ns\": %.0f, \"decode0_ns\": %.0f, \"decode0123_cycling_210_ns\": %.0f, "
                "\"decode0123_same_pattern_ns\": %.0f, \"ecx_mul_add_ns\": %.0f, \"hipPointerGetAttributes_ns\": %.0f, "
                "\"cpu_calls\": %ld}\n",
                S, enc, dec0, dec4, dec4_same, ecx, attr_ns, ecgpu_cpu_call_count() - calls0);
  }
  return 0;
}
