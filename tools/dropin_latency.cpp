// dropin_latency.cpp -- what a C++ caller of the reference surface sees: the
// reference client's call shapes (jerasure_matrix_encode, client_main.cpp:
// 1060; jerasure_matrix_decode with row_k_ones = 0, :2118) through
// libjerasure_amd.so on ordinary malloc'd (pageable) host buffers, timed per
// call for the BASELINE configs C1-C5 (median of reps, after warm-up).
// Two layouts: every shard its own malloc, and the client's own (data shards
// at buffer + i * chunk_size in ONE stripe buffer, coding shards malloc'd one
// by one, client_main.cpp:1619-1647).  Prints one JSON line per case.
//
//   g++ -O2 -std=c++17 tools/dropin_latency.cpp -Iinclude/dropin \
//       -Lerasure_coding_test_amd/lib -ljerasure_amd \
//       -Wl,-rpath,$PWD/erasure_coding_test_amd/lib -o /tmp/dropin_latency
//   /tmp/dropin_latency
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "jerasure.h"
#include "reed_sol.h"

namespace {

double now_us() {
  using namespace std::chrono;
  return duration<double, std::micro>(steady_clock::now().time_since_epoch()).count();
}

struct Case {
  const char* name;
  int k, m, size, reps;
};

}  // namespace

int main() {
  const Case cases[] = {{"C1 RS(4,2) 64 KiB", 4, 2, 64 << 10, 200},
                        {"C2 RS(6,3) 1 MiB", 6, 3, 1 << 20, 50},
                        {"C3 RS(10,4) 4 MiB", 10, 4, 4 << 20, 20},
                        {"C5 RS(12,4) 16 MiB", 12, 4, 16 << 20, 8}};
  for (int stripe_buffer = 0; stripe_buffer < 2; ++stripe_buffer)
  for (const Case& c : cases) {
    int* matrix = reed_sol_vandermonde_coding_matrix(c.k, c.m, 8);
    std::vector<char*> data(size_t(c.k)), coding(size_t(c.m));
    unsigned seed = 12345u;
    char* buffer = stripe_buffer ? static_cast<char*>(std::malloc(size_t(c.k) * size_t(c.size))) : nullptr;
    for (int j = 0; j < c.k; ++j) {
      char*& p = data[size_t(j)];
      p = buffer ? buffer + size_t(j) * size_t(c.size) : static_cast<char*>(std::malloc(size_t(c.size)));
      for (int i = 0; i < c.size; ++i) p[i] = char((seed = seed * 1103515245u + 12345u) >> 16);
    }
    for (auto& p : coding) p = static_cast<char*>(std::calloc(size_t(c.size), 1));
    std::vector<double> enc, dec;
    std::vector<char> saved(data[0], data[0] + c.size);
    int erasures[2] = {0, -1};
    bool ok = true;
    for (int r = 0; r < c.reps + 3; ++r) {
      double t0 = now_us();
      jerasure_matrix_encode(c.k, c.m, 8, matrix, data.data(), coding.data(), c.size);
      double t1 = now_us();
      std::memset(data[0], 0, size_t(c.size));
      double t2 = now_us();
      const int rc = jerasure_matrix_decode(c.k, c.m, 8, matrix, 0, erasures, data.data(), coding.data(), c.size);
      double t3 = now_us();
      ok = ok && rc == 0 && std::memcmp(data[0], saved.data(), size_t(c.size)) == 0;
      if (r >= 3) {
        enc.push_back(t1 - t0);
        dec.push_back(t3 - t2);
      }
    }
    std::sort(enc.begin(), enc.end());
    std::sort(dec.begin(), dec.end());
    const double e = enc[enc.size() / 2], d = dec[dec.size() / 2];
    std::printf(
        "{\"case\": \"%s\", \"buffers\": \"%s\", \"encode_us\": %.1f, \"decode0_us\": %.1f, "
        "\"encode_data_GiBps\": %.2f, \"decode_ok\": %s}\n",
        c.name, buffer ? "client stripe buffer + malloc'd coding (pageable)" : "one malloc per shard (pageable)", e, d,
        double(c.k) * c.size / (e * 1e-6) / double(1 << 30), ok ? "true" : "false");
    if (buffer)
      std::free(buffer);
    else
      for (auto* p : data) std::free(p);
    for (auto* p : coding) std::free(p);
    std::free(matrix);
  }
  return 0;
}
