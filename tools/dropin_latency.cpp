// dropin_latency.cpp -- what a C++ caller of the reference surface sees:
// the reference's own call shapes through libjerasure_amd.so on ordinary
// malloc'd (pageable) host buffers, timed per call (median of reps after
// warm-up).  One JSON line per case.
//
//  * client encode / decode{0} (jerasure_matrix_encode, client_main.cpp:1060;
//    jerasure_matrix_decode with row_k_ones = 0, :2118) for the reference's
//    default operating point RS(3,3) with 1 MiB chunks (ych_ec_test.h:5-10)
//    and BASELINE configs C1-C5, in two layouts: every shard its own malloc,
//    and the client's own (data shards at buffer + i * chunk_size in ONE
//    stripe buffer, coding shards malloc'd one by one, client_main.cpp:
//    1619-1647);
//  * C4: decode of erasures {0,1,2,3} at 4 MiB, and decode calls that each
//    meet a NEW erasure pattern (4 KiB shards, cycling through all 210
//    4-of-10 data patterns, so every call plans, inverts and uploads afresh);
//  * the unchanged ECX datanode's per-block sequence (ecx_datanode_main.cpp:
//    699-735): for each arriving block, m separate memcpy /
//    galois_region_xor / galois_w08_region_multiply calls into the m
//    accumulators, blocks of chunk / EC_N = 349,525 B (client_main.cpp:
//    1450-1451), accumulators block_size + sizeof(long) (ecx:684).
//
// Built by tools/build_tools.sh (g++ -O2 against include/dropin and
// erasure_coding_test_amd/lib/libjerasure_amd.so, rpath relative to tools/).
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "galois.h"
#include "jerasure.h"
#include "reed_sol.h"

// libecgpu.so (include/ecgpu.h): no timed call may have completed on the CPU
// fallback; the tool turns it off and reports the count.  Every
// case runs twice: mode "gpu" (ECGPU_MIN_OFFLOAD_KIB=0, every call on the
// MI355X) and mode "lib" (the library's defaults: calls below the measured
// crossover on its CPU executor, counted in "cpu_calls").
extern "C" long ecgpu_fallback_count(void);
extern "C" long ecgpu_cpu_call_count(void);
extern "C" int ecgpu_set_knob(const char* name, int value);
extern "C" int ecgpu_reset_knob(const char* name);

namespace {

const char* g_mode = "lib";

// "mode" and this case's CPU-executor calls, spliced before a line's closing brace
long g_cpu0 = 0;
void begin_case() { g_cpu0 = ecgpu_cpu_call_count(); }
void end_line(const char* json) {
  std::string s(json);
  while (!s.empty() && (s.back() == '\n' || s.back() == '}')) s.pop_back();
  std::printf("%s, \"mode\": \"%s\", \"cpu_calls\": %ld}\n", s.c_str(), g_mode, ecgpu_cpu_call_count() - g_cpu0);
  std::fflush(stdout);
}

double now_us() {
  using namespace std::chrono;
  return duration<double, std::micro>(steady_clock::now().time_since_epoch()).count();
}

double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

void fill(char* p, size_t n, unsigned seed) {
  for (size_t i = 0; i < n; ++i) p[i] = char((seed = seed * 1103515245u + 12345u) >> 16);
}

struct Case {
  const char* name;
  int k, m, size, reps;
};

void client_case(const Case& c, bool stripe_buffer, const int* erased, int n_erased) {
  begin_case();
  int* matrix = reed_sol_vandermonde_coding_matrix(c.k, c.m, 8);
  std::vector<char*> data(size_t(c.k)), coding(size_t(c.m));
  char* buffer = stripe_buffer ? static_cast<char*>(std::malloc(size_t(c.k) * size_t(c.size))) : nullptr;
  for (int j = 0; j < c.k; ++j) {
    data[size_t(j)] = buffer ? buffer + size_t(j) * size_t(c.size) : static_cast<char*>(std::malloc(size_t(c.size)));
    fill(data[size_t(j)], size_t(c.size), 12345u + unsigned(j));
  }
  for (auto& p : coding) p = static_cast<char*>(std::calloc(size_t(c.size), 1));
  std::vector<std::vector<char>> saved;
  for (int e = 0; e < n_erased; ++e) saved.emplace_back(data[size_t(erased[e])], data[size_t(erased[e])] + c.size);
  std::vector<int> erasures(erased, erased + n_erased);
  erasures.push_back(-1);
  std::vector<double> enc, dec;
  bool ok = true;
  for (int r = 0; r < c.reps + 3; ++r) {
    double t0 = now_us();
    jerasure_matrix_encode(c.k, c.m, 8, matrix, data.data(), coding.data(), c.size);
    double t1 = now_us();
    for (int e = 0; e < n_erased; ++e) std::memset(data[size_t(erased[e])], 0, size_t(c.size));
    double t2 = now_us();
    const int rc =
        jerasure_matrix_decode(c.k, c.m, 8, matrix, 0, erasures.data(), data.data(), coding.data(), c.size);
    double t3 = now_us();
    ok = ok && rc == 0;
    for (int e = 0; e < n_erased; ++e)
      ok = ok && std::memcmp(data[size_t(erased[e])], saved[size_t(e)].data(), size_t(c.size)) == 0;
    if (r >= 3) {
      enc.push_back(t1 - t0);
      dec.push_back(t3 - t2);
    }
  }
  const double e = median(enc), d = median(dec);
  std::string er;
  char line[1024];
  for (int i = 0; i < n_erased; ++i) er += (i ? "," : "") + std::to_string(erased[i]);
  std::snprintf(line, sizeof line,
      "{\"case\": \"%s\", \"buffers\": \"%s\", \"encode_us\": %.1f, \"decode_us\": %.1f, \"erasures\": [%s], "
      "\"encode_data_GiBps\": %.2f, \"decode_data_GiBps\": %.2f, \"decode_ok\": %s}\n",
      c.name, buffer ? "client stripe buffer + malloc'd coding (pageable)" : "one malloc per shard (pageable)", e, d,
      er.c_str(), double(c.k) * c.size / (e * 1e-6) / double(1 << 30), double(c.k) * c.size / (d * 1e-6) / double(1 << 30),
      ok ? "true" : "false");
  end_line(line);
  if (buffer)
    std::free(buffer);
  else
    for (auto* p : data) std::free(p);
  for (auto* p : coding) std::free(p);
  std::free(matrix);
}

// Every call decodes a pattern the previous 209 calls did not use.
void new_pattern_case(int size) {
  begin_case();
  const int k = 10, m = 4;
  int* matrix = reed_sol_vandermonde_coding_matrix(k, m, 8);
  std::vector<char*> data(static_cast<size_t>(k)), coding(static_cast<size_t>(m));
  for (int j = 0; j < k; ++j) {
    data[size_t(j)] = static_cast<char*>(std::malloc(size_t(size)));
    fill(data[size_t(j)], size_t(size), 777u + unsigned(j));
  }
  for (auto& p : coding) p = static_cast<char*>(std::calloc(size_t(size), 1));
  jerasure_matrix_encode(k, m, 8, matrix, data.data(), coding.data(), size);
  std::vector<std::vector<char>> orig;
  for (int j = 0; j < k; ++j) orig.emplace_back(data[size_t(j)], data[size_t(j)] + size);
  std::vector<std::vector<int>> patterns;
  for (int a = 0; a < k; ++a)
    for (int b = a + 1; b < k; ++b)
      for (int c = b + 1; c < k; ++c)
        for (int d = c + 1; d < k; ++d) patterns.push_back({a, b, c, d, -1});
  std::vector<double> t;
  bool ok = true;
  for (int pass = 0; pass < 2; ++pass)
    for (auto& p : patterns) {
      for (int i = 0; i < 4; ++i) std::memset(data[size_t(p[size_t(i)])], 0, size_t(size));
      const double t0 = now_us();
      const int rc = jerasure_matrix_decode(k, m, 8, matrix, 0, p.data(), data.data(), coding.data(), size);
      const double t1 = now_us();
      ok = ok && rc == 0;
      for (int i = 0; i < 4; ++i)
        ok = ok && std::memcmp(data[size_t(p[size_t(i)])], orig[size_t(p[size_t(i)])].data(), size_t(size)) == 0;
      if (pass == 1) t.push_back(t1 - t0);
    }
  char line[1024];
  std::snprintf(line, sizeof line,
      "{\"case\": \"C4 new erasure pattern per call\", \"workload\": \"RS(10,4) decode, %d-byte pageable shards, "
      "cycling through all %zu 4-of-10 data patterns\", \"decode_us\": %.1f, \"decode_ok\": %s}\n",
      size, patterns.size(), median(t), ok ? "true" : "false");
  end_line(line);
  for (auto* p : data) std::free(p);
  for (auto* p : coding) std::free(p);
  std::free(matrix);
}

// ecx_datanode_main.cpp:699-735, unchanged, one arriving block at a time.
void ecx_case(int k, int m, int block_size, int stripes) {
  begin_case();
  int* matrix = reed_sol_vandermonde_coding_matrix(k, m, 8);
  char* block_multiply_m = static_cast<char*>(std::malloc((size_t(block_size) + sizeof(long)) * size_t(m)));
  std::vector<char*> blocks(static_cast<size_t>(k));
  for (int j = 0; j < k; ++j) {
    blocks[size_t(j)] = static_cast<char*>(std::malloc(size_t(block_size) + sizeof(long)));
    fill(blocks[size_t(j)], size_t(block_size), 99u + unsigned(j));
  }
  std::vector<int> init(static_cast<size_t>(m));
  std::vector<double> per_block;
  for (int s = 0; s < stripes + 1; ++s) {
    for (int cur_eck = 0; cur_eck < k; ++cur_eck) {
      const double t0 = now_us();
      if (cur_eck == 0)
        for (int i = 0; i < m; ++i) init[size_t(i)] = 0;
      char* buffer_block = blocks[size_t(cur_eck)];
      for (int i = 0; i < m; ++i) {
        const int v = matrix[i * k + cur_eck];
        char* acc = block_multiply_m + size_t(i) * (size_t(block_size) + sizeof(long));
        if (v == 1) {
          if (init[size_t(i)] == 0) {
            std::memcpy(acc, buffer_block, size_t(block_size));
            init[size_t(i)] = 1;
          } else {
            galois_region_xor(buffer_block, acc, acc, block_size);
          }
        }
        if (v != 0 && v != 1) {
          galois_w08_region_multiply(buffer_block, v, block_size, acc, init[size_t(i)]);
          init[size_t(i)] = 1;
        }
      }
      if (s > 0) per_block.push_back(now_us() - t0);
    }
  }
  // check: accumulators == encode of the k blocks
  std::vector<char*> coding(static_cast<size_t>(m));
  for (auto& p : coding) p = static_cast<char*>(std::calloc(size_t(block_size) + 8, 1));
  jerasure_matrix_encode(k, m, 8, matrix, blocks.data(), coding.data(), block_size);
  bool ok = true;
  for (int i = 0; i < m; ++i)
    ok = ok && std::memcmp(coding[size_t(i)], block_multiply_m + size_t(i) * (size_t(block_size) + sizeof(long)),
                           size_t(block_size)) == 0;
  const double b = median(per_block);
  char line[1024];
  std::snprintf(line, sizeof line,
      "{\"case\": \"ECX per-block sequence RS(%d,%d)\", \"workload\": \"ecx_datanode_main.cpp:699-735 unchanged, "
      "%d-byte blocks, m separate galois_* calls per block (pageable)\", \"per_block_us\": %.1f, "
      "\"block_GiBps\": %.3f, \"parity_ok\": %s}\n",
      k, m, block_size, b, double(block_size) / (b * 1e-6) / double(1 << 30), ok ? "true" : "false");
  end_line(line);
  for (auto* p : coding) std::free(p);
  for (auto* p : blocks) std::free(p);
  std::free(block_multiply_m);
  std::free(matrix);
}

}  // namespace

// --threads N: N threads each encoding its own stripes (client stripe buffer
// + malloc'd coding, pageable) back to back for ~1 s; aggregate data rate.
// The reference client's ENC_THREAD_NUM > 1, or several clients in one
// process: every thread gets its own context (stream + staging) from the pool.
void threads_case(const char* name, int k, int m, int size, int nthreads) {
  int* matrix = reed_sol_vandermonde_coding_matrix(k, m, 8);
  std::vector<double> rate(static_cast<size_t>(nthreads), 0.0);
  std::vector<std::thread> ts;
  for (int t = 0; t < nthreads; ++t)
    ts.emplace_back([&, t] {
      char* buffer = static_cast<char*>(std::malloc(size_t(k) * size_t(size)));
      std::vector<char*> data(static_cast<size_t>(k)), coding(static_cast<size_t>(m));
      for (int j = 0; j < k; ++j) {
        data[size_t(j)] = buffer + size_t(j) * size_t(size);
        fill(data[size_t(j)], size_t(size), 999u + unsigned(t * 31 + j));
      }
      for (auto& p : coding) p = static_cast<char*>(std::calloc(size_t(size), 1));
      for (int w = 0; w < 3; ++w) jerasure_matrix_encode(k, m, 8, matrix, data.data(), coding.data(), size);
      int calls = 0;
      const double t0 = now_us();
      while (now_us() - t0 < 1e6) {
        jerasure_matrix_encode(k, m, 8, matrix, data.data(), coding.data(), size);
        ++calls;
      }
      rate[size_t(t)] = double(calls) * k * size / ((now_us() - t0) * 1e-6) / double(1 << 30);
      std::free(buffer);
      for (auto* p : coding) std::free(p);
    });
  for (auto& th : ts) th.join();
  double total = 0;
  for (double r : rate) total += r;
  std::printf("{\"case\": \"%s\", \"threads\": %d, \"encode_data_GiBps_total\": %.2f, \"per_thread_GiBps\": %.2f}\n",
              name, nthreads, total, total / nthreads);
  std::fflush(stdout);
  std::free(matrix);
}

int report_fallbacks() {
  const long n = ecgpu_fallback_count();
  std::printf("{\"cpu_fallbacks\": %ld}\n", n);
  return n == 0 ? 0 : 1;
}

int main(int argc, char** argv) {
  ecgpu_set_knob("ECGPU_CPU_FALLBACK", 0);
  if (argc > 1 && std::strcmp(argv[1], "--threads") == 0) {
    for (int n : {1, 2, 4, 8}) {
      threads_case("C1 RS(4,2) 64 KiB", 4, 2, 64 << 10, n);
      threads_case("default RS(3,3) 1 MiB", 3, 3, 1 << 20, n);
      threads_case("C2 RS(6,3) 1 MiB", 6, 3, 1 << 20, n);
      threads_case("C3 RS(10,4) 4 MiB", 10, 4, 4 << 20, n);
    }
    return report_fallbacks();
  }
  const bool quick = argc > 1 && std::strcmp(argv[1], "--quick") == 0;
  // --only PREFIX: the client cases whose name starts with PREFIX, stripe buffer layout only
  const char* only = argc > 2 && std::strcmp(argv[1], "--only") == 0 ? argv[2] : nullptr;
  const int e0[] = {0};
  const int e0123[] = {0, 1, 2, 3};
  const Case cases[] = {{"default RS(3,3) 1 MiB (ych_ec_test.h)", 3, 3, 1 << 20, 100},
                        {"C1 RS(4,2) 64 KiB", 4, 2, 64 << 10, 300},
                        {"C2 RS(6,3) 1 MiB", 6, 3, 1 << 20, 100},
                        {"C3 RS(10,4) 4 MiB", 10, 4, 4 << 20, 30},
                        {"C5 RS(12,4) 16 MiB", 12, 4, 16 << 20, quick ? 4 : 10}};
  if (only) {
    for (const Case& c : cases)
      if (std::strncmp(c.name, only, std::strlen(only)) == 0) client_case(c, true, e0, 1);
    return report_fallbacks();
  }
  for (const char* mode : {"gpu", "lib"}) {
    g_mode = mode;
    ecgpu_reset_knob("ECGPU_MIN_OFFLOAD_KIB");
    if (std::strcmp(mode, "gpu") == 0) ecgpu_set_knob("ECGPU_MIN_OFFLOAD_KIB", 0);
    for (int stripe_buffer = 1; stripe_buffer >= 0; --stripe_buffer)
      for (const Case& c : cases) client_case(c, stripe_buffer != 0, e0, 1);
    client_case({"C4 RS(10,4) 4 MiB", 10, 4, 4 << 20, 30}, true, e0123, 4);
    new_pattern_case(4096);
    ecx_case(3, 3, 349525, quick ? 10 : 40);
    ecx_case(10, 4, 349525, quick ? 4 : 12);
  }
  return report_fallbacks();
}
