// crossover.cpp -- where a synchronous host-memory call is cheaper on the
// GPU than on the library's own CPU executor (cpu_exec.hpp), per call shape,
// through the reference's own names (libjerasure_amd.so) as an unchanged
// caller sees them.  Sets SURVEY §5's "min offload size" default
// (ECGPU_MIN_OFFLOAD_KIB).
//
// For each shape and shard size, three arms interleaved in one process
// (knobs switched with ecgpu_set_knob between calls):
//   gpu    ECGPU_MIN_OFFLOAD_KIB=0            (every call on the MI355X)
//   cpu    ECGPU_GPU=0                        (every call on the CPU executor)
//   lib    the library's defaults             (what a deployment gets)
// Median per-call microseconds over `reps` calls per arm.  Buffers: pageable
// (malloc, the reference's callers) or pinned (hipHostRegister'd through
// ecgpu_host_register), "warm" (the same buffers every call, as for a block
// the caller just received) or "cold" (a pool of buffer sets of >= 192 MiB,
// cycled, so each call reads memory no recent call touched).
//
// One JSON line per (shape, size, memory, temperature), then one summary
// line per (shape, memory, temperature): the smallest bytes-moved at which
// the GPU arm beats the CPU arm.
//
// Built by tools/build_tools.sh.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "galois.h"
#include "jerasure.h"
#include "reed_sol.h"

extern "C" long ecgpu_fallback_count(void);
extern "C" long ecgpu_cpu_call_count(void);
extern "C" int ecgpu_set_knob(const char* name, int value);
extern "C" int ecgpu_reset_knob(const char* name);
extern "C" int ecgpu_host_register(void* ptr, long bytes);
extern "C" int ecgpu_host_unregister(void* ptr);

namespace {

double now_us() {
  using namespace std::chrono;
  return duration<double, std::micro>(steady_clock::now().time_since_epoch()).count();
}

double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

// 64 KiB of LCG bytes, repeated (filling 192 MiB pools byte by byte is slow)
void fill(char* p, size_t n, unsigned seed) {
  const size_t head = std::min(n, size_t(64) << 10);
  for (size_t i = 0; i < head; ++i) p[i] = char((seed = seed * 1103515245u + 12345u) >> 16);
  for (size_t i = head; i < n; i += head) std::memcpy(p + i, p, std::min(head, n - i));
}

enum Kind { kXor3, kXorAcc, kMulAcc, kEncode, kDecode };

struct Shape {
  const char* name;
  Kind kind;
  int k, m;             // encode / decode
  int nerased;          // decode: data shards 0..nerased-1
  int buffers;          // distinct buffers a call names (bytes moved = buffers x size)
};

// One set of buffers for a call.
struct Set {
  std::vector<char*> data, coding;
};

struct Arm {
  const char* name;
  void (*apply)();
};

void arm_gpu() {
  ecgpu_reset_knob(nullptr);
  ecgpu_set_knob("ECGPU_CPU_FALLBACK", 0);
  ecgpu_set_knob("ECGPU_MIN_OFFLOAD_KIB", 0);
}
void arm_cpu() {
  ecgpu_reset_knob(nullptr);
  ecgpu_set_knob("ECGPU_CPU_FALLBACK", 0);
  ecgpu_set_knob("ECGPU_GPU", 0);
}
void arm_lib() {
  ecgpu_reset_knob(nullptr);
  ecgpu_set_knob("ECGPU_CPU_FALLBACK", 0);
}

const Arm kArms[] = {{"gpu", arm_gpu}, {"cpu", arm_cpu}, {"lib", arm_lib}};

void call(const Shape& sh, Set& s, int* matrix, int* erasures, int size) {
  switch (sh.kind) {
    case kXor3:
      galois_region_xor(s.data[0], s.data[1], s.coding[0], size);
      break;
    case kXorAcc:  // ecx_datanode_main.cpp:714 (r3 == r2: the accumulator)
      galois_region_xor(s.data[0], s.coding[0], s.coding[0], size);
      break;
    case kMulAcc:  // ecx_datanode_main.cpp:724 (add into the accumulator)
      galois_w08_region_multiply(s.data[0], 0x8E, size, s.coding[0], 1);
      break;
    case kEncode:
      jerasure_matrix_encode(sh.k, sh.m, 8, matrix, s.data.data(), s.coding.data(), size);
      break;
    case kDecode:
      if (jerasure_matrix_decode(sh.k, sh.m, 8, matrix, 0, erasures, s.data.data(), s.coding.data(), size) != 0) {
        std::fprintf(stderr, "decode failed\n");
        std::exit(2);
      }
      break;
  }
}

struct Result {
  std::string shape, memory, temp;
  long long moved;
  double gpu, cpu;
};
std::vector<Result> g_results;

void run(const Shape& sh, int size, bool pinned, bool cold, int reps) {
  const int nd = sh.kind == kEncode || sh.kind == kDecode ? sh.k : sh.kind == kXor3 ? 2 : 1;
  const int nc = sh.kind == kEncode || sh.kind == kDecode ? sh.m : 1;
  const size_t set_bytes = size_t(nd + nc) * size_t(size);
  const int nsets = cold ? int(std::min<size_t>(4096, std::max<size_t>(2, (size_t(192) << 20) / set_bytes))) : 1;
  // one slab per set (the client's stripe buffer shape), so a pinned set is one registration
  std::vector<char*> slabs;
  std::vector<Set> sets(static_cast<size_t>(nsets));
  for (int t = 0; t < nsets; ++t) {
    char* slab = static_cast<char*>(std::aligned_alloc(4096, (set_bytes + 4095) & ~size_t(4095)));
    fill(slab, set_bytes, 77u + unsigned(t));
    if (pinned && ecgpu_host_register(slab, long(set_bytes)) != 0) {
      std::fprintf(stderr, "ecgpu_host_register failed\n");
      std::exit(2);
    }
    slabs.push_back(slab);
    for (int j = 0; j < nd; ++j) sets[size_t(t)].data.push_back(slab + size_t(j) * size_t(size));
    for (int j = 0; j < nc; ++j) sets[size_t(t)].coding.push_back(slab + size_t(nd + j) * size_t(size));
  }
  int* matrix = sh.k ? reed_sol_vandermonde_coding_matrix(sh.k, sh.m, 8) : nullptr;
  std::vector<int> erasures;
  for (int e = 0; e < sh.nerased; ++e) erasures.push_back(e);
  erasures.push_back(-1);
  if (sh.kind == kDecode)  // valid codewords: the decode's survivors are consistent
    for (auto& s : sets) jerasure_matrix_encode(sh.k, sh.m, 8, matrix, s.data.data(), s.coding.data(), size);
  std::vector<std::vector<double>> t(3);
  int next = 0;
  for (int r = 0; r < reps + 2; ++r)
    for (int a = 0; a < 3; ++a) {
      kArms[a].apply();
      Set& s = sets[size_t(next++ % nsets)];
      const double t0 = now_us();
      call(sh, s, matrix, erasures.data(), size);
      const double dt = now_us() - t0;
      if (r >= 2) t[size_t(a)].push_back(dt);
    }
  ecgpu_reset_knob(nullptr);
  const double g = median(t[0]), c = median(t[1]), l = median(t[2]);
  std::printf(
      "{\"shape\": \"%s\", \"shard_bytes\": %d, \"bytes_moved\": %lld, \"memory\": \"%s\", \"buffers\": \"%s\", "
      "\"gpu_us\": %.1f, \"cpu_us\": %.1f, \"lib_us\": %.1f, \"faster\": \"%s\", \"lib_vs_best\": %.3f, \"reps\": %d}\n",
      sh.name, size, (long long)sh.buffers * size, pinned ? "pinned" : "pageable", cold ? "cold" : "warm", g, c, l,
      g < c ? "gpu" : "cpu", l / std::min(g, c), reps);
  std::fflush(stdout);
  g_results.push_back({sh.name, pinned ? "pinned" : "pageable", cold ? "cold" : "warm", (long long)sh.buffers * size, g, c});
  for (char* p : slabs) {
    if (pinned) ecgpu_host_unregister(p);
    std::free(p);
  }
  std::free(matrix);
}

}  // namespace

int main(int argc, char** argv) {
  const bool quick = argc > 1 && std::strcmp(argv[1], "--quick") == 0;
  const Shape shapes[] = {
      {"ECX region multiply-add (r2 accumulator)", kMulAcc, 0, 0, 0, 2},
      {"ECX region xor (r3 == r2 accumulator)", kXorAcc, 0, 0, 0, 2},
      {"region xor r1 ^ r2 -> r3", kXor3, 0, 0, 0, 3},
      {"RS(4,2) encode (C1)", kEncode, 4, 2, 0, 6},
      {"RS(3,3) encode (client default)", kEncode, 3, 3, 0, 6},
      {"RS(6,3) encode (C2)", kEncode, 6, 3, 0, 9},
      {"RS(10,4) encode (C3)", kEncode, 10, 4, 0, 14},
      {"RS(10,4) decode{0}", kDecode, 10, 4, 1, 11},
      {"RS(10,4) decode{0,1,2,3} (C4)", kDecode, 10, 4, 4, 14},
  };
  const int sizes[] = {1 << 10, 4 << 10, 16 << 10, 64 << 10, 128 << 10, 256 << 10, 349525, 512 << 10, 1 << 20,
                       2 << 20, 4 << 20};
  for (int pinned = 0; pinned <= 1; ++pinned)
    for (int cold = 0; cold <= 1; ++cold) {
      if (pinned && cold) continue;  // registering 192 MiB of sets per size: not the callers' shape
      for (const Shape& sh : shapes)
        for (int size : sizes) {
          if (quick && size != (64 << 10) && size != 349525 && size != (4 << 20)) continue;
          const long long moved = (long long)sh.buffers * size;
          const int reps = moved >= (32 << 20) ? 15 : moved >= (4 << 20) ? 30 : 60;
          run(sh, size, pinned != 0, cold != 0, reps);
        }
    }
  // per (shape, memory, temperature): the smallest bytes moved from which on
  // the GPU arm is faster at every measured size (-1: never)
  for (size_t i = 0; i < g_results.size();) {
    size_t j = i;
    while (j < g_results.size() && g_results[j].shape == g_results[i].shape && g_results[j].memory == g_results[i].memory &&
           g_results[j].temp == g_results[i].temp)
      ++j;
    long long cross = -1;
    for (size_t q = j; q-- > i;) {
      if (g_results[q].gpu >= g_results[q].cpu) break;
      cross = g_results[q].moved;
    }
    std::printf("{\"summary\": \"%s\", \"memory\": \"%s\", \"buffers\": \"%s\", \"gpu_faster_from_bytes_moved\": %lld}\n",
                g_results[i].shape.c_str(), g_results[i].memory.c_str(), g_results[i].temp.c_str(), cross);
    i = j;
  }
  std::printf("{\"cpu_fallbacks\": %ld, \"cpu_calls\": %ld}\n", ecgpu_fallback_count(), ecgpu_cpu_call_count());
  return ecgpu_fallback_count() == 0 ? 0 : 1;
}
