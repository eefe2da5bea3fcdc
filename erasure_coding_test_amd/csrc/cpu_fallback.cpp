// cpu_fallback.cpp -- see cpu_fallback.hpp.  Host-only (g++): the
// bookkeeping of the failure contract and of the calls routed to the CPU
// executor (cpu_exec.cpp) by choice.
#include "cpu_fallback.hpp"

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <mutex>

#include "ecgpu.h"
#include "knobs.hpp"

namespace ecgpu {
namespace __attribute__((visibility("hidden"))) rt {

int fail(int code, const std::string& msg);  // capi_host.cpp

namespace {

thread_local bool t_written = false;
// One flag per device ordinal the library accepts (ECGPU_DEVICES parses
// 0..1023): a lost device never sends another device's calls to the CPU.
constexpr int kMaxDevices = 1024;
std::atomic<bool> g_lost[kMaxDevices];
std::atomic<int64_t> g_fallbacks{0};
std::atomic<int64_t> g_cpu_calls{0};
std::once_flag g_log_once;

bool valid_device(int device) { return device >= 0 && device < kMaxDevices; }

}  // namespace

void trace_begin() { t_written = false; }
void note_caller_write() { t_written = true; }
bool caller_written() { return t_written; }

void mark_device_lost(int device) {
  if (valid_device(device)) g_lost[device].store(true, std::memory_order_relaxed);
}

bool device_lost(int device) { return valid_device(device) && g_lost[device].load(std::memory_order_relaxed); }

bool fallback_enabled() { return knob(Knob::kCpuFallback) != 0; }

int injected_failure(int device, int stage) {
  const int v = knob(Knob::kTestInjectHip);
  if (v <= 0) return ECGPU_OK;
  if ((v == 1 || v == 2) && stage == 0) {
    if (v == 2) mark_device_lost(device);
    return fail(ECGPU_ERR_HIP, "injected HIP failure before the first launch (test_inject_hip=" + std::to_string(v) +
                                   ")");
  }
  if (v == 3 && stage == 1)
    return fail(ECGPU_ERR_HIP, "injected HIP failure after caller memory was written (test_inject_hip=3)");
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

// The crossover per executor SIMD level (tools/crossover.cpp on the MI355X
// host, scored by tools/crossover_fit.py: profiles/r06_crossover_fit.txt,
// r06_crossover_simd.txt): GFNI 16 MiB, AVX2 4 MiB, scalar 256 KiB.
int64_t min_offload_bytes() {
  const int kib = knob(Knob::kMinOffloadKib);
  if (kib >= 0) return int64_t(kib) << 10;
  static const int64_t by_level[3] = {int64_t(256) << 10, int64_t(4) << 20, int64_t(16) << 20};
  return by_level[std::max(0, std::min(2, cpu_simd_level()))];
}

bool cpu_by_choice(int64_t bytes_moved) {
  if (knob(Knob::kGpu) == 0) return true;
  return bytes_moved < min_offload_bytes();
}

void record_cpu_call() { g_cpu_calls.fetch_add(1, std::memory_order_relaxed); }

int64_t cpu_call_count() { return g_cpu_calls.load(std::memory_order_relaxed); }

}  // namespace rt
}  // namespace ecgpu

extern "C" {
ECGPU_API int64_t ecgpu_fallback_count(void) { return ecgpu::rt::fallback_count(); }
ECGPU_API int64_t ecgpu_cpu_call_count(void) { return ecgpu::rt::cpu_call_count(); }
ECGPU_API int64_t ecgpu_min_offload_bytes(void) { return ecgpu::rt::min_offload_bytes(); }
ECGPU_API int ecgpu_device_lost(int device) { return ecgpu::rt::device_lost(device) ? 1 : 0; }
}
