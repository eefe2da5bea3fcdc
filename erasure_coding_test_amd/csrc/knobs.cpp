// knobs.cpp -- see knobs.hpp.
#include "knobs.hpp"

#include <atomic>
#include <cerrno>
#include <climits>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

#include "ecgpu.h"

namespace ecgpu {
namespace __attribute__((visibility("hidden"))) rt {
int fail(int code, const std::string& msg);  // capi_host.cpp
}

namespace {

struct KnobDef {
  const char* env;  // the knob's long name (ECGPU_*), read from the environment unless set_only
  const char* name;
  int dflt;
  bool set_only = false;  // settable only through ecgpu_set_knob (test hooks: never from a deployment's environment)
  const char* alias = nullptr;  // a second environment name, read when `env` is unset
};

// Defaults are the production choices (measured).
constexpr KnobDef kDefs[int(Knob::kCount)] = {
    {"ECGPU_CAP", "cap", -1},
    {"ECGPU_BLOCKS_PER_CU", "blocks_per_cu", -1},
    {"ECGPU_KERNEL", "kernel", ECGPU_KERNEL_PERM},
    {"ECGPU_NT", "nt", 1},
    {"ECGPU_WIDE", "wide", 0},
    {"ECGPU_NIB16", "nib16", 1},
    {"ECGPU_WIDE_UNITS", "wide_units", 1},
    {"ECGPU_WIDE_PIPE", "wide_pipe", 1},
    {"ECGPU_WIDE16_BPCU", "wide16_bpcu", 3},
    {"ECGPU_WIDE16_UNITS", "wide16_units", 1},
    {"ECGPU_DEVICE", "device", -1},
    {"ECGPU_BOUNCE_KIB", "bounce_kib", 2048},
    {"ECGPU_ZC_KIB", "zc_kib", 1024},
    {"ECGPU_ZC_OUT_KIB", "zc_out_kib", 4096},
    {"ECGPU_ZC_OUT_SHARD_KIB", "zc_out_shard_kib", 1024},
    {"ECGPU_ZC_PINNED", "zc_pinned", 1},
    {"ECGPU_ZC_GRID", "zc_grid", 64},
    {"ECGPU_INLINE", "inline", 1},
    {"ECGPU_PIPE_2D", "pipe_2d", 1},
    {"ECGPU_PIPE_D2H_WORKER", "pipe_d2h_worker", 1},
    {"ECGPU_PACKET", "packet", 0},
    {"ECGPU_SHARD_SKEW_KIB", "shard_skew_kib", -1},
    {"ECGPU_SPLIT", "split", 0},
    {"ECGPU_SPLIT_MIN_KIB", "split_min_kib", 1024},
    {nullptr, "test_d2h_delay_us", 0},
    {"ECGPU_CPU_FALLBACK", "cpu_fallback", 1},
    {"ECGPU_TEST_INJECT_HIP", "test_inject_hip", 0, true},
    {"ECGPU_GPU", "gpu", 1, false, "EC_GPU"},  // EC_GPU=0/1: SURVEY §5's switch
    {"ECGPU_MIN_OFFLOAD_KIB", "min_offload_kib", -1},
    {"ECGPU_CPU_SIMD", "cpu_simd", -1},
    {"ECGPU_PIPE_ZC", "pipe_zc", 0},
    {"ECGPU_PIPE_CONTIG", "pipe_contig", 1},
    {"ECGPU_PIPE_FLAT", "pipe_flat", 1},
    {"ECGPU_LINK_CALLS", "link_calls", 1},
};

constexpr int kUnset = INT_MIN;
std::once_flag g_once;
int g_base[int(Knob::kCount)];                // the environment's value (or the default), fixed at first use
std::atomic<int> g_over[int(Knob::kCount)];   // ecgpu_set_knob's value, kUnset if none

// A whole-string decimal integer, else the default (so "", "x", "12k" keep it).
int parse_env(const KnobDef& d) {
  const char* e = d.env && !d.set_only ? std::getenv(d.env) : nullptr;
  if ((!e || !*e) && d.alias && !d.set_only) e = std::getenv(d.alias);
  if (!e || !*e) return d.dflt;
  errno = 0;
  char* end = nullptr;
  const long v = std::strtol(e, &end, 10);
  if (*end != '\0' || errno != 0 || v < INT_MIN + 1 || v > INT_MAX) return d.dflt;
  return int(v);
}

void init() {
  std::call_once(g_once, [] {
    for (int i = 0; i < int(Knob::kCount); ++i) {
      g_base[i] = parse_env(kDefs[i]);
      g_over[i].store(kUnset, std::memory_order_relaxed);
    }
  });
}

}  // namespace

int knob(Knob k) {
  init();
  const int v = g_over[int(k)].load(std::memory_order_relaxed);
  return v != kUnset ? v : g_base[int(k)];
}

bool knob_by_name(const char* name, Knob* out) {
  if (!name) return false;
  for (int i = 0; i < int(Knob::kCount); ++i)
    if ((kDefs[i].env && std::strcmp(name, kDefs[i].env) == 0) || std::strcmp(name, kDefs[i].name) == 0) {
      *out = Knob(i);
      return true;
    }
  return false;
}

}  // namespace ecgpu

extern "C" {

ECGPU_API int ecgpu_set_knob(const char* name, int value) {
  ecgpu::Knob k;
  if (!ecgpu::knob_by_name(name, &k))
    return ecgpu::rt::fail(ECGPU_ERR_ARG, std::string("ecgpu_set_knob: unknown knob ") + (name ? name : "(null)"));
  if (value == INT_MIN) return ecgpu::rt::fail(ECGPU_ERR_ARG, "ecgpu_set_knob: INT_MIN is reserved");
  ecgpu::init();
  ecgpu::g_over[int(k)].store(value, std::memory_order_relaxed);
  return ECGPU_OK;
}

ECGPU_API int ecgpu_reset_knob(const char* name) {
  ecgpu::init();
  if (!name) {
    for (auto& o : ecgpu::g_over) o.store(INT_MIN, std::memory_order_relaxed);
    return ECGPU_OK;
  }
  ecgpu::Knob k;
  if (!ecgpu::knob_by_name(name, &k))
    return ecgpu::rt::fail(ECGPU_ERR_ARG, std::string("ecgpu_reset_knob: unknown knob ") + name);
  ecgpu::g_over[int(k)].store(INT_MIN, std::memory_order_relaxed);
  return ECGPU_OK;
}

ECGPU_API int ecgpu_get_knob(const char* name, int* value) {
  if (!value) return ecgpu::rt::fail(ECGPU_ERR_ARG, "ecgpu_get_knob: value is NULL");
  ecgpu::Knob k;
  if (!ecgpu::knob_by_name(name, &k))
    return ecgpu::rt::fail(ECGPU_ERR_ARG, std::string("ecgpu_get_knob: unknown knob ") + (name ? name : "(null)"));
  *value = ecgpu::knob(k);
  return ECGPU_OK;
}

}  // extern "C"
