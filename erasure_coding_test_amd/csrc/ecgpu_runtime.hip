// ecgpu_runtime.hip -- device side of include/ecgpu.h: plans, contexts,
// staging of host buffers, the synchronous calls with their failure contract,
// and the hot-path C ABI.  How a plan launches is dispatch_w8.hip (w = 8) and
// dispatch_wide.hip (w = 16 / 32).  The ECX accumulators (accum.hip), host
// pipelines (pipeline.hip) and GF(2) packet coding (packets.hip) build on the
// helpers this file exports to them through runtime.hpp.
//
// Execution model (MI355X-first, not the reference's byte loops):
//   * every hot-path call is planned on the host into ONE fused
//     rows x nsrc GF(2^8) matrix apply (planner.hpp) and runs as one
//     streaming launch per <= 4 output rows;
//   * buffers are classified per pointer: device memory is used in place,
//     host memory is staged through a per-context HBM slab with
//     hipMemcpyAsync on that context's own stream (ordered after the null stream);
//   * contexts (stream + staging + plan cache) come from a process-wide
//     pool, so concurrent callers (the reference's encode pthreads,
//     client_main.cpp:1074-1164) never share a stream or a lock on the
//     submit path; tables are built once (std::call_once in gf_host).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <list>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "buffer_contract.hpp"
#include "cpu_fallback.hpp"
#include "ecgpu.h"
#include "gf_host.hpp"
#include "gf_kernels.hpp"
#include "gf_spec.hpp"
#include "host_sync.hpp"
#include "knobs.hpp"
#include "matrix_host.hpp"
#include "planner.hpp"
#include "runtime.hpp"

using namespace ecgpu;
using namespace ecgpu::rt;
using dev::ApplyArgs;
using dev::u32x4;

ECGPU_RT_BEGIN

// t_err / fail / ecgpu_last_error live in capi_host.cpp (host code, so the
// host-only checks -- buffer contract, knobs -- report through them too)

// Errors after which the device's context is unusable for the rest of the
// process (a kernel fault, a lost / missing device or driver): the device is
// marked lost, and with ECGPU_CPU_FALLBACK later synchronous calls on it go
// straight to the CPU (cpu_fallback.hpp).  hipErrorInvalidDevice is not one:
// a bad ordinal argument returns it (ecgpu_device_pci_bus_id(99)) on a
// healthy device.
bool sticky(hipError_t e) {
  switch (e) {
    case hipErrorNotInitialized:
    case hipErrorDeinitialized:
    case hipErrorInsufficientDriver:
    case hipErrorNoDevice:
    case hipErrorNoBinaryForGpu:
    case hipErrorECCNotCorrectable:
    case hipErrorIllegalAddress:
    case hipErrorLaunchTimeOut:
    case hipErrorContextIsDestroyed:
    case hipErrorAssert:
    case hipErrorLaunchFailure:
      return true;
    default:
      return false;
  }
}

// The device the current synchronous call targets (CallDeviceScope), -1
// outside one.
thread_local int t_call_device = -1;

CallDeviceScope::CallDeviceScope(int device) : prev(t_call_device) { t_call_device = device; }
CallDeviceScope::~CallDeviceScope() { t_call_device = prev; }

int fail_hip(hipError_t e, const char* what) {
  std::string msg = std::string(what) + ": " + hipGetErrorString(e);
  int d = t_call_device;
  if (d < 0 && hipGetDevice(&d) != hipSuccess) d = -1;
  bool lost = sticky(e);
  if (!lost && e == hipErrorUnknown && d >= 0) {
    // ordinary failures return it too: sticky only when the device still
    // fails a synchronize afterwards
    DeviceGuard g(d);
    (void)hipGetLastError();
    lost = hipDeviceSynchronize() != hipSuccess;
    (void)hipGetLastError();
  }
  if (lost && d >= 0) mark_device_lost(d);
  // The library reports the error through its own channel; HIP's per-thread
  // last error is shared with the caller's HIP code in the same process, so
  // a handled failure (a bad ordinal, an OOM the CPU completed) must not
  // surface in the caller's next error check (torch's launch checks did).
  (void)hipGetLastError();
  return fail(ECGPU_ERR_HIP, msg);
}


// One non-blocking stream per device for coefficient-table uploads: a plan's
// creation does not wait for its tables (one blocking copy cost ~12 us,
// tools/hip_overheads.cpp); its launches wait on the upload's event instead.
hipStream_t upload_stream(int device) {
  static hostsync::PerDevice<hipStream_t> streams;
  return streams.get(device, [](int dev) {
    DeviceGuard g(dev);
    hipStream_t s = nullptr;
    return hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess ? s : nullptr;
  });
}

// Allocates p->d_tabs and uploads `host` into it without waiting (the plan
// keeps `host` alive until the upload has completed).
int plan_upload_tables(ecgpu_plan* p, std::vector<uint8_t>&& host) {
  DeviceGuard g(p->device);
  ECGPU_HIP(hipMalloc(reinterpret_cast<void**>(&p->d_tabs), host.size()));
  p->host_tabs = std::move(host);
  const hipStream_t s = upload_stream(p->device);
  if (!s) {  // no stream: a blocking copy
    ECGPU_HIP(hipMemcpy(p->d_tabs, p->host_tabs.data(), p->host_tabs.size(), hipMemcpyHostToDevice));
    return ECGPU_OK;
  }
  ECGPU_HIP(hipEventCreateWithFlags(&p->uploaded, hipEventDisableTiming));
  ECGPU_HIP(hipMemcpyAsync(p->d_tabs, p->host_tabs.data(), p->host_tabs.size(), hipMemcpyHostToDevice, s));
  ECGPU_HIP(hipEventRecord(p->uploaded, s));
  p->upload_pending = true;
  return ECGPU_OK;
}

// Waits for the plan's table upload on the host (a no-op once it completed).
int plan_sync_tables(ecgpu_plan* p) {
  if (!p->upload_pending) return ECGPU_OK;
  ECGPU_HIP(hipEventSynchronize(p->uploaded));
  p->upload_pending = false;
  std::vector<uint8_t>().swap(p->host_tabs);
  return ECGPU_OK;
}

// Orders `stream` after the plan's table upload (a no-op once it completed).
// A blocking bind has already waited for it, so a bound plan launches inside
// a stream capture without touching the event; a plan bound on a stream
// (the synchronous calls) may not be captured before its upload completed.
int plan_wait_tables(ecgpu_plan* p, hipStream_t stream) {
  if (!p->upload_pending) return ECGPU_OK;
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &cap) == hipSuccess && cap != hipStreamCaptureStatusNone)
    return fail(ECGPU_ERR, "plan tables still uploading: bind the plan without a stream before capturing it");
  (void)hipGetLastError();
  const hipError_t q = hipEventQuery(p->uploaded);
  if (q == hipSuccess) {
    p->upload_pending = false;
    std::vector<uint8_t>().swap(p->host_tabs);
    return ECGPU_OK;
  }
  if (q != hipErrorNotReady) return fail_hip(q, "table upload");
  (void)hipGetLastError();  // not ready is not an error
  ECGPU_HIP(hipStreamWaitEvent(stream, p->uploaded, 0));
  return ECGPU_OK;
}

void plan_free(ecgpu_plan* p) {
  if (!p) return;
  DeviceGuard g(p->device);
  if (p->uploaded) {
    (void)hipEventSynchronize(p->uploaded);  // the table upload may still read host_tabs
    (void)hipEventDestroy(p->uploaded);
  }
  if (p->d_tabs) (void)hipFree(p->d_tabs);
  if (p->d_ptrs) (void)hipFree(p->d_ptrs);
  delete p;
}

int plan_init(ecgpu_plan* p, int rows, int nsrc, const int* coefs, int device, int w) {
  p->device = device;
  p->rows = rows;
  p->nsrc = nsrc;
  p->w = w;
  p->kind = knob(Knob::kKernel);
  p->nt = std::min(kStorePolicies - 1, std::max(0, knob(Knob::kNt)));
  const size_t n = size_t(rows) * nsrc;
  p->coef.resize(n);
  if (w != 8) return plan_init_wide(p, coefs);
  return plan_init_w8(p, coefs);
}

// With a stream the pointer tables are uploaded asynchronously on it; unless
// `keep_alive` (the caller keeps src/dst alive until it synchronises the
// stream, as execute() does) the call waits for the upload.
int plan_bind(ecgpu_plan* p, int stripes, const uint8_t* const* src, uint8_t* const* dst, int64_t size,
              hipStream_t stream, bool keep_alive) {
  const size_t ns = size_t(stripes) * p->nsrc, nd = size_t(stripes) * p->rows;
  DeviceGuard g(p->device);
  // a blocking bind settles the table upload too (it overlapped the table
  // build-up to here); a bind on a stream leaves it to the launch
  if (!stream)
    if (int rc = plan_sync_tables(p)) return rc;
  if (ns + nd > p->cap_ptrs) {
    if (p->d_ptrs) ECGPU_HIP(hipFree(p->d_ptrs));
    p->d_ptrs = nullptr;
    p->cap_ptrs = 0;
    ECGPU_HIP(hipMalloc(reinterpret_cast<void**>(&p->d_ptrs), (ns + nd) * sizeof(void*)));
    p->cap_ptrs = ns + nd;
  }
  p->d_src = static_cast<const uint8_t**>(static_cast<void*>(p->d_ptrs));
  p->d_dst = static_cast<uint8_t**>(static_cast<void*>(p->d_ptrs + ns));
  bool aligned = true;
  for (size_t i = 0; i < ns; ++i) aligned &= (reinterpret_cast<uintptr_t>(src[i]) & 15u) == 0;
  for (size_t i = 0; i < nd; ++i) aligned &= (reinterpret_cast<uintptr_t>(dst[i]) & 15u) == 0;
  if (stream && keep_alive) {
    // the caller's arrays outlive the stream sync: no wait here
    ECGPU_HIP(hipMemcpyAsync(p->d_src, src, ns * sizeof(void*), hipMemcpyHostToDevice, stream));
    ECGPU_HIP(hipMemcpyAsync(p->d_dst, dst, nd * sizeof(void*), hipMemcpyHostToDevice, stream));
  } else {
    // one upload of [sources | destinations]
    std::vector<const void*> host(ns + nd);
    std::memcpy(host.data(), src, ns * sizeof(void*));
    std::memcpy(host.data() + ns, dst, nd * sizeof(void*));
    if (stream) {
      ECGPU_HIP(hipMemcpyAsync(p->d_ptrs, host.data(), (ns + nd) * sizeof(void*), hipMemcpyHostToDevice, stream));
      ECGPU_HIP(hipStreamSynchronize(stream));  // the host table dies on return
    } else {
      ECGPU_HIP(hipMemcpy(p->d_ptrs, host.data(), (ns + nd) * sizeof(void*), hipMemcpyHostToDevice));
    }
  }
  p->stripes = stripes;
  p->size = size;
  p->aligned = aligned;
  return ECGPU_OK;
}

// ------------------------------------------------------ context pool ----

hostsync::IdlePool<Ctx> g_pool;  // idle contexts (process lifetime)

int visible_devices();

// A forced ECGPU_DEVICE that names a visible device (or any, when HIP cannot
// tell), else -1: a device this process cannot see is ignored, with one
// stderr line, instead of failing every call (or sending it to the CPU).
int forced_device() {
  const int forced = knob(Knob::kDevice);
  if (forced < 0) return -1;
  static const int visible = visible_devices();
  if (visible <= 0 || forced < visible) return forced;
  static std::once_flag once;
  std::call_once(once, [&] {
    std::fprintf(stderr, "libecgpu: ECGPU_DEVICE=%d ignored (%d visible)\n", forced, visible);
  });
  return -1;
}

int current_device() {
  const int forced = forced_device();
  if (forced >= 0) return forced;
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess) d = 0;
  return d;
}

// ECGPU_DEVICES (or ecgpu_set_devices): the devices the synchronous
// host-memory calls spread over.  Each calling thread is given one of them,
// round-robin in the order threads make their first such call, and keeps it
// -- so the reference client's byte-range encode pthreads
// (client_main.cpp:1074-1164) each drive their own GPU and PCIe link.  Unset
// (the default): the caller's current device, as before.  "all" = every
// visible device; otherwise a comma-separated list (repeats allowed).
std::mutex g_devices_mu;
std::shared_ptr<const std::vector<int>> g_devices;  // null: unset
std::atomic<uint64_t> g_device_rr{0};

std::vector<int> parse_devices(const char* s, int visible) {
  std::vector<int> out;
  if (!s || !*s) return out;
  if (std::strcmp(s, "all") == 0) {
    for (int d = 0; d < visible; ++d) out.push_back(d);
    return out;
  }
  const char* q = s;
  while (*q) {
    char* end = nullptr;
    const long v = std::strtol(q, &end, 10);
    if (end == q || v < 0 || v > 1023) return {};  // malformed: ignored as a whole
    out.push_back(int(v));
    q = end;
    if (*q == ',') ++q;
    else if (*q) return {};
  }
  return out;
}

// Visible devices, or 0 when HIP cannot tell (no GPU: lists are not checked).
int visible_devices() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n < 0) {
    (void)hipGetLastError();
    n = 0;
  }
  return n;
}

// The first entry of `list` that is not a visible device, or -1.
int invisible_entry(const std::vector<int>& list, int visible) {
  for (int d : list)
    if (visible > 0 && d >= visible) return d;
  return -1;
}

std::shared_ptr<const std::vector<int>> device_list() {
  static std::once_flag once;
  std::call_once(once, [] {
    const char* e = std::getenv("ECGPU_DEVICES");
    if (!e || !*e) return;
    const int n = visible_devices();
    auto v = std::make_shared<const std::vector<int>>(parse_devices(e, n));
    // a malformed list, or one naming a device this process cannot see, is
    // ignored as a whole (every call would otherwise fail or fall back)
    const int bad = invisible_entry(*v, n);
    if (v->empty() || bad >= 0) {
      std::fprintf(stderr, "libecgpu: ECGPU_DEVICES=\"%s\" ignored (%s)\n", e,
                   bad >= 0 ? ("device " + std::to_string(bad) + " is not visible; " + std::to_string(n) +
                               " visible").c_str()
                            : "expected \"all\" or a comma-separated list of device ordinals");
      return;
    }
    std::lock_guard<std::mutex> lk(g_devices_mu);
    if (!g_devices) g_devices = v;
  });
  std::lock_guard<std::mutex> lk(g_devices_mu);
  return g_devices;
}

// The device a synchronous call on host memory runs on: a forced
// ECGPU_DEVICE, else this thread's device from the ECGPU_DEVICES list, else
// the caller's current device.
int host_call_device() {
  if (const int forced = forced_device(); forced >= 0) return forced;
  const auto list = device_list();
  if (!list || list->empty()) return current_device();
  thread_local std::shared_ptr<const std::vector<int>> t_list;
  thread_local int t_dev = -1;
  if (t_list != list) {
    t_list = list;
    t_dev = (*list)[size_t(g_device_rr.fetch_add(1, std::memory_order_relaxed) % list->size())];
  }
  return t_dev;
}

// A call naming device memory runs where that memory is (the current device,
// as before: classify() rejects another device's buffers); an all-host call
// takes host_call_device().
int call_device(const std::vector<void*>& a, const std::vector<void*>& b) {
  if (const int forced = forced_device(); forced >= 0) return forced;
  const auto list = device_list();
  if (!list || list->empty()) return current_device();
  if (!all_host(a) || !all_host(b)) return current_device();
  return host_call_device();
}

Ctx* acquire_ctx(int device, int* rc) {
  if (Ctx* c = g_pool.acquire(device)) {
    *rc = ECGPU_OK;
    return c;
  }
  auto* c = new Ctx();
  c->device = device;
  DeviceGuard g(device);
  // A blocking stream: a synchronous call on device buffers is ordered after
  // work the caller queued on the null stream (PyTorch's default stream,
  // e.g. the fill of a freshly allocated output), and that stream's later
  // work after the call.  Calls from different threads still run on
  // different contexts, unordered against each other.
  hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamDefault);
  if (e != hipSuccess) {
    *rc = fail_hip(e, "hipStreamCreateWithFlags");
    delete c;
    return nullptr;
  }
  *rc = ECGPU_OK;
  return c;
}

void release_ctx(Ctx* c) { g_pool.release(c->device, c); }


int ctx_plan(Ctx* c, int rows, int nsrc, const std::vector<uint32_t>& coef, int w, ecgpu_plan** out) {
  // the engine and store policy are part of the key: a knob switched between
  // calls (an in-process A/B) must reach the next launch (plan_init reads them)
  const int kind = knob(Knob::kKernel), nt = std::min(kStorePolicies - 1, std::max(0, knob(Knob::kNt)));
  PlanKey key{rows, nsrc, w, kind, nt, coef};
  for (auto it = c->plans.begin(); it != c->plans.end(); ++it)
    if (it->first == key) {
      c->plans.splice(c->plans.begin(), c->plans, it);
      *out = it->second;
      return ECGPU_OK;
    }
  auto* p = new ecgpu_plan();
  std::vector<int> ci(coef.begin(), coef.end());
  int rc = plan_init(p, rows, nsrc, ci.data(), c->device, w);
  if (rc != ECGPU_OK) {
    plan_free(p);
    return rc;
  }
  c->plans.emplace_front(std::move(key), p);
  if (c->plans.size() > 64) {
    plan_free(c->plans.back().second);
    c->plans.pop_back();
  }
  *out = p;
  return ECGPU_OK;
}

// How a synchronous call moves host (pageable or pinned) buffers, by the
// bytes it stages (measured on MI355X, tools/hip_overheads.cpp,
// tools/zero_copy_probe.cpp): every DMA costs ~10 us of setup
// and a launch + sync ~11 us, so
//   * up to zc_max() staged bytes: NO DMA.  The calling thread copies the
//     host side into coherent pinned memory and the kernel reads its sources
//     and writes its outputs there directly over PCIe (zero-copy; reads and
//     writes travel opposite directions of the link): one launch per call.
//   * up to bounce_max(): the host side is copied by the CPU through a pinned
//     mirror of the staging slab and crosses PCIe as one H2D DMA plus one D2H
//     DMA per run of adjacent outputs.
//   * above: HIP's own pageable copies (a 6 MiB pageable DMA runs at the
//     pinned rate, 120 us), one 2-D copy per run of evenly spaced shards
//     (copy_shards).  Staging large calls through a pinned ring filled by
//     this thread instead lost 10-40 % (a single thread copies cold memory at
//     ~35 GB/s, below the link; profiles/r02_dropin_ab.txt).
size_t bounce_max() { return size_t(std::max(0, knob(Knob::kBounceKib))) << 10; }  // 2 MiB by default

size_t zc_max() { return size_t(std::max(0, knob(Knob::kZcKib))) << 10; }

// A call above bounce_max() whose staged outputs total at most zc_out_max()
// bytes, each at most zc_out_shard_max(), has the kernel write its outputs
// into coherent pinned memory (see execute).  A pageable D2H costs 67 us per
// 1 MiB shard but runs at link rate from 4 MiB (86 us): drop-in C2 encode 333
// -> 296 us, C3 decode{0} (one 4 MiB output) 871 -> 1005 us if it took this
// path (profiles/r02_zc_out_ab.txt).
size_t zc_out_max() { return size_t(std::max(0, knob(Knob::kZcOutKib))) << 10; }

size_t zc_out_shard_max() { return size_t(std::max(0, knob(Knob::kZcOutShardKib))) << 10; }

bool zero_copy_pinned() { return knob(Knob::kZcPinned) != 0; }

bool inline_enabled() { return knob(Knob::kInline) != 0; }

int ensure_bounce(Ctx* c, size_t bytes) {
  if (bytes <= c->bounce_cap) return ECGPU_OK;
  DeviceGuard g(c->device);
  if (c->bounce) ECGPU_HIP(hipHostFree(c->bounce));
  c->bounce = nullptr;
  c->bounce_cap = 0;
  ECGPU_HIP(hipHostMalloc(reinterpret_cast<void**>(&c->bounce), bytes, hipHostMallocDefault));
  c->bounce_cap = bytes;
  return ECGPU_OK;
}

// Coherent (fine-grained) pinned memory: the GPU does not cache it, so CPU
// writes before a launch and GPU writes before its completion are visible to
// the other side without cache maintenance.  Grows geometrically.
int ensure_zc(Ctx* c, size_t bytes) {
  if (bytes <= c->zc_cap) return ECGPU_OK;
  DeviceGuard g(c->device);
  if (c->zc) ECGPU_HIP(hipHostFree(c->zc));
  c->zc = nullptr;
  c->zc_cap = 0;
  const size_t want = std::max(bytes, size_t(256) << 10);
  ECGPU_HIP(hipHostMalloc(reinterpret_cast<void**>(&c->zc), want, hipHostMallocMapped | hipHostMallocCoherent));
  c->zc_cap = want;
  return ECGPU_OK;
}

int ensure_stage(Ctx* c, size_t bytes) {
  if (bytes <= c->stage_cap) return ECGPU_OK;
  DeviceGuard g(c->device);
  if (c->stage) ECGPU_HIP(hipFree(c->stage));
  c->stage = nullptr;
  c->stage_cap = 0;
  ECGPU_HIP(hipMalloc(reinterpret_cast<void**>(&c->stage), bytes));
  c->stage_cap = bytes;
  return ECGPU_OK;
}

// Is p device memory of `device` (usable in place)?  Host memory (pageable or
// pinned) is staged; device memory of another GPU is rejected.
int classify(const void* p, int device, bool* on_device) {
  hipPointerAttribute_t attr;
  hipError_t e = hipPointerGetAttributes(&attr, p);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    *on_device = false;
    return ECGPU_OK;
  }
  if (attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged) {
    if (attr.device != device)
      return fail(ECGPU_ERR_ARG, "buffer lives on device " + std::to_string(attr.device) + ", call runs on " +
                                     std::to_string(device));
    *on_device = true;
    return ECGPU_OK;
  }
  *on_device = false;
  return ECGPU_OK;
}

// Host memory the GPU addresses in place -- hipHostMalloc'd, or registered
// with hipHostRegister -- when [p, p + bytes) lies inside ONE such
// allocation (HIP's range attributes; a range that leaves it would fault).
// *dev = the device address of p.
bool host_mapped(const void* p, size_t bytes, void** dev) {
  hipPointerAttribute_t attr;
  if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  if (attr.type != hipMemoryTypeHost) return false;
  void* start = nullptr;
  size_t range = 0;
  if (hipPointerGetAttribute(&start, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, hipDeviceptr_t(p)) != hipSuccess ||
      hipPointerGetAttribute(&range, HIP_POINTER_ATTRIBUTE_RANGE_SIZE, hipDeviceptr_t(p)) != hipSuccess ||
      hipHostGetDevicePointer(dev, const_cast<void*>(p), 0) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  const char* c = static_cast<const char*>(p);
  const char* s0 = static_cast<const char*>(start);
  return c >= s0 && bytes <= range && size_t(c - s0) <= range - bytes;
}

bool is_pinned(const void* p) {
  hipPointerAttribute_t attr;
  if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return attr.type == hipMemoryTypeHost;
}

// ------------------------------------------------------ stats counters ----
std::mutex g_stats_mu;
double g_stats[3] = {0, 0, 0};  // xor, gf, memcpy -- jerasure.cpp:1145-1147 order

void add_stats(const FusedOp& op) {
  std::lock_guard<std::mutex> lk(g_stats_mu);
  g_stats[0] += op.xor_bytes;
  g_stats[1] += op.gf_bytes;
  g_stats[2] += op.memcpy_bytes;
}

// Moves n shards of `bytes` between host pointers hp[i] and device shards
// d0 + i * dstride.  Every run of >= 2 evenly spaced host shards (a stripe
// laid out in one host slab, as the reference client's stripe buffer is,
// client_main.cpp:1619-1647) goes as ONE 2-D copy, the rest one copy per
// shard.  ECGPU_PIPE_2D=0 always copies per shard.  Used by the pipelines and
// by synchronous calls on large host buffers.
int copy_shards(bool h2d, uint8_t* d0, size_t dstride, const std::vector<char*>& hp, size_t bytes, hipStream_t s) {
  const bool two_d = knob(Knob::kPipe2d) != 0;
  const size_t n = hp.size();
  for (size_t a = 0; a < n;) {
    size_t b = a + 1;  // [a, b): maximal run with one pitch >= bytes
    const ptrdiff_t pitch = b < n ? hp[b] - hp[a] : 0;
    // pageable memory only when the run is contiguous (pitch == bytes): a
    // pageable 2-D copy with gaps between rows ran 15x slower than per-shard
    // copies (RS(6,3) 1 MiB, shards malloc'd one by one, 16 B apart)
    bool ok = two_d && pitch > 0 && size_t(pitch) >= bytes;
    if (ok && size_t(pitch) != bytes) ok = is_pinned(hp[a]);  // pinned or registered
    if (ok)
      while (b < n && hp[b] - hp[b - 1] == pitch) ++b;
    // a gapped run must be pinned at both ends (one registration or
    // allocation spans it; HIP rejects a span across separately registered
    // buffers at enqueue, which falls back below)
    if (b - a >= 2 && size_t(pitch) != bytes && !is_pinned(hp[b - 1] + bytes - 1)) b = a + 1;
    uint8_t* d = d0 + a * dstride;
    if (b - a >= 2) {
      // contiguous on both sides: one 1-D copy.  HIP's 2-D copies lost 40 % of
      // the link when two processes shared the GPU in some allocation states
      // (bench.py's N = 2 rehearsal after its C5 leg: 27 vs 44 GiB/s; 1-D
      // copies 41)
      // (ECGPU_PIPE_FLAT=0 keeps flat runs on hipMemcpy2DAsync too: an A/B switch)
      const bool flat = size_t(pitch) == bytes && dstride == bytes && knob(Knob::kPipeFlat) != 0;
      const hipError_t e =
          flat ? (h2d ? hipMemcpyAsync(d, hp[a], bytes * (b - a), hipMemcpyHostToDevice, s)
                      : hipMemcpyAsync(hp[a], d, bytes * (b - a), hipMemcpyDeviceToHost, s))
          : h2d ? hipMemcpy2DAsync(d, dstride, hp[a], size_t(pitch), bytes, b - a, hipMemcpyHostToDevice, s)
                : hipMemcpy2DAsync(hp[a], size_t(pitch), d, dstride, bytes, b - a, hipMemcpyDeviceToHost, s);
      if (e == hipSuccess) {
        a = b;
        continue;
      }
      // not enqueued: fall back to one copy per shard (the error is not sticky)
      (void)hipGetLastError();
    }
    for (size_t i = a; i < b; ++i) {
      if (h2d)
        ECGPU_HIP(hipMemcpyAsync(d0 + i * dstride, hp[i], bytes, hipMemcpyDefault, s));
      else
        ECGPU_HIP(hipMemcpyAsync(hp[i], d0 + i * dstride, bytes, hipMemcpyDefault, s));
    }
    a = b;
  }
  return ECGPU_OK;
}

// P3 tables of one coefficient (see build_tables).
void build_p3(uint32_t c, uint32_t* p3) {
  const auto& T = gf8().mul[c & 0xFF];
  for (int i = 0; i < dev::kP3Words; ++i) p3[i] = 0;
  for (int e = 0; e < 8; ++e) {
    p3[e >> 2] |= uint32_t(T[e]) << (8 * (e & 3));
    p3[2 + (e >> 2)] |= uint32_t(T[e << 3]) << (8 * (e & 3));
  }
  for (int e = 0; e < 4; ++e) p3[4] |= uint32_t(T[e << 6]) << (8 * e);
}

// Can a fused op run as gf_apply_inl launches (everything in the kernel
// arguments, no table or pointer upload)?  w = 8, 1..16 sources, the
// production engine, and no output that is also a source when the rows need
// more than one launch.
bool inline_ok(const FusedOp& op, int64_t size) {
  const int rows = int(op.dsts.size()), nsrc = int(op.srcs.size());
  // The inline kernels with 15-16 sources and a full 4-row launch hold more
  // coefficient tables than the SGPR file and spill them to VGPR lanes (the
  // plan kernel loads them as it goes): a dense RS(16,4) 64 MiB encode ran
  // 574 us inline against 229 us as a plan launch (tools/probe_inline.py,
  // profiles/r03_inline_vs_plan.csv); K = 14 and below are equal.  Large
  // such calls take the plan; small ones stay inline, where the table upload
  // a plan needs would cost more than the spills.
  const bool spills = nsrc >= 15 && rows >= dev::kMaxRows && size > (int64_t(1) << 20);
  return inline_enabled() && op.w == 8 && nsrc >= 1 && nsrc <= dev::kMaxSpecK && rows >= 1 && !spills &&
         knob(Knob::kKernel) == ECGPU_KERNEL_PERM && !(op.dst_is_src && rows > dev::kMaxRows);
}

// Workgroups of an inline launch that reads or writes host memory in place
// (zero-copy): queued 4 MiB pinned reads ran at 52.5 GB/s with 256
// grid-stride workgroups and 41 GB/s with 1024+ (too many PCIe requests in
// flight; tools/zero_copy_probe.cpp); through the drop-in, 32-64 workgroups
// were best (C3 pinned encode 0.83 ms vs 0.93-0.96 uncapped,
// profiles/r02_zc_grid_sweep.txt).  0 = uncapped.
int64_t zc_grid() { return knob(Knob::kZcGrid); }

// One gf_apply_inl launch per <= 4 output rows over `size` bytes.  host_io:
// some pointer is host memory the kernel reads / writes over PCIe (grid
// capped at zc_grid()).
int launch_inline(const FusedOp& op, const std::vector<const uint8_t*>& sp, const std::vector<uint8_t*>& dp,
                  int64_t size, hipStream_t s, bool host_io) {
  const int K = int(sp.size()), rows = int(dp.size());
  bool aligned = true;
  for (auto* p : sp) aligned &= (reinterpret_cast<uintptr_t>(p) & 15u) == 0;
  for (auto* p : dp) aligned &= (reinterpret_cast<uintptr_t>(p) & 15u) == 0;
  const int64_t nvec = aligned ? size / 16 : 0, byte0 = nvec * 16;
  int64_t nbv = (nvec + dev::kBlock - 1) / dev::kBlock;
  if (host_io && zc_grid() > 0) nbv = std::min(nbv, zc_grid());
  const int64_t nbb = (size - byte0 + dev::kBlock - 1) / dev::kBlock;
  for (int r0 = 0; r0 < rows; r0 += dev::kMaxRows) {
    const int R = std::min(dev::kMaxRows, rows - r0);
    // the grid-stride form only where the grid is capped (host memory in place)
    const bool zc = nbv * dev::kBlock < nvec;
    const InlineKernelFn fn = inline_kernel(K, R, unit_variant(op.coef, K, r0, R), zc);
    if (!fn) return fail(ECGPU_ERR, "no inline kernel for K = " + std::to_string(K));
    dev::InlineArgs a{};
    for (int j = 0; j < K; ++j) a.src[j] = sp[size_t(j)];
    for (int r = 0; r < R; ++r) a.dst[r] = dp[size_t(r0 + r)];
    a.nvec = nvec;
    a.size = size;
    a.byte0 = byte0;
    a.nblk_vec = int(nbv);
    int mul_terms = 0;  // coefficients that are neither 0 nor 1
    for (int r = 0; r < R; ++r)
      for (int j = 0; j < K; ++j) {
        const uint32_t c = op.coef[size_t(r0 + r) * K + j];
        build_p3(c, &a.ptab[(r * K + j) * dev::kP3Words]);
        mul_terms += c > 1u;
      }
    // device buffers: the plan launches' residency cap (cap_for) -- a large
    // one-stripe call streams K + R shards per lane like a batched launch
    // (RS(10,4) 64 MiB encode, separately allocated shards: 275 us uncapped)
    const unsigned lds =
        !host_io && nvec > 0 && cap_for(K, R, mul_terms) ? residency_lds_bytes(current_device(), K + R) : 0u;
    void* args[] = {&a};
    ECGPU_HIP(hipLaunchKernel(reinterpret_cast<const void*>(fn), dim3(unsigned(nbv + nbb)), dim3(dev::kBlock), args,
                              lds, s));
  }
  return ECGPU_OK;
}

// Where every distinct buffer of one synchronous call lives: sources first
// (as op.srcs), then the outputs that are not also sources.  devp[i] is the
// device address the kernel uses (the buffer itself, its mapping in place, or
// a staging slot); staged[i] marks host memory that must be copied.
struct CallMap {
  std::vector<void*> bufs;
  std::vector<uint8_t*> devp;
  std::vector<char> staged;
  size_t nstage = 0;
  size_t slot = 0;   // staging slot bytes (size rounded to 256)
  int64_t size = 0;
  int rows = 0, nsrc = 0;
  bool host_io = false;  // some buffer is host memory the kernel uses in place
  size_t index(const void* p) const { return size_t(std::find(bufs.begin(), bufs.end(), p) - bufs.begin()); }
  std::vector<const uint8_t*> sources() const { return {devp.begin(), devp.begin() + nsrc}; }
  std::vector<uint8_t*> outputs(const FusedOp& op) const {
    std::vector<uint8_t*> dp(static_cast<size_t>(rows));
    for (int r = 0; r < rows; ++r) dp[size_t(r)] = devp[index(op.dsts[size_t(r)])];
    return dp;
  }
};

int map_buffers(const FusedOp& op, int64_t size, int device, bool inl, CallMap* m) {
  m->bufs = op.srcs;
  for (void* d : op.dsts)
    if (std::find(m->bufs.begin(), m->bufs.end(), d) == m->bufs.end()) m->bufs.push_back(d);
  m->size = size;
  m->slot = (size_t(size) + 255) & ~size_t(255);
  m->rows = int(op.dsts.size());
  m->nsrc = int(op.srcs.size());
  m->devp.assign(m->bufs.size(), nullptr);
  m->staged.assign(m->bufs.size(), 0);
  for (size_t i = 0; i < m->bufs.size(); ++i) {
    bool on_dev = false;
    if (int rc = classify(m->bufs[i], device, &on_dev)) return rc;
    if (on_dev) {
      m->devp[i] = static_cast<uint8_t*>(m->bufs[i]);
    } else {
      m->staged[i] = 1;
      ++m->nstage;
    }
  }
  if (inl && zero_copy_pinned()) {
    // pinned / registered host buffers are read and written by the kernel in
    // place over PCIe: no staging copy, no DMA setup, and a call's reads and
    // writes overlap on the two directions of the link
    for (size_t i = 0; i < m->bufs.size(); ++i) {
      void* d = nullptr;
      if (m->staged[i] && host_mapped(m->bufs[i], size_t(size), &d)) {
        m->staged[i] = 0;
        --m->nstage;
        m->devp[i] = static_cast<uint8_t*>(d);
        m->host_io = true;
      }
    }
  }
  return ECGPU_OK;
}

// The call is about to write caller memory (a D2H or host copy into an
// output, or a kernel writing an output in place).  The fused map reads its
// sources only, so a partly written output is recomputed whole by the CPU
// executor -- unless some output is also a source, whose original bytes are
// then gone: from here on such a call cannot be completed on the CPU
// (cpu_fallback.hpp).  Also the test injection's "after the first write"
// failure point.
int caller_write_point(const FusedOp& op, int device) {
  if (op.dst_is_src) note_caller_write();
  return injected_failure(device, 1);
}

// Does a launch write some output in place (device memory, or pinned host
// memory mapped for the kernel) rather than into staging?
bool writes_in_place(const FusedOp& op, const CallMap& m) {
  for (int r = 0; r < m.rows; ++r)
    if (!m.staged[m.index(op.dsts[size_t(r)])]) return true;
  return false;
}

int launch_and_sync(Ctx* c, const FusedOp& op, const CallMap& m, bool host_io) {
  if (int rc = launch_inline(op, m.sources(), m.outputs(op), m.size, c->stream, host_io)) return rc;
  ECGPU_HIP(hipStreamSynchronize(c->stream));
  ECGPU_HIP(hipGetLastError());
  return ECGPU_OK;
}

// Small calls: every staged buffer goes through coherent pinned memory the
// kernel reads and writes in place -- host copies and ONE launch, no DMA.
int exec_zero_copy(Ctx* c, const FusedOp& op, CallMap& m) {
  if (int rc = ensure_zc(c, m.nstage * m.slot)) return rc;
  size_t next = 0;
  for (size_t i = 0; i < m.bufs.size(); ++i)
    if (m.staged[i]) m.devp[i] = c->zc + (next++) * m.slot;
  for (int j = 0; j < m.nsrc; ++j)
    if (m.staged[size_t(j)]) std::memcpy(m.devp[size_t(j)], op.srcs[size_t(j)], size_t(m.size));
  if (writes_in_place(op, m))
    if (int rc = caller_write_point(op, c->device)) return rc;
  if (int rc = launch_and_sync(c, op, m, /*host_io=*/true)) return rc;
  if (int rc = caller_write_point(op, c->device)) return rc;
  for (int r = 0; r < m.rows; ++r) {
    const size_t i = m.index(op.dsts[size_t(r)]);
    if (m.staged[i]) std::memcpy(op.dsts[size_t(r)], m.devp[i], size_t(m.size));
  }
  return ECGPU_OK;
}

// Larger calls with few output bytes: sources cross by HIP's copies (a
// contiguous pageable run goes as one pinned blit at link rate), the kernel
// writes the outputs straight into coherent pinned memory and the calling
// thread copies them out: no per-output pageable D2H (67 us per 1 MiB shard,
// tools/pageable_duplex_probe.cpp).  Returns ECGPU_OK with *done = false when
// the call does not qualify (an output that is also a source, or outputs
// above zc_out_max() / zc_out_shard_max()).
int exec_outputs_zero_copy(Ctx* c, const FusedOp& op, CallMap& m, bool* done) {
  *done = false;
  size_t nout = 0;
  std::vector<char> is_out(m.bufs.size(), 0);
  for (int r = 0; r < m.rows; ++r) {
    const size_t i = m.index(op.dsts[size_t(r)]);
    if (!m.staged[i] || is_out[i]) continue;
    if (i < size_t(m.nsrc)) return ECGPU_OK;  // aliased: keep the staged path
    is_out[i] = 1;
    ++nout;
  }
  if (nout == 0 || nout * size_t(m.size) > zc_out_max() || size_t(m.size) > zc_out_shard_max()) return ECGPU_OK;
  const size_t nin = m.nstage - nout;
  if (int rc = ensure_zc(c, nout * m.slot)) return rc;
  if (int rc = ensure_stage(c, std::max<size_t>(nin, 1) * m.slot)) return rc;
  size_t ni = 0, no = 0;
  std::vector<char*> staged_hp;
  for (size_t i = 0; i < m.bufs.size(); ++i) {
    if (!m.staged[i]) continue;
    if (is_out[i]) {
      m.devp[i] = c->zc + (no++) * m.slot;
    } else {
      m.devp[i] = c->stage + (ni++) * m.slot;
      staged_hp.push_back(static_cast<char*>(m.bufs[i]));
    }
  }
  if (int rc = copy_shards(true, c->stage, m.slot, staged_hp, size_t(m.size), c->stream)) return rc;
  if (writes_in_place(op, m))
    if (int rc = caller_write_point(op, c->device)) return rc;
  if (int rc = launch_and_sync(c, op, m, /*host_io=*/true)) return rc;
  if (int rc = caller_write_point(op, c->device)) return rc;
  for (size_t i = 0; i < m.bufs.size(); ++i)
    if (m.staged[i] && is_out[i]) std::memcpy(m.bufs[i], m.devp[i], size_t(m.size));
  *done = true;
  return ECGPU_OK;
}

// Everything else: staged buffers go through the context's HBM slab, by the
// pinned bounce (mid-size) or HIP's copies (large); non-inline ops (w = 16 /
// 32, > 16 sources, the LDS engine) run a cached bound plan.
int exec_staged(Ctx* c, const FusedOp& op, CallMap& m, bool inl) {
  const size_t slot = m.slot, size = size_t(m.size);
  const int rows = m.rows, nsrc = m.nsrc;
  // With several launches (> 4 rows) an output that is also a source must
  // not be overwritten before the last launch reads it: write to temps.
  const bool via_temp = op.dst_is_src && rows > dev::kMaxRows;
  const size_t ntemp = via_temp ? size_t(rows) : 0;
  if (int rc = ensure_stage(c, (m.nstage + ntemp) * slot)) return rc;
  size_t next = 0;
  for (size_t i = 0; i < m.bufs.size(); ++i)
    if (m.staged[i]) m.devp[i] = c->stage + (next++) * slot;
  // Staged sources take the first staging slots (bufs lists sources first),
  // so with the pinned bounce they go up as one contiguous DMA.
  const bool bounce = m.nstage > 0 && m.nstage * slot <= bounce_max();
  if (bounce)
    if (int rc = ensure_bounce(c, m.nstage * slot)) return rc;
  auto bounce_of = [&](size_t i) { return c->bounce + (m.devp[i] - c->stage); };
  std::vector<char*> staged_hp;
  for (size_t j = 0; j < op.srcs.size(); ++j)
    if (m.staged[j]) {
      staged_hp.push_back(static_cast<char*>(op.srcs[j]));
      if (bounce) std::memcpy(bounce_of(j), op.srcs[j], size);
    }
  if (bounce && !staged_hp.empty()) {
    ECGPU_HIP(hipMemcpyAsync(c->stage, c->bounce, staged_hp.size() * slot, hipMemcpyHostToDevice, c->stream));
  } else if (int rc = copy_shards(true, c->stage, slot, staged_hp, size, c->stream)) {
    return rc;
  }

  const std::vector<const uint8_t*> sp = m.sources();
  std::vector<uint8_t*> dp = m.outputs(op);
  if (via_temp)
    for (int r = 0; r < rows; ++r) dp[size_t(r)] = c->stage + (m.nstage + size_t(r)) * slot;
  if (writes_in_place(op, m))
    if (int rc = caller_write_point(op, c->device)) return rc;
  if (nsrc == 0) {
    // Every output is identically zero (e.g. region multiply by 0 without
    // add, galois.cpp:447-451): nothing to read.
    for (int r = 0; r < rows; ++r) ECGPU_HIP(hipMemsetAsync(dp[size_t(r)], 0, size, c->stream));
  } else if (inl) {
    if (int rc = launch_inline(op, sp, dp, m.size, c->stream, m.host_io)) return rc;
  } else {
    ecgpu_plan* p = nullptr;
    if (int rc = ctx_plan(c, rows, nsrc, op.coef, op.w, &p)) return rc;
    // sp/dp outlive the stream sync below
    if (int rc = plan_bind(p, 1, sp.data(), dp.data(), m.size, c->stream, /*keep_alive=*/true)) return rc;
    if (int rc = plan_launch(p, c->stream)) return rc;
  }
  // staged outputs, in slot order
  std::vector<std::pair<uint8_t*, char*>> outs;  // (device slot, host pointer)
  for (int r = 0; r < rows; ++r) {
    const size_t i = m.index(op.dsts[size_t(r)]);
    if (via_temp)
      ECGPU_HIP(hipMemcpyAsync(m.devp[i], dp[size_t(r)], size, hipMemcpyDeviceToDevice, c->stream));
    if (m.staged[i]) outs.emplace_back(m.devp[i], static_cast<char*>(op.dsts[size_t(r)]));
  }
  std::sort(outs.begin(), outs.end());
  if (bounce) {
    // one D2H per run of adjacent slots (the bounce mirrors the slab)
    for (size_t a = 0; a < outs.size();) {
      size_t b = a + 1;
      while (b < outs.size() && outs[b].first == outs[b - 1].first + slot) ++b;
      const size_t off = size_t(outs[a].first - c->stage);
      ECGPU_HIP(hipMemcpyAsync(c->bounce + off, outs[a].first, (b - a - 1) * slot + size, hipMemcpyDeviceToHost,
                               c->stream));
      a = b;
    }
    ECGPU_HIP(hipStreamSynchronize(c->stream));
    ECGPU_HIP(hipGetLastError());
    if (!outs.empty())
      if (int rc = caller_write_point(op, c->device)) return rc;
    for (const auto& o : outs) std::memcpy(o.second, c->bounce + (o.first - c->stage), size);
    return ECGPU_OK;
  }
  // from here the D2H copies write the caller's outputs directly
  if (!outs.empty())
    if (int rc = caller_write_point(op, c->device)) return rc;
  // outputs in consecutive slots: one 2-D copy per evenly spaced run of host outputs
  bool consecutive = true;
  for (size_t i = 1; i < outs.size() && consecutive; ++i) consecutive = outs[i].first == outs[0].first + i * slot;
  if (consecutive && !outs.empty()) {
    std::vector<char*> hp;
    for (const auto& o : outs) hp.push_back(o.second);
    if (int rc = copy_shards(false, outs[0].first, slot, hp, size, c->stream)) return rc;
  } else {
    for (const auto& o : outs) ECGPU_HIP(hipMemcpyAsync(o.second, o.first, size, hipMemcpyDeviceToHost, c->stream));
  }
  ECGPU_HIP(hipStreamSynchronize(c->stream));
  ECGPU_HIP(hipGetLastError());
  return ECGPU_OK;
}

// Runs a fused op synchronously over `size` bytes of every buffer on
// `device`: maps the buffers, then the cheapest staging mode for the host
// ones (§8 of DESIGN.md; the thresholds are measured, see bounce_max / zc_max
// / zc_out_max).
int execute_on_gpu(const FusedOp& op, int64_t size, int device) {
  CtxLease lease(device);
  if (!lease.c) return lease.rc;
  Ctx* c = lease.c;
  DeviceGuard g(device);
  const bool inl = inline_ok(op, size);
  CallMap m;
  int rc = map_buffers(op, size, device, inl, &m);
  if (rc == ECGPU_OK) rc = injected_failure(device, 0);
  if (rc == ECGPU_OK) {
    bool done = false;
    if (inl && m.nstage > 0 && m.nstage * size_t(size) <= zc_max()) {
      rc = exec_zero_copy(c, op, m);
      done = true;
    } else if (inl && m.nstage > 0 && m.nstage * m.slot > bounce_max()) {
      rc = exec_outputs_zero_copy(c, op, m, &done);
    }
    if (rc == ECGPU_OK && !done) rc = exec_staged(c, op, m, inl);
  }
  // a failure returns with nothing of the call still in flight: a launch or
  // copy queued before the failing step no longer writes caller memory
  // behind the CPU executor's back (cpu_fallback.hpp)
  if (rc != ECGPU_OK) {
    (void)hipStreamSynchronize(c->stream);
    (void)hipGetLastError();
  }
  return rc;
}

Where where(const void* p) {
  hipPointerAttribute_t attr;
  const hipError_t e = hipPointerGetAttributes(&attr, p);
  if (e == hipSuccess)
    return attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged ? Where::kDevice : Where::kHost;
  (void)hipGetLastError();
  // unregistered pageable memory, or no GPU runtime at all (then no device
  // memory can exist); any other failure proves nothing
  return e == hipErrorInvalidValue || e == hipErrorNoDevice || e == hipErrorInsufficientDriver ? Where::kHost
                                                                                                : Where::kUnknown;
}

bool all_host(const std::vector<void*>& bufs) {
  for (void* p : bufs)
    if (where(p) != Where::kHost) return false;
  return true;
}

bool all_host(const FusedOp& op) { return all_host(op.srcs) && all_host(op.dsts); }

// execute_on_gpu under SURVEY §8b's failure contract (cpu_fallback.hpp): a
// HIP error on a call whose buffers are all host memory, before it wrote a
// source (an output that is also one), completes on the CPU
// (ECGPU_CPU_FALLBACK, default on); a device marked lost by a sticky error
// sends such calls straight there.
int execute_on(const FusedOp& op, int64_t size, int device, const char* call) {
  trace_begin();
  CallDeviceScope scope(device);
  const bool fallback = fallback_enabled();
  if (fallback && device_lost(device) && all_host(op)) {
    record_fallback(call, "device " + std::to_string(device) + " marked lost by an earlier HIP error");
    cpu_apply(op, size);
    return ECGPU_OK;
  }
  const int rc = execute_on_gpu(op, size, device);
  if (rc != ECGPU_ERR_HIP || !fallback || caller_written() || !all_host(op)) return rc;
  record_fallback(call, "HIP error: " + t_err);
  cpu_apply(op, size);
  t_err = std::string(call) + ": completed on the CPU after a HIP error: " + t_err;
  return ECGPU_OK;
}

// ------------------------------------------------------- split calls ----
// A synchronous call on host memory can be cut into contiguous 16-B-aligned
// byte ranges that run concurrently, each on its own context (thread, stream,
// staging) and device.  Every byte column of a fused op is independent -- a
// column's outputs depend on that column of the sources only, identical
// buffers included -- so the ranges' bytes are the call's.  This is the
// reference client's own split (encode_mul_thread, client_main.cpp:1074-1164)
// done inside one call, and SURVEY §8e's "one huge stripe: contiguous byte
// ranges of S/N" over the visible GPUs: each range crosses its own PCIe link.
// ECGPU_SPLIT: 0 off (default), -1 one range per visible device (or per entry
// of ECGPU_DEVICES), N > 0 N ranges over the devices in turn (N > 1 on one
// GPU: N contexts on it; a forced ECGPU_DEVICE keeps them all there);
// ranges are at least ECGPU_SPLIT_MIN_KIB.  Calls with a device buffer stay
// whole (the buffer fixes the device).
int split_ways(const FusedOp& op, int64_t size, int* ndev) {
  const int v = knob(Knob::kSplit);
  if (v == 0) return 1;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
    (void)hipGetLastError();
    return 1;
  }
  *ndev = n;
  const int64_t min_bytes = int64_t(std::max(16, knob(Knob::kSplitMinKib))) << 10;
  const auto list = device_list();
  const int per_device = list && !list->empty() ? int(list->size()) : n;  // -1: one range per listed / visible device
  const int ways = int(std::min<int64_t>(v < 0 ? per_device : v, size / min_bytes));
  if (ways <= 1) return 1;
  return all_host(op) ? ways : 1;
}

FusedOp shifted(const FusedOp& op, int64_t off) {
  FusedOp s;
  for (void* p : op.srcs) s.srcs.push_back(static_cast<char*>(p) + off);
  for (void* p : op.dsts) s.dsts.push_back(static_cast<char*>(p) + off);
  s.coef = op.coef;
  s.w = op.w;
  s.dst_is_src = op.dst_is_src;
  return s;
}

int execute_split(const FusedOp& op, int64_t size, int ways, int ndev, const char* call) {
  const int64_t per = (size / ways) & ~int64_t(15);  // whole words at w = 16 / 32
  const int first = current_device();
  // range i's device: a forced ECGPU_DEVICE keeps every range on it (N
  // contexts there); an ECGPU_DEVICES list is walked from this thread's entry;
  // otherwise every visible device in turn from the current one
  const int forced = forced_device();
  const auto list = device_list();
  size_t list_pos = 0;
  if (forced < 0 && list && !list->empty()) {
    const int mine = host_call_device();
    list_pos = size_t(std::find(list->begin(), list->end(), mine) - list->begin()) % list->size();
  }
  auto range_device = [&](int i) {
    if (forced >= 0) return forced;
    if (list && !list->empty()) return (*list)[(list_pos + size_t(i)) % list->size()];
    return (first + i) % ndev;
  };
  std::vector<int> rc(size_t(ways), ECGPU_OK);
  std::vector<std::string> msg(static_cast<size_t>(ways));
  auto run = [&](int i) {
    const int64_t off = per * i, len = i + 1 < ways ? per : size - off;
    rc[size_t(i)] = execute_on(shifted(op, off), len, range_device(i), call);
    if (rc[size_t(i)]) msg[size_t(i)] = t_err;
  };
  std::vector<std::thread> workers;
  int next = 1;
  try {
    for (; next < ways; ++next) workers.emplace_back(run, next);
  } catch (const std::system_error&) {  // no thread: the rest run here, in turn
  }
  run(0);
  for (int i = next; i < ways; ++i) run(i);
  for (auto& t : workers) t.join();
  for (int i = 0; i < ways; ++i)
    if (rc[size_t(i)])
      return fail(rc[size_t(i)], msg[size_t(i)] + " (byte range " + std::to_string(per * i) + " of a call split " +
                                     std::to_string(ways) + " ways)");
  return ECGPU_OK;
}

// Distinct buffers x size: the bytes a call reads and writes once each.
int64_t bytes_moved(const FusedOp& op, int64_t size) {
  size_t n = op.srcs.size();
  for (void* d : op.dsts)
    if (std::find(op.srcs.begin(), op.srcs.end(), d) == op.srcs.end()) ++n;
  return int64_t(n) * size;
}

// Host-memory synchronous calls in flight on each device's link (the PCIe
// link a staged or zero-copy call moves its bytes over).  One such call
// already runs the link at its ceiling (2 concurrent C3 4 MiB pageable
// encodes: 36.0 GiB/s together against 34.3 alone), so with ECGPU_LINK_CALLS
// (default 1) calls in flight, a further one runs on the CPU executor on its
// own thread instead of queueing for the link: concurrent
// callers then add cores rather than wait.
constexpr int kLinkSlots = 64;
std::atomic<int> g_link_calls[kLinkSlots];

struct LinkScope {
  int slot = -1;
  LinkScope(int device, bool host_io) {
    if (host_io && device >= 0) {
      slot = device % kLinkSlots;
      g_link_calls[slot].fetch_add(1, std::memory_order_relaxed);
    }
  }
  ~LinkScope() {
    if (slot >= 0) g_link_calls[slot].fetch_sub(1, std::memory_order_relaxed);
  }
  LinkScope(const LinkScope&) = delete;
  LinkScope& operator=(const LinkScope&) = delete;
};

bool link_busy(int device) {
  const int limit = knob(Knob::kLinkCalls);
  return limit > 0 && device >= 0 && g_link_calls[device % kLinkSlots].load(std::memory_order_relaxed) >= limit;
}

// A synchronous call over `size` bytes of every buffer of the fused op.
int execute(const FusedOp& op, int64_t size, const char* call) {
  if (op.w != 8 && size % (op.w / 8) != 0)
    return fail(ECGPU_ERR_ARG, "w = " + std::to_string(op.w) + ": size must be a multiple of the word size");
  // identical or disjoint buffers, checked before anything touches the GPU
  if (int rc = check_op_buffers(call, op, size)) return rc;
  add_stats(op);
  if (op.dsts.empty() || size <= 0) return ECGPU_OK;
  // small host-memory calls (and all of them with ECGPU_GPU=0) on the CPU
  // executor: below the crossover the GPU round trip costs more than the
  // arithmetic (cpu_fallback.hpp)
  // (pointer classification costs ~0.15 us a buffer: only when a rule needs it)
  const bool small = cpu_by_choice(bytes_moved(op, size));
  const bool host = (small || knob(Knob::kLinkCalls) > 0) && all_host(op);
  if (small && host) {
    record_cpu_call();
    cpu_apply(op, size);
    return ECGPU_OK;
  }
  int ndev = 1;
  const int ways = split_ways(op, size, &ndev);
  if (ways > 1) return execute_split(op, size, ways, ndev, call);
  const int device = call_device(op.srcs, op.dsts);
  if (host && link_busy(device)) {  // the link is taken: this caller's core does the work
    record_cpu_call();
    cpu_apply(op, size);
    return ECGPU_OK;
  }
  LinkScope link(device, host);
  return execute_on(op, size, device, call);
}

ECGPU_RT_END
// ================================================================ C ABI ====
extern "C" {


ECGPU_API ecgpu_plan* ecgpu_plan_create(int rows, int nsrc, const int* coefs, int device) {
  if (rows <= 0 || nsrc <= 0 || !coefs) {
    fail(ECGPU_ERR_ARG, "ecgpu_plan_create: rows, nsrc > 0 and coefs required");
    return nullptr;
  }
  if (device < 0) device = current_device();
  auto* p = new ecgpu_plan();
  if (plan_init(p, rows, nsrc, coefs, device) != ECGPU_OK) {
    plan_free(p);
    return nullptr;
  }
  return p;
}

ECGPU_API int ecgpu_plan_bind(ecgpu_plan* p, int stripes, const uint8_t* const* src_ptrs, uint8_t* const* dst_ptrs,
                              int64_t size) {
  if (!p || stripes < 0 || size < 0 || (stripes && (!src_ptrs || !dst_ptrs)))
    return fail(ECGPU_ERR_ARG, "ecgpu_plan_bind: bad arguments");
  if (int rc = ecgpu_plan_check_buffers(p->rows, p->nsrc, stripes, src_ptrs, dst_ptrs, size)) return rc;
  return plan_bind(p, stripes, src_ptrs, dst_ptrs, size, nullptr);
}

ECGPU_API int ecgpu_plan_set_kernel(ecgpu_plan* p, int kind, int nontemporal) {
  if (!p || (kind != ECGPU_KERNEL_PERM && kind != ECGPU_KERNEL_LDS))
    return fail(ECGPU_ERR_ARG, "ecgpu_plan_set_kernel: bad arguments");
  p->kind = kind;
  p->nt = std::min(kStorePolicies - 1, std::max(0, nontemporal));
  return ECGPU_OK;
}

ECGPU_API int ecgpu_plan_launch(ecgpu_plan* p, void* stream) {
  if (!p) return fail(ECGPU_ERR_ARG, "ecgpu_plan_launch: null plan");
  return plan_launch(p, static_cast<hipStream_t>(stream));
}

ECGPU_API void ecgpu_plan_destroy(ecgpu_plan* p) { plan_free(p); }

ECGPU_API int ecgpu_set_devices(int n, const int* devices) {
  if (n < 0 || (n > 0 && !devices)) return fail(ECGPU_ERR_ARG, "ecgpu_set_devices: bad arguments");
  for (int i = 0; i < n; ++i)
    if (devices[i] < 0) return fail(ECGPU_ERR_ARG, "ecgpu_set_devices: negative device");
  const int visible = visible_devices();
  if (const int bad = invisible_entry(std::vector<int>(devices, devices + n), visible); bad >= 0)
    return fail(ECGPU_ERR_ARG, "ecgpu_set_devices: device " + std::to_string(bad) + " is not visible (" +
                                   std::to_string(visible) + " visible)");
  (void)device_list();  // the environment's list is read first, so this call overrides it
  std::lock_guard<std::mutex> lk(g_devices_mu);
  g_devices = n > 0 ? std::make_shared<const std::vector<int>>(devices, devices + n) : nullptr;
  return ECGPU_OK;
}

ECGPU_API int ecgpu_get_devices(int* out, int cap) {
  const auto list = device_list();
  const int n = list ? int(list->size()) : 0;
  for (int i = 0; i < n && i < cap && out; ++i) out[i] = (*list)[size_t(i)];
  return n;
}

ECGPU_API int ecgpu_call_device(void) { return host_call_device(); }

ECGPU_API int ecgpu_device_pci_bus_id(int device, char* buf, int len) {
  if (!buf || len < 13) return fail(ECGPU_ERR_ARG, "ecgpu_device_pci_bus_id: buffer of >= 13 bytes required");
  ECGPU_HIP(hipDeviceGetPCIBusId(buf, len, device));
  return ECGPU_OK;
}

ECGPU_API int ecgpu_host_register(void* ptr, int64_t bytes) {
  if (!ptr || bytes <= 0) return fail(ECGPU_ERR_ARG, "ecgpu_host_register: bad arguments");
  ECGPU_HIP(hipHostRegister(ptr, size_t(bytes), hipHostRegisterDefault));
  return ECGPU_OK;
}

ECGPU_API int ecgpu_host_unregister(void* ptr) {
  if (!ptr) return fail(ECGPU_ERR_ARG, "ecgpu_host_unregister: null");
  ECGPU_HIP(hipHostUnregister(ptr));
  return ECGPU_OK;
}

ECGPU_API int ecgpu_encode_batch(int k, int m, const int* matrix, int stripes, const uint8_t* const* data,
                                 uint8_t* const* coding, int64_t size, void* stream) {
  if (k <= 0 || m <= 0 || !matrix || stripes < 0 || size < 0 || (stripes && (!data || !coding)))
    return fail(ECGPU_ERR_ARG, "ecgpu_encode_batch: bad arguments");
  if (int rc = ecgpu_plan_check_buffers(m, k, stripes, data, coding, size)) return rc;
  ecgpu_plan* p = ecgpu_plan_create(m, k, matrix, -1);
  if (!p) return ECGPU_ERR_HIP;
  int rc = plan_bind(p, stripes, data, coding, size, static_cast<hipStream_t>(stream));
  if (rc == ECGPU_OK) rc = plan_launch(p, static_cast<hipStream_t>(stream));
  if (rc == ECGPU_OK && stream) {
    hipError_t e = hipStreamSynchronize(static_cast<hipStream_t>(stream));
    if (e != hipSuccess) rc = fail(ECGPU_ERR_HIP, hipGetErrorString(e));
  } else if (rc == ECGPU_OK) {
    hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) rc = fail(ECGPU_ERR_HIP, hipGetErrorString(e));
  }
  plan_free(p);
  return rc;
}

namespace {
bool valid_w(int w) { return w == 8 || w == 16 || w == 32; }
}  // namespace

ECGPU_API int ecgpu_jerasure_matrix_encode(int k, int m, int w, int* matrix, char** data_ptrs, char** coding_ptrs,
                                           int size) {
  if (!valid_w(w)) return fail(ECGPU_ERR_ARG, "ecgpu_jerasure_matrix_encode: w must be 8, 16 or 32");
  LinearTracker t(w);
  plan_encode(t, k, m, matrix, data_ptrs, coding_ptrs, size);
  return execute(t.finish(), size, "jerasure_matrix_encode");
}

ECGPU_API int ecgpu_jerasure_matrix_decode(int k, int m, int w, int* matrix, int row_k_ones, int* erasures,
                                           char** data_ptrs, char** coding_ptrs, int size) {
  if (!valid_w(w)) return ECGPU_ERR;  // jerasure.cpp:165: any other w returns -1
  LinearTracker t(w);
  if (plan_decode(t, k, m, matrix, row_k_ones, erasures, data_ptrs, coding_ptrs, size) < 0) return ECGPU_ERR;
  return execute(t.finish(), size, "jerasure_matrix_decode");
}

ECGPU_API int ecgpu_jerasure_matrix_dotprod(int k, int w, int* matrix_row, int* src_ids, int dest_id,
                                            char** data_ptrs, char** coding_ptrs, int size) {
  if (w == 1) {
    // jerasure.cpp:561-620 at w = 1: coefficient 1 copies (first) or XORs the
    // source; any other non-zero coefficient has no region multiply at w = 1
    // (the reference's switch has no case for it) but still counts its bytes
    // as gf and marks the destination initialised.  So the map is the XOR of
    // the unit-coefficient sources -- the XOR-only kernel over GF(2^8)
    // bytes, where 1 * x = x.
    LinearTracker t(8);
    auto buf = [&](int i) -> void* {
      const int id = src_ids ? src_ids[i] : i;
      return id < k ? static_cast<void*>(data_ptrs[id]) : static_cast<void*>(coding_ptrs[id - k]);
    };
    void* dst = dest_id < k ? static_cast<void*>(data_ptrs[dest_id]) : static_cast<void*>(coding_ptrs[dest_id - k]);
    bool init = false;
    for (int i = 0; i < k; ++i) {
      if (matrix_row[i] != 1) continue;
      if (!init) {
        t.copy(dst, buf(i));
        t.count(0, 0, double(size));
        init = true;
      } else {
        t.xor3(buf(i), dst, dst);
        t.count(double(size), 0, 0);
      }
    }
    for (int i = 0; i < k; ++i)
      if (matrix_row[i] != 0 && matrix_row[i] != 1) t.count(0, double(size), 0);
    return execute(t.finish(), size, "jerasure_matrix_dotprod");
  }
  if (!valid_w(w)) return fail(ECGPU_ERR_ARG, "ecgpu_jerasure_matrix_dotprod: w must be 1, 8, 16 or 32");
  LinearTracker t(w);
  t.dotprod(k, matrix_row, src_ids, dest_id, data_ptrs, coding_ptrs, size);
  return execute(t.finish(), size, "jerasure_matrix_dotprod");
}

ECGPU_API int ecgpu_jerasure_do_parity(int k, char** data_ptrs, char* parity_ptr, int size) {
  LinearTracker t;
  t.copy(parity_ptr, data_ptrs[0]);
  for (int i = 1; i < k; ++i) t.xor3(data_ptrs[i], parity_ptr, parity_ptr);
  t.count(double(size) * (k - 1), 0, double(size));
  return execute(t.finish(), size, "jerasure_do_parity");
}

ECGPU_API int ecgpu_galois_w08_region_multiply(char* region, int multby, int nbytes, char* r2, int add) {
  LinearTracker t;
  if (r2 == nullptr)
    t.mul(region, multby, region, false);  // galois.cpp:429,447: in place, add ignored
  else
    t.mul(region, multby, r2, add != 0);
  return execute(t.finish(), nbytes, "galois_w08_region_multiply");
}

// galois.cpp:469-542: nbytes/2 words; multby 0 zeroes (no add) or does
// nothing (add); in place (r2 NULL) ignores add.
ECGPU_API int ecgpu_galois_w16_region_multiply(char* region, int multby, int nbytes, char* r2, int add) {
  LinearTracker t(16);
  char* dst = r2 ? r2 : region;
  if (multby == 0) {
    if (!add) t.mul(region, 0, dst, false);
  } else {
    t.mul(region, multby, dst, r2 != nullptr && add != 0);
  }
  return execute(t.finish(), nbytes & ~1, "galois_w16_region_multiply");
}

// galois.cpp:666-727: nbytes/4 words; add applies even in place.
ECGPU_API int ecgpu_galois_w32_region_multiply(char* region, int multby, int nbytes, char* r2, int add) {
  LinearTracker t(32);
  t.mul(region, multby, r2 ? r2 : region, add != 0);
  return execute(t.finish(), nbytes & ~3, "galois_w32_region_multiply");
}

ECGPU_API int ecgpu_galois_region_xor(char* r1, char* r2, char* r3, int nbytes) {
  LinearTracker t;
  t.xor3(r1, r2, r3);
  return execute(t.finish(), nbytes, "galois_region_xor");
}

ECGPU_API int ecgpu_reed_sol_galois_w08_region_multby_2(char* region, int nbytes) {
  LinearTracker t;
  t.mul(region, 2, region, false);
  return execute(t.finish(), nbytes);
}

// reed_sol.cpp:158-198 / :90-106 (whole words).
ECGPU_API int ecgpu_reed_sol_galois_w16_region_multby_2(char* region, int nbytes) {
  LinearTracker t(16);
  t.mul(region, 2, region, false);
  return execute(t.finish(), nbytes & ~1);
}

ECGPU_API int ecgpu_reed_sol_galois_w32_region_multby_2(char* region, int nbytes) {
  LinearTracker t(32);
  t.mul(region, 2, region, false);
  return execute(t.finish(), nbytes & ~3);
}

// reed_sol.cpp:200-225: P = XOR of data; Q = Horner sum of 2^j d_j.
// Returns 1, or 0 for a w the reference does not handle.
ECGPU_API int ecgpu_reed_sol_r6_encode(int k, int w, char** data_ptrs, char** coding_ptrs, int size) {
  if (!valid_w(w)) return 0;
  LinearTracker t(w);
  t.copy(coding_ptrs[0], data_ptrs[0]);
  for (int i = 1; i < k; ++i) t.xor3(coding_ptrs[0], data_ptrs[i], coding_ptrs[0]);
  t.copy(coding_ptrs[1], data_ptrs[k - 1]);
  for (int i = k - 2; i >= 0; --i) {
    t.mul(coding_ptrs[1], 2, coding_ptrs[1], false);
    t.xor3(coding_ptrs[1], data_ptrs[i], coding_ptrs[1]);
  }
  const int rc = execute(t.finish(), size, "reed_sol_r6_encode");
  return rc == ECGPU_OK ? 1 : rc;
}

ECGPU_API int ecgpu_jerasure_get_stats(double* fill_in) {
  std::lock_guard<std::mutex> lk(g_stats_mu);
  for (int i = 0; i < 3; ++i) {
    fill_in[i] = g_stats[i];
    g_stats[i] = 0;
  }
  return ECGPU_OK;
}

}  // extern "C"
