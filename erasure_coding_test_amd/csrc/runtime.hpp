// runtime.hpp -- internal interface shared by the runtime's translation
// units (not installed; the public surface is include/ecgpu.h):
//   ecgpu_runtime.hip  plans, kernel dispatch, contexts, staging of host
//                      buffers, synchronous calls and their C ABI
//   accum.hip          HBM-resident ECX parity accumulators
//   pipeline.hip       host-memory pipelines and multi-device groups
//   packets.hip        GF(2) bit-matrix / schedule coding
// Everything here lives in ecgpu::rt with hidden visibility: the shared
// library exports only the ECGPU_API functions.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <list>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "ecgpu.h"
#include "gf_kernels.hpp"
#include "knobs.hpp"
#include "planner.hpp"

#define ECGPU_RT_BEGIN \
  namespace ecgpu {    \
  namespace __attribute__((visibility("hidden"))) rt {
#define ECGPU_RT_END \
  }                  \
  }

// A bound coefficient matrix (ecgpu_plan_* in include/ecgpu.h).
struct ecgpu_plan {
  int device = 0, rows = 0, nsrc = 0, w = 8;
  int kind = ECGPU_KERNEL_PERM, nt = 1;
  std::vector<uint32_t> coef;  // host copy, rows x nsrc
  // one device allocation for all coefficient tables, carved below
  uint8_t* d_tabs = nullptr;
  ecgpu::dev::u32x4* d_q = nullptr;
  uint32_t* d_p3 = nullptr;    // 3-bit-slice tables, kP3Words per coefficient
  uint8_t* d_nib = nullptr;
  uint32_t* d_w = nullptr;     // wide-word tables (w = 16 / 32)
  uint8_t* d_wcls = nullptr;   // wide coefficient classes
  uint32_t* d_wnib = nullptr;  // wide-word LDS nibble tables, kNibWords per coefficient
  int stripes = 0;
  int64_t size = 0;
  bool aligned = true;
  // one device allocation for the pointer tables: sources, then destinations
  void** d_ptrs = nullptr;
  size_t cap_ptrs = 0;
  const uint8_t** d_src = nullptr;
  uint8_t** d_dst = nullptr;
  // the coefficient tables go up asynchronously on the device's upload
  // stream (plan_init); launches wait for `uploaded` until it has completed.
  // host_tabs is the copy's source, kept until then.
  hipEvent_t uploaded = nullptr;
  bool upload_pending = false;
  std::vector<uint8_t> host_tabs;
};

ECGPU_RT_BEGIN

// ---- errors and knobs -------------------------------------------------------
extern thread_local std::string t_err;  // ecgpu_last_error()
int fail(int code, const std::string& msg);  // knobs: knobs.hpp

// A HIP failure: ECGPU_ERR_HIP with the message; an error that leaves the
// device's context unusable (sticky: a kernel fault, a lost or missing
// device) also marks the device lost (cpu_fallback.hpp) -- the device the
// current synchronous call targets (CallDeviceScope), else the current one.
int fail_hip(hipError_t e, const char* what);

// Names the device a synchronous call runs on for fail_hip, for its lifetime.
struct CallDeviceScope {
  int prev;
  explicit CallDeviceScope(int device);
  ~CallDeviceScope();
  CallDeviceScope(const CallDeviceScope&) = delete;
  CallDeviceScope& operator=(const CallDeviceScope&) = delete;
};

// Where a buffer lives: host memory (pageable, pinned or registered), device
// (or managed) memory, or unknown (the pointer query failed for a reason that
// does not prove host memory -- e.g. a sticky error; the CPU must not touch it).
enum class Where { kHost, kDevice, kUnknown };
Where where(const void* p);
// Every buffer host memory, positively known (the CPU executor may run the call).
bool all_host(const std::vector<void*>& bufs);

#define ECGPU_HIP(expr)                                 \
  do {                                                  \
    hipError_t e_ = (expr);                             \
    if (e_ != hipSuccess) return ::ecgpu::rt::fail_hip(e_, #expr); \
  } while (0)

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

int current_device();
// The device a synchronous call on these buffers runs on (ECGPU_DEVICE,
// ECGPU_DEVICES, or the current device; ecgpu_runtime.hip).
int call_device(const std::vector<void*>& a, const std::vector<void*>& b);

// ---- kernel launches -----------------------------------------------------------
using KernelFn = void (*)(ecgpu::dev::ApplyArgs);

inline hipError_t launch(KernelFn fn, dim3 grid, dim3 block, ecgpu::dev::ApplyArgs& a, hipStream_t s,
                         unsigned lds_bytes = 0) {
  void* args[] = {&a};
  return hipLaunchKernel(reinterpret_cast<const void*>(fn), grid, block, args, lds_bytes, s);
}

// dispatch_w8.hip: which compile-time unit structure holds exactly for rows
// [r0, r0 + R) (gf_kernels_w8.hpp UnitMask index), the residency cap's
// dynamic LDS bytes for a launch streaming `streams` shards per lane, and
// whether a launch takes the cap
int unit_variant(const std::vector<uint32_t>& coef, int K, int r0, int R);
unsigned residency_lds_bytes(int device, int streams, unsigned static_bytes = 0);
bool cap_for(int K, int R, int mul_terms);

// ---- plans --------------------------------------------------------------------
void plan_free(ecgpu_plan* p);
// one asynchronous upload of a plan's coefficient tables (ecgpu_runtime.hip);
// launches wait for it through plan_wait_tables
int plan_upload_tables(ecgpu_plan* p, std::vector<uint8_t>&& host);
int plan_wait_tables(ecgpu_plan* p, hipStream_t stream);
// the width-specific halves of plan_init / plan_launch (dispatch_w8.hip,
// dispatch_wide.hip); p->coef is sized rows x nsrc
int plan_init_w8(ecgpu_plan* p, const int* coefs);
int plan_init_wide(ecgpu_plan* p, const int* coefs);
int plan_launch_wide(ecgpu_plan* p, hipStream_t stream);
int plan_init(ecgpu_plan* p, int rows, int nsrc, const int* coefs, int device, int w = 8);
// With a stream the pointer tables are uploaded asynchronously on it; unless
// `keep_alive` (the caller keeps src/dst alive until it synchronises the
// stream) the call waits for the upload.
int plan_bind(ecgpu_plan* p, int stripes, const uint8_t* const* src, uint8_t* const* dst, int64_t size,
              hipStream_t stream, bool keep_alive = false);
int plan_launch(ecgpu_plan* p, hipStream_t stream);

// ---- contexts of the synchronous calls ----------------------------------------
struct PlanKey {
  int rows, nsrc, w, kind, nt;  // kind / nt: the engine and store-policy knobs the plan was made under
  std::vector<uint32_t> coef;
  bool operator==(const PlanKey& o) const {
    return rows == o.rows && nsrc == o.nsrc && w == o.w && kind == o.kind && nt == o.nt && coef == o.coef;
  }
};

struct Ctx {
  int device = -1;
  hipStream_t stream = nullptr;
  uint8_t* stage = nullptr;
  size_t stage_cap = 0;
  uint8_t* bounce = nullptr;  // pinned host mirror of the staging slab (mid-size calls, see execute)
  size_t bounce_cap = 0;
  uint8_t* zc = nullptr;      // coherent pinned memory the kernel reads / writes in place (small calls)
  size_t zc_cap = 0;
  std::list<std::pair<PlanKey, ecgpu_plan*>> plans;  // LRU, front = newest
};

Ctx* acquire_ctx(int device, int* rc);
void release_ctx(Ctx* c);

struct CtxLease {
  int rc = ECGPU_OK;  // declared first: initialised before acquire_ctx writes it
  Ctx* c = nullptr;
  explicit CtxLease(int device) : c(acquire_ctx(device, &rc)) {}
  ~CtxLease() {
    if (c) release_ctx(c);
  }
};

int ctx_plan(Ctx* c, int rows, int nsrc, const std::vector<uint32_t>& coef, int w, ecgpu_plan** out);
int ensure_bounce(Ctx* c, size_t bytes);
int ensure_zc(Ctx* c, size_t bytes);
int ensure_stage(Ctx* c, size_t bytes);

// ---- host memory --------------------------------------------------------------
bool zero_copy_pinned();
int classify(const void* p, int device, bool* on_device);
bool host_mapped(const void* p, size_t bytes, void** dev);
bool is_pinned(const void* p);
int copy_shards(bool h2d, uint8_t* d0, size_t dstride, const std::vector<char*>& hp, size_t bytes, hipStream_t s);

// ---- synchronous execution ----------------------------------------------------
void add_stats(const FusedOp& op);
bool inline_ok(const FusedOp& op, int64_t size);
int launch_inline(const FusedOp& op, const std::vector<const uint8_t*>& sp, const std::vector<uint8_t*>& dp,
                  int64_t size, hipStream_t s, bool host_io);
// Runs a fused op synchronously; `call` names the entry point in errors
// (e.g. a buffer-contract rejection, buffer_contract.hpp).
int execute(const FusedOp& op, int64_t size, const char* call = "ecgpu");

ECGPU_RT_END
