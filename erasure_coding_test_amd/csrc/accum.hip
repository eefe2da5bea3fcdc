// accum.hip -- HBM-resident ECX parity accumulators (ecgpu_accum_* in
// include/ecgpu.h): the ECX datanode's per-block update
// (ecx_datanode_main.cpp:680-735) as one fused launch per arriving block.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "buffer_contract.hpp"
#include "ecgpu.h"
#include "gf_host.hpp"
#include "matrix_host.hpp"
#include "planner.hpp"
#include "schedule_host.hpp"
#include "runtime.hpp"

using namespace ecgpu;
using namespace ecgpu::rt;

extern "C" {

// ---------------------------------------------------- ECX accumulators ----
struct ecgpu_accum {
  int device = 0, m = 0;
  int64_t size = 0;
  size_t slot = 0;
  uint8_t* d_acc = nullptr;  // m slots, each `slot` bytes (skewed shard stride)
  std::vector<char> init;
  // queued adds (ecgpu_accum_add_async): a host block is copied into the
  // device block buffer and applied, both on the accumulator's own stream,
  // and the call returns; the copy of block j+1 queues behind the update of
  // block j (stream order protects the buffer) with no host round trip
  uint8_t* d_blk = nullptr;
  hipStream_t stream = nullptr;
  bool pending = false;  // queued work not yet synchronised
};

}  // extern "C"

namespace {

// The reference's per-accumulator update (ecx_datanode_main.cpp:699-735) for
// one arriving block as ONE fused op: coefficient 0 leaves an accumulator
// alone, 1 copies (first touch) or XORs, any other multiplies (first touch)
// or multiply-adds.
FusedOp accum_op(ecgpu_accum* a, const char* block, const int* coefs) {
  LinearTracker t;
  char* src = const_cast<char*>(block);
  for (int i = 0; i < a->m; ++i) {
    const int c = coefs[i] & 0xFF;
    if (c == 0) continue;
    char* acc = ecgpu_accum_device_ptr(a, i);
    if (c == 1) {
      if (a->init[i])
        t.xor3(src, acc, acc);
      else
        t.copy(acc, src);
    } else {
      t.mul(src, c, acc, a->init[i] != 0);
    }
  }
  return t.finish();
}

int accum_sync(ecgpu_accum* a) {
  if (!a->pending) return ECGPU_OK;
  ECGPU_HIP(hipStreamSynchronize(a->stream));
  ECGPU_HIP(hipGetLastError());
  a->pending = false;
  return ECGPU_OK;
}

int accum_async_init(ecgpu_accum* a) {
  if (a->stream) return ECGPU_OK;
  DeviceGuard g(a->device);
  ECGPU_HIP(hipMalloc(reinterpret_cast<void**>(&a->d_blk), a->slot));
  // a blocking stream: ordered after the caller's null-stream work like every
  // synchronous call (a device-resident block filled by PyTorch, say)
  ECGPU_HIP(hipStreamCreateWithFlags(&a->stream, hipStreamDefault));
  return ECGPU_OK;
}

}  // namespace

extern "C" {

ECGPU_API ecgpu_accum* ecgpu_accum_create(int m, int64_t size, int device) {
  if (m <= 0 || size < 0) {
    fail(ECGPU_ERR_ARG, "ecgpu_accum_create: m > 0 and size >= 0 required");
    return nullptr;
  }
  auto* a = new ecgpu_accum();
  a->device = device < 0 ? current_device() : device;
  a->m = m;
  a->size = size;
  a->slot = size_t(ecgpu_recommended_shard_stride(size));
  a->init.assign(size_t(m), 0);
  DeviceGuard g(a->device);
  hipError_t e = hipMalloc(reinterpret_cast<void**>(&a->d_acc), a->slot * size_t(m));
  if (e != hipSuccess) {
    fail(ECGPU_ERR_HIP, std::string("ecgpu_accum_create: ") + hipGetErrorString(e));
    delete a;
    return nullptr;
  }
  return a;
}

ECGPU_API char* ecgpu_accum_device_ptr(ecgpu_accum* a, int i) {
  if (!a || i < 0 || i >= a->m) return nullptr;
  return reinterpret_cast<char*>(a->d_acc + size_t(i) * a->slot);
}

ECGPU_API int ecgpu_accum_add(ecgpu_accum* a, const char* block, const int* coefs) {
  if (!a || !block || !coefs) return fail(ECGPU_ERR_ARG, "ecgpu_accum_add: bad arguments");
  if (int rc = accum_sync(a)) return rc;  // after every earlier asynchronous add
  DeviceGuard g(a->device);
  const int rc = execute(accum_op(a, block, coefs), a->size, "ecgpu_accum_add");
  if (rc != ECGPU_OK) return rc;
  for (int i = 0; i < a->m; ++i)
    if (coefs[i] & 0xFF) a->init[i] = 1;
  return ECGPU_OK;
}

// Queued add: the block's H2D copy (host blocks, into the device block
// buffer) and its fused update go onto the accumulator's stream and the
// call returns, so consecutive blocks stream over PCIe back to back with no
// host round trip per block.  (A second copy stream overlapping block j+1's
// H2D with block j's ~6 us update measured slower: the cross-stream event
// waits cost more than the overlap buys)  The block must stay
// valid and unchanged until ecgpu_accum_sync (or a read, a reset, a
// synchronous add) returns.
ECGPU_API int ecgpu_accum_add_async(ecgpu_accum* a, const char* block, const int* coefs) {
  if (!a || !block || !coefs) return fail(ECGPU_ERR_ARG, "ecgpu_accum_add_async: bad arguments");
  bool any = false;
  for (int i = 0; i < a->m; ++i) any |= (coefs[i] & 0xFF) != 0;
  if (!any || a->size == 0) return ECGPU_OK;
  // a block that shares bytes with an accumulator it updates: rejected
  // before anything is queued (buffer_contract.hpp)
  if (int rc = check_op_buffers("ecgpu_accum_add_async", accum_op(a, block, coefs), a->size)) return rc;
  if (int rc = accum_async_init(a)) return rc;
  DeviceGuard g(a->device);
  bool on_dev = false;
  if (int rc = classify(block, a->device, &on_dev)) return rc;
  const char* src = block;
  void* mapped = nullptr;
  bool in_place = false;
  if (!on_dev && zero_copy_pinned() && host_mapped(block, size_t(a->size), &mapped)) {
    src = static_cast<const char*>(mapped);  // pinned: the update kernel reads it in place over PCIe
    in_place = true;
  } else if (!on_dev) {
    ECGPU_HIP(hipMemcpyAsync(a->d_blk, block, size_t(a->size), hipMemcpyHostToDevice, a->stream));
    src = reinterpret_cast<const char*>(a->d_blk);
  }
  a->pending = true;
  const FusedOp op = accum_op(a, src, coefs);
  if (inline_ok(op, a->size)) {
    add_stats(op);
    std::vector<const uint8_t*> sp;
    for (void* p : op.srcs) sp.push_back(static_cast<const uint8_t*>(p));
    std::vector<uint8_t*> dp;
    for (void* p : op.dsts) dp.push_back(static_cast<uint8_t*>(p));
    if (int rc = launch_inline(op, sp, dp, a->size, a->stream, /*host_io=*/in_place)) return rc;
  } else {
    // engine override or > 4 aliased rows: the synchronous path, which
    // classifies and maps host memory itself -- so it gets the caller's
    // pointer, not the device alias of a pinned block
    if (int rc = accum_sync(a)) return rc;
    if (int rc = execute(in_place ? accum_op(a, block, coefs) : op, a->size, "ecgpu_accum_add_async")) return rc;
  }
  for (int i = 0; i < a->m; ++i)
    if (coefs[i] & 0xFF) a->init[i] = 1;
  return ECGPU_OK;
}

ECGPU_API int ecgpu_accum_sync(ecgpu_accum* a) {
  if (!a) return fail(ECGPU_ERR_ARG, "ecgpu_accum_sync: null");
  return accum_sync(a);
}

ECGPU_API int ecgpu_accum_read(ecgpu_accum* a, int i, char* out, int64_t nbytes) {
  if (!a || i < 0 || i >= a->m || !out || nbytes < 0 || nbytes > a->size)
    return fail(ECGPU_ERR_ARG, "ecgpu_accum_read: bad arguments");
  if (int rc = accum_sync(a)) return rc;
  if (!a->init[i]) return ECGPU_ERR;
  DeviceGuard g(a->device);
  if (a->stream) {  // on the accumulator's own stream, not the device-wide null stream
    ECGPU_HIP(hipMemcpyAsync(out, ecgpu_accum_device_ptr(a, i), size_t(nbytes), hipMemcpyDefault, a->stream));
    ECGPU_HIP(hipStreamSynchronize(a->stream));
  } else {
    ECGPU_HIP(hipMemcpy(out, ecgpu_accum_device_ptr(a, i), size_t(nbytes), hipMemcpyDefault));
  }
  return ECGPU_OK;
}

ECGPU_API int ecgpu_accum_reset(ecgpu_accum* a) {
  if (!a) return fail(ECGPU_ERR_ARG, "ecgpu_accum_reset: null");
  if (int rc = accum_sync(a)) return rc;
  std::fill(a->init.begin(), a->init.end(), 0);
  return ECGPU_OK;
}

ECGPU_API void ecgpu_accum_destroy(ecgpu_accum* a) {
  if (!a) return;
  (void)accum_sync(a);
  DeviceGuard g(a->device);
  if (a->stream) (void)hipStreamDestroy(a->stream);
  if (a->d_blk) (void)hipFree(a->d_blk);
  if (a->d_acc) (void)hipFree(a->d_acc);
  delete a;
}

}  // extern "C"
