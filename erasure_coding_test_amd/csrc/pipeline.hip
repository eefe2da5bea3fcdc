// pipeline.hip -- host-memory pipelines (ecgpu_pipeline_*) and multi-device
// groups (ecgpu_pipeline_group_*): the client's write / read paths
// (client_main.cpp:1714-1815, :2055-2182) with H2D, coding and D2H of
// consecutive stripes overlapped on three streams.  The ticket / slot / D2H
// worker logic and the group members' queues are host_sync.hpp's (tested
// under ThreadSanitizer on a fake device, tests/test_sanitizers.py); this
// file supplies their HIP side.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "buffer_contract.hpp"
#include "ecgpu.h"
#include "gf_host.hpp"
#include "host_sync.hpp"
#include "matrix_host.hpp"
#include "planner.hpp"
#include "runtime.hpp"
#include "schedule_host.hpp"

using namespace ecgpu;
using namespace ecgpu::rt;

namespace {
// The HIP side of a host pipeline (hostsync::StripePipeline's Ops): a ring
// of `depth` device stripe slots, one bound plan per slot, three streams and
// per-slot loaded / computed / drained events.
struct PipeDevice {
  int device = 0, k = 0, m = 0, depth = 0;
  int64_t size = 0;
  std::vector<int> src_ids, out_ids;  // shard ids read / written (id < k: data_ptrs[id], else coding_ptrs[id-k])
  size_t slot_stride = 0;             // bytes between shards inside a ring slot
  uint8_t* d_ring = nullptr;          // depth slots x (nsrc inputs, then rows outputs)
  std::vector<ecgpu_plan*> plans;     // one bound plan per ring slot (none when nsrc or rows is 0)
  hipStream_t s_h2d = nullptr, s_comp = nullptr, s_d2h = nullptr;
  std::vector<hipEvent_t> loaded, computed, drained;
  // ECGPU_PIPE_ZC (read at creation): 1 the kernel writes the outputs into
  // pinned host buffers in place, 2 it also reads the sources there (no DMA);
  // a stripe whose buffers are not all mapped host memory takes the DMA path.
  int zc_mode = 0;
  FusedOp zc_op;                      // the map for gf_apply_inl launches (coef only; pointers per stripe)
  std::vector<char> zc_slot;          // per slot: its outputs were written in place (no D2H)

  int nsrc() const { return int(src_ids.size()); }
  int rows() const { return int(out_ids.size()); }
  uint8_t* slot_shard(int slot, int j) const {
    return d_ring + slot_stride * (size_t(nsrc() + rows()) * size_t(slot) + size_t(j));
  }

  // The stripe's zero-copy launch (ECGPU_PIPE_ZC), or false when a buffer is
  // not mapped host memory: sources from the slot after its H2D (mode 1) or
  // read in place (mode 2), outputs written in place over PCIe.
  int stage_zc(int sl, const std::function<char*(int)>& host, bool* done) {
    *done = false;
    const int ns = nsrc(), nr = rows();
    const size_t bytes = size_t(size);
    std::vector<uint8_t*> dp(size_t(nr), nullptr);
    std::vector<const uint8_t*> sp(size_t(ns), nullptr);
    for (int i = 0; i < nr; ++i) {
      void* dv = nullptr;
      if (!host_mapped(host(out_ids[i]), bytes, &dv)) return ECGPU_OK;
      dp[size_t(i)] = static_cast<uint8_t*>(dv);
    }
    for (int j = 0; j < ns; ++j) {
      void* dv = nullptr;
      if (zc_mode == 2 && !host_mapped(host(src_ids[j]), bytes, &dv)) return ECGPU_OK;
      sp[size_t(j)] = zc_mode == 2 ? static_cast<const uint8_t*>(dv) : slot_shard(sl, j);
    }
    if (zc_mode == 1) {
      std::vector<char*> hp;
      for (int j = 0; j < ns; ++j) hp.push_back(host(src_ids[j]));
      if (int rc = copy_shards(true, slot_shard(sl, 0), slot_stride, hp, bytes, s_h2d)) return rc;
    }
    ECGPU_HIP(hipEventRecord(loaded[sl], s_h2d));
    ECGPU_HIP(hipStreamWaitEvent(s_comp, loaded[sl], 0));
    // the host outputs of the stripe that last used this slot were written by
    // an earlier launch on this same stream: no event needed between them
    if (int rc = launch_inline(zc_op, sp, dp, size, s_comp, /*host_io=*/true)) return rc;
    ECGPU_HIP(hipEventRecord(computed[sl], s_comp));
    *done = true;
    return ECGPU_OK;
  }

  // H2D of the sources (s_h2d), the fused apply (s_comp), the computed event.
  int stage(int sl, char** data_ptrs, char** coding_ptrs, std::vector<char*>* out, bool* out_blocks) {
    auto host = [&](int id) { return id < k ? data_ptrs[id] : coding_ptrs[id - k]; };
    const int ns = nsrc(), nr = rows();
    const size_t bytes = size_t(size);
    zc_slot[size_t(sl)] = 0;
    if (zc_mode != 0 && ns > 0 && nr > 0) {
      bool done = false;
      if (int rc = stage_zc(sl, host, &done)) return rc;
      if (done) {
        zc_slot[size_t(sl)] = 1;
        out->clear();
        *out_blocks = false;
        return ECGPU_OK;
      }
    }
    if (nr > 0) {  // nothing to read when no shard is written
      std::vector<char*> hp;
      for (int j = 0; j < ns; ++j) hp.push_back(host(src_ids[j]));
      if (int rc = copy_shards(true, slot_shard(sl, 0), slot_stride, hp, bytes, s_h2d)) return rc;
    }
    ECGPU_HIP(hipEventRecord(loaded[sl], s_h2d));
    ECGPU_HIP(hipStreamWaitEvent(s_comp, loaded[sl], 0));
    if (ns > 0 && nr > 0) {
      if (int rc = plan_launch(plans[sl], s_comp)) return rc;
    } else {
      for (int i = 0; i < nr; ++i)  // rows with no source: all-zero output
        ECGPU_HIP(hipMemsetAsync(slot_shard(sl, ns + i), 0, bytes, s_comp));
    }
    ECGPU_HIP(hipEventRecord(computed[sl], s_comp));
    out->clear();
    bool pageable = false;
    for (int i = 0; i < nr; ++i) {
      out->push_back(host(out_ids[i]));
      pageable = pageable || !is_pinned(out->back());
    }
    *out_blocks = pageable;  // HIP's pageable D2H blocks the issuing thread
    return ECGPU_OK;
  }

  // D2H of a slot's outputs (s_d2h, after the slot's compute), then drained.
  int d2h(int sl, const std::vector<char*>& hp) {
    ECGPU_HIP(hipStreamWaitEvent(s_d2h, computed[sl], 0));
    if (!zc_slot[size_t(sl)])  // (written in place by the kernel: nothing to copy)
      if (int rc = copy_shards(false, slot_shard(sl, nsrc()), slot_stride, hp, size_t(size), s_d2h)) return rc;
    ECGPU_HIP(hipEventRecord(drained[sl], s_d2h));
    return ECGPU_OK;
  }

  int sync_drained(int sl) {
    ECGPU_HIP(hipEventSynchronize(drained[sl]));  // (event waits need no current-device switch)
    return ECGPU_OK;
  }

  void sync_all() {
    for (hipStream_t s : {s_h2d, s_comp, s_d2h})
      if (s) (void)hipStreamSynchronize(s);
  }

  void bind_thread() { (void)hipSetDevice(device); }  // once: the worker only ever drives this device
  int fail(int rc, const std::string& msg) { return rt::fail(rc, msg); }
  std::string last_error() const { return t_err; }
};

bool pipe_d2h_worker_enabled() { return knob(Knob::kPipeD2hWorker) != 0; }
}  // namespace

extern "C" {

// ---------------------------------------------------- host pipeline ----
struct ecgpu_pipeline {
  PipeDevice dev;
  std::unique_ptr<hostsync::StripePipeline<PipeDevice>> core;
};

namespace {
void pipeline_free(ecgpu_pipeline* p) {
  if (!p) return;
  p->core.reset();  // joins the D2H worker
  PipeDevice& d = p->dev;
  DeviceGuard g(d.device);
  for (auto* pl : d.plans) plan_free(pl);
  for (auto& v : {&d.loaded, &d.computed, &d.drained})
    for (auto e : *v)
      if (e) (void)hipEventDestroy(e);
  for (auto s : {d.s_h2d, d.s_comp, d.s_d2h})
    if (s) (void)hipStreamDestroy(s);
  if (d.d_ring) (void)hipFree(d.d_ring);
  delete p;
}

// rows x nsrc coefficient map from shard ids src_ids to shard ids out_ids.
ecgpu_pipeline* pipeline_build(int k, int m, int rows, int nsrc, const int* coef, const int* src_ids,
                               const int* out_ids, int64_t size, int depth, int device) {
  auto* p = new ecgpu_pipeline();
  PipeDevice& d = p->dev;
  d.device = device < 0 ? current_device() : device;
  d.k = k;
  d.m = m;
  d.depth = depth;
  d.size = size;
  d.src_ids.assign(src_ids, src_ids + nsrc);
  d.out_ids.assign(out_ids, out_ids + rows);
  // ECGPU_PIPE_CONTIG (default 1): a slot's shards back to back when the size
  // keeps them 256-B aligned, so a stripe laid out contiguously in host memory
  // crosses PCIe as one 1-D copy each way (copy_shards); the shard-stride skew
  // (§4) buys a few us of a one-stripe launch that hides under a 0.8 ms copy
  d.slot_stride = knob(Knob::kPipeContig) != 0 && size % 256 == 0
                      ? size_t(size)
                      : size_t(ecgpu_recommended_shard_stride_km(size, k, m));
  DeviceGuard g(d.device);
  auto bad = [&](hipError_t e, const char* what) {
    fail(ECGPU_ERR_HIP, std::string("ecgpu_pipeline: ") + what + ": " + hipGetErrorString(e));
    pipeline_free(p);
    return static_cast<ecgpu_pipeline*>(nullptr);
  };
  hipError_t e = hipSuccess;
  const size_t ring = d.slot_stride * size_t(nsrc + rows) * size_t(depth);
  if (ring && (e = hipMalloc(reinterpret_cast<void**>(&d.d_ring), ring)) != hipSuccess) return bad(e, "hipMalloc");
  for (hipStream_t* s : {&d.s_h2d, &d.s_comp, &d.s_d2h})
    if ((e = hipStreamCreateWithFlags(s, hipStreamNonBlocking)) != hipSuccess) return bad(e, "stream");
  for (auto* v : {&d.loaded, &d.computed, &d.drained}) {
    v->assign(size_t(depth), nullptr);
    for (auto& ev : *v)
      if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return bad(e, "event");
  }
  d.zc_slot.assign(size_t(depth), 0);
  d.zc_op.w = 8;
  d.zc_op.coef.assign(coef, coef + size_t(rows) * size_t(nsrc));
  d.zc_op.srcs.assign(size_t(nsrc), nullptr);  // counts only (inline_ok); pointers are per stripe
  d.zc_op.dsts.assign(size_t(rows), nullptr);
  d.zc_mode = std::max(0, std::min(2, knob(Knob::kPipeZc)));
  if (d.zc_mode && !(nsrc > 0 && rows > 0 && inline_ok(d.zc_op, size))) d.zc_mode = 0;
  if (nsrc > 0 && rows > 0) {
    for (int sl = 0; sl < depth; ++sl) {
      std::vector<const uint8_t*> src(static_cast<size_t>(nsrc));
      std::vector<uint8_t*> dst(static_cast<size_t>(rows));
      for (int j = 0; j < nsrc; ++j) src[j] = d.slot_shard(sl, j);
      for (int i = 0; i < rows; ++i) dst[i] = d.slot_shard(sl, nsrc + i);
      auto* pl = new ecgpu_plan();
      if (plan_init(pl, rows, nsrc, coef, d.device) != ECGPU_OK ||
          plan_bind(pl, 1, src.data(), dst.data(), size, nullptr) != ECGPU_OK) {
        plan_free(pl);
        pipeline_free(p);
        return nullptr;
      }
      d.plans.push_back(pl);
    }
  }
  // the test_d2h_delay_us knob (tests only, no environment variable: set with
  // ecgpu_set_knob): the D2H worker sleeps between taking a job and issuing
  // it, which widens the window in which the submitting thread races it
  p->core = std::make_unique<hostsync::StripePipeline<PipeDevice>>(
      &p->dev, depth, pipe_d2h_worker_enabled(), std::max(0, knob(Knob::kTestD2hDelayUs)));
  return p;
}
}  // namespace

ECGPU_API ecgpu_pipeline* ecgpu_pipeline_create(int k, int m, const int* matrix, int64_t size, int depth,
                                                int device) {
  if (k <= 0 || m <= 0 || !matrix || size <= 0 || depth <= 0) {
    fail(ECGPU_ERR_ARG, "ecgpu_pipeline_create: bad arguments");
    return nullptr;
  }
  std::vector<int> src(static_cast<size_t>(k)), out(static_cast<size_t>(m));
  for (int j = 0; j < k; ++j) src[j] = j;
  for (int i = 0; i < m; ++i) out[i] = k + i;
  return pipeline_build(k, m, m, k, matrix, src.data(), out.data(), size, depth, device);
}

ECGPU_API ecgpu_pipeline* ecgpu_pipeline_create_decode(int k, int m, int w, const int* matrix, int row_k_ones,
                                                       const int* erasures, int64_t size, int depth, int device) {
  if (k <= 0 || m <= 0 || w != 8 || !matrix || !erasures || size <= 0 || depth <= 0) {
    fail(ECGPU_ERR_ARG, "ecgpu_pipeline_create_decode: bad arguments");
    return nullptr;
  }
  const size_t n = size_t(k + m);
  std::vector<int> out(n), src(n), coef(n * n);
  int n_out = 0, n_src = 0;
  if (ecgpu_decode_plan(k, m, w, matrix, row_k_ones, erasures, out.data(), &n_out, src.data(), &n_src,
                        coef.data()) != ECGPU_OK) {
    fail(ECGPU_ERR, "ecgpu_pipeline_create_decode: erasure pattern not decodable (reference decode returns -1)");
    return nullptr;
  }
  return pipeline_build(k, m, n_out, n_src, coef.data(), src.data(), out.data(), size, depth, device);
}

// Queues stripe t into ring slot t % depth: H2D of the sources, the fused
// apply, then D2H of the outputs -- issued here, or by the pipeline's D2H
// worker when an output is pageable or an earlier D2H is still unissued.
ECGPU_API int64_t ecgpu_pipeline_submit(ecgpu_pipeline* p, char** data_ptrs, char** coding_ptrs) {
  if (!p || !data_ptrs || !coding_ptrs) return fail(ECGPU_ERR_ARG, "ecgpu_pipeline_submit: bad arguments");
  // an output sharing bytes with another shard of the stripe: rejected before
  // anything is queued (buffer_contract.hpp)
  if (int rc = check_stripe_buffers("ecgpu_pipeline_submit", p->dev.k, data_ptrs, coding_ptrs, p->dev.src_ids,
                                    p->dev.out_ids, p->dev.size))
    return rc;
  DeviceGuard g(p->dev.device);
  return p->core->submit(data_ptrs, coding_ptrs);
}

ECGPU_API int ecgpu_pipeline_wait(ecgpu_pipeline* p, int64_t ticket) {
  if (!p || ticket < 0) return fail(ECGPU_ERR_ARG, "ecgpu_pipeline_wait: bad arguments");
  return p->core->wait(ticket);
}

ECGPU_API int ecgpu_pipeline_drain(ecgpu_pipeline* p) {
  if (!p) return fail(ECGPU_ERR_ARG, "ecgpu_pipeline_drain: null");
  return p->core->drain();
}

ECGPU_API void ecgpu_pipeline_destroy(ecgpu_pipeline* p) {
  if (!p) return;
  (void)p->core->drain();
  pipeline_free(p);
}

// ---------------------------------------------- multi-device pipeline ----
// Stripes are independent, so a process driving several GPUs
// shards them round-robin: stripe t runs on member t % n as that member's
// local ticket t / n.  No collective and no cross-device traffic.  Each
// member is a complete single-device pipeline with its own ring and streams
// AND its own submit thread, bound to its device once (hipSetDevice at
// thread start, never again): group_submit only hands the stripe's pointer
// lists to member t % n's queue (hostsync::MemberQueue: a per-member lock;
// tickets come from an atomic counter, no group-wide lock) and returns, the
// worker issues the stripe's copies and launch, so pageable staging on one
// device never holds up another.  Waits sync on the member's events (no
// device switch).
namespace {
struct GroupJob {
  std::vector<char*> data, coding;
};

struct GroupMember {
  ecgpu_pipeline* p = nullptr;
  int k = 0, m = 0;
  std::unique_ptr<hostsync::MemberQueue<GroupJob>> q;
  std::thread worker;

  void run() {
    (void)hipSetDevice(p->dev.device);  // once: every submit below runs on this device
    q->run([this](GroupJob& job, std::string* msg) {
      const int64_t r = ecgpu_pipeline_submit(p, job.data.data(), job.coding.data());
      if (r < 0) *msg = t_err;
      return r;
    });
  }
};
}  // namespace

struct ecgpu_pipeline_group {
  std::vector<std::unique_ptr<GroupMember>> members;
  std::atomic<int64_t> next_ticket{0};
};

namespace {
void group_free(ecgpu_pipeline_group* g) {
  if (!g) return;
  for (auto& mb : g->members) {
    if (mb->worker.joinable()) {
      mb->q->stop();
      mb->worker.join();
    }
    ecgpu_pipeline_destroy(mb->p);
  }
  delete g;
}

ecgpu_pipeline_group* group_build(int ndev, const int* devices, int k, int m, int depth,
                                  const std::function<ecgpu_pipeline*(int)>& make) {
  if (ndev <= 0 || !devices) {
    fail(ECGPU_ERR_ARG, "ecgpu_pipeline_group: ndev > 0 and a device list required");
    return nullptr;
  }
  auto* g = new ecgpu_pipeline_group();
  for (int i = 0; i < ndev; ++i) {
    ecgpu_pipeline* p = make(devices[i]);
    if (!p) {  // make() left the message in ecgpu_last_error
      const std::string msg = t_err;
      group_free(g);
      t_err = msg;
      return nullptr;
    }
    auto mb = std::make_unique<GroupMember>();
    mb->p = p;
    mb->k = k;
    mb->m = m;
    mb->q = std::make_unique<hostsync::MemberQueue<GroupJob>>(depth);  // back-pressure at `depth` queued stripes
    g->members.push_back(std::move(mb));
  }
  for (auto& mb : g->members) {
    GroupMember* raw = mb.get();
    raw->worker = std::thread([raw] { raw->run(); });
  }
  return g;
}
}  // namespace

ECGPU_API ecgpu_pipeline_group* ecgpu_pipeline_group_create(int k, int m, const int* matrix, int64_t size, int depth,
                                                            int ndev, const int* devices) {
  return group_build(ndev, devices, k, m, depth,
                     [&](int dev) { return ecgpu_pipeline_create(k, m, matrix, size, depth, dev); });
}

ECGPU_API ecgpu_pipeline_group* ecgpu_pipeline_group_create_decode(int k, int m, int w, const int* matrix,
                                                                   int row_k_ones, const int* erasures, int64_t size,
                                                                   int depth, int ndev, const int* devices) {
  return group_build(ndev, devices, k, m, depth, [&](int dev) {
    return ecgpu_pipeline_create_decode(k, m, w, matrix, row_k_ones, erasures, size, depth, dev);
  });
}

ECGPU_API int64_t ecgpu_pipeline_group_submit(ecgpu_pipeline_group* g, char** data_ptrs, char** coding_ptrs) {
  if (!g || !data_ptrs || !coding_ptrs) return fail(ECGPU_ERR_ARG, "ecgpu_pipeline_group_submit: bad arguments");
  // checked here, before a ticket is taken, so a rejected stripe leaves no gap
  // in the member queues (every member runs the same shard map)
  const PipeDevice& d0 = g->members[0]->p->dev;
  if (int rc = check_stripe_buffers("ecgpu_pipeline_group_submit", d0.k, data_ptrs, coding_ptrs, d0.src_ids,
                                    d0.out_ids, d0.size))
    return rc;
  const int64_t n = int64_t(g->members.size());
  const int64_t t = g->next_ticket.fetch_add(1);
  GroupMember& mb = *g->members[size_t(t % n)];
  GroupJob job;
  job.data.assign(data_ptrs, data_ptrs + mb.k);
  job.coding.assign(coding_ptrs, coding_ptrs + mb.m);
  mb.q->put(t / n, std::move(job));
  return t;
}

ECGPU_API int ecgpu_pipeline_group_wait(ecgpu_pipeline_group* g, int64_t ticket) {
  if (!g || ticket < 0) return fail(ECGPU_ERR_ARG, "ecgpu_pipeline_group_wait: bad arguments");
  if (ticket >= g->next_ticket.load()) return fail(ECGPU_ERR_ARG, "ecgpu_pipeline_group_wait: ticket not submitted");
  const int64_t n = int64_t(g->members.size());
  GroupMember& mb = *g->members[size_t(ticket % n)];
  const int64_t local = ticket / n;
  std::string msg;
  if (int rc = mb.q->wait_handled(local, &msg)) return fail(rc, msg);  // the worker has queued it
  return ecgpu_pipeline_wait(mb.p, local);
}

ECGPU_API int ecgpu_pipeline_group_drain(ecgpu_pipeline_group* g) {
  if (!g) return fail(ECGPU_ERR_ARG, "ecgpu_pipeline_group_drain: null");
  const int64_t end = g->next_ticket.load(), n = int64_t(g->members.size());
  int rc = ECGPU_OK;
  for (int64_t t = std::max<int64_t>(0, end - n); t < end; ++t) {  // each member's last ticket
    const int r = ecgpu_pipeline_group_wait(g, t);
    if (r != ECGPU_OK && rc == ECGPU_OK) rc = r;
  }
  return rc;
}

ECGPU_API int ecgpu_pipeline_group_size(ecgpu_pipeline_group* g) { return g ? int(g->members.size()) : 0; }

ECGPU_API void ecgpu_pipeline_group_destroy(ecgpu_pipeline_group* g) {
  if (!g) return;
  (void)ecgpu_pipeline_group_drain(g);
  group_free(g);
}

}  // extern "C"
