// pipeline.hip -- host-memory pipelines (ecgpu_pipeline_*) and multi-device
// groups (ecgpu_pipeline_group_*): the client's write / read paths
// (client_main.cpp:1714-1815, :2055-2182) with H2D, coding and D2H of
// consecutive stripes overlapped on three streams.
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

#include "ecgpu.h"
#include "gf_host.hpp"
#include "matrix_host.hpp"
#include "planner.hpp"
#include "schedule_host.hpp"
#include "runtime.hpp"

using namespace ecgpu;
using namespace ecgpu::rt;

extern "C" {

// ---------------------------------------------------- host pipeline ----
struct ecgpu_pipeline {
  int device = 0, k = 0, m = 0, depth = 0;
  int64_t size = 0;
  std::vector<int> src_ids, out_ids;  // shard ids read / written (id < k: data_ptrs[id], else coding_ptrs[id-k])
  size_t slot_stride = 0;             // bytes between shards inside a ring slot
  uint8_t* d_ring = nullptr;          // depth slots x (nsrc inputs, then rows outputs)
  std::vector<ecgpu_plan*> plans;     // one bound plan per ring slot (none when nsrc or rows is 0)
  hipStream_t s_h2d = nullptr, s_comp = nullptr, s_d2h = nullptr;
  std::vector<hipEvent_t> loaded, computed, drained;
  std::vector<int64_t> slot_ticket;  // ticket occupying each slot (-1: free)
  int64_t next_ticket = 0;
  int64_t done_below = 0;             // every ticket < done_below has completed
  std::mutex mu;
  // D2H worker (pipeline_d2h_worker): HIP's pageable copies block the
  // thread that issues them, so a stripe's D2H into pageable buffers is
  // issued by this thread while the submitting thread already moves the next
  // stripe's H2D -- the two directions of the link overlap.  Pinned outputs
  // are issued inline when no job is pending (their copies do not block).
  struct D2HJob {
    int slot;
    int64_t ticket;
    std::vector<char*> hp;
  };
  std::thread worker;
  std::mutex qmu;
  std::condition_variable qcv;
  std::deque<D2HJob> q;
  int64_t issued_below = 0;  // every ticket < issued_below has its D2H enqueued (drained event recorded)
  bool stop = false;
  int worker_rc = 0;  // ECGPU_OK, or the first failure of a worker-issued D2H
  std::string worker_err;

  int nsrc() const { return int(src_ids.size()); }
  int rows() const { return int(out_ids.size()); }
  uint8_t* slot_shard(int slot, int j) const {
    return d_ring + slot_stride * (size_t(nsrc() + rows()) * size_t(slot) + size_t(j));
  }
};

namespace {
void pipeline_free(ecgpu_pipeline* p) {
  if (!p) return;
  if (p->worker.joinable()) {
    {
      std::lock_guard<std::mutex> lk(p->qmu);
      p->stop = true;
    }
    p->qcv.notify_all();
    p->worker.join();
  }
  DeviceGuard g(p->device);
  for (auto* pl : p->plans) plan_free(pl);
  for (auto& v : {&p->loaded, &p->computed, &p->drained})
    for (auto e : *v)
      if (e) (void)hipEventDestroy(e);
  for (auto s : {p->s_h2d, p->s_comp, p->s_d2h})
    if (s) (void)hipStreamDestroy(s);
  if (p->d_ring) (void)hipFree(p->d_ring);
  delete p;
}

int pipeline_retire(ecgpu_pipeline* p, int slot) {
  const int64_t t = p->slot_ticket[slot];
  if (t < 0) return ECGPU_OK;
  {
    // the slot's drained event is only meaningful once its D2H is enqueued
    std::unique_lock<std::mutex> lk(p->qmu);
    p->qcv.wait(lk, [&] { return p->issued_below > t; });
    if (p->worker_rc != ECGPU_OK) return fail(p->worker_rc, p->worker_err);
  }
  ECGPU_HIP(hipEventSynchronize(p->drained[slot]));
  p->slot_ticket[slot] = -1;
  // tickets complete in submission order (the D2H stream is in order)
  if (t + 1 > p->done_below) p->done_below = t + 1;
  return ECGPU_OK;
}

// rows x nsrc coefficient map from shard ids src_ids to shard ids out_ids.
ecgpu_pipeline* pipeline_build(int k, int m, int rows, int nsrc, const int* coef, const int* src_ids,
                               const int* out_ids, int64_t size, int depth, int device) {
  auto* p = new ecgpu_pipeline();
  p->device = device < 0 ? current_device() : device;
  p->k = k;
  p->m = m;
  p->depth = depth;
  p->size = size;
  p->src_ids.assign(src_ids, src_ids + nsrc);
  p->out_ids.assign(out_ids, out_ids + rows);
  p->slot_stride = size_t(ecgpu_recommended_shard_stride(size));
  DeviceGuard g(p->device);
  auto bad = [&](hipError_t e, const char* what) {
    fail(ECGPU_ERR_HIP, std::string("ecgpu_pipeline: ") + what + ": " + hipGetErrorString(e));
    pipeline_free(p);
    return static_cast<ecgpu_pipeline*>(nullptr);
  };
  hipError_t e = hipSuccess;
  const size_t ring = p->slot_stride * size_t(nsrc + rows) * size_t(depth);
  if (ring && (e = hipMalloc(reinterpret_cast<void**>(&p->d_ring), ring)) != hipSuccess) return bad(e, "hipMalloc");
  for (hipStream_t* s : {&p->s_h2d, &p->s_comp, &p->s_d2h})
    if ((e = hipStreamCreateWithFlags(s, hipStreamNonBlocking)) != hipSuccess) return bad(e, "stream");
  for (auto* v : {&p->loaded, &p->computed, &p->drained}) {
    v->assign(size_t(depth), nullptr);
    for (auto& ev : *v)
      if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return bad(e, "event");
  }
  p->slot_ticket.assign(size_t(depth), -1);
  if (nsrc > 0 && rows > 0) {
    for (int sl = 0; sl < depth; ++sl) {
      std::vector<const uint8_t*> src(static_cast<size_t>(nsrc));
      std::vector<uint8_t*> dst(static_cast<size_t>(rows));
      for (int j = 0; j < nsrc; ++j) src[j] = p->slot_shard(sl, j);
      for (int i = 0; i < rows; ++i) dst[i] = p->slot_shard(sl, nsrc + i);
      auto* pl = new ecgpu_plan();
      if (plan_init(pl, rows, nsrc, coef, p->device) != ECGPU_OK ||
          plan_bind(pl, 1, src.data(), dst.data(), size, nullptr) != ECGPU_OK) {
        plan_free(pl);
        pipeline_free(p);
        return nullptr;
      }
      p->plans.push_back(pl);
    }
  }
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


namespace {
bool pipe_d2h_worker_enabled() {
  static const bool v = env_int("ECGPU_PIPE_D2H_WORKER", 1) != 0;
  return v;
}

// D2H of a slot's outputs to the host pointers hp (s_d2h, after the slot's
// compute), then the slot's drained event.
int pipeline_d2h(ecgpu_pipeline* p, int sl, const std::vector<char*>& hp) {
  ECGPU_HIP(hipStreamWaitEvent(p->s_d2h, p->computed[sl], 0));
  if (int rc = copy_shards(false, p->slot_shard(sl, p->nsrc()), p->slot_stride, hp, size_t(p->size), p->s_d2h))
    return rc;
  ECGPU_HIP(hipEventRecord(p->drained[sl], p->s_d2h));
  return ECGPU_OK;
}

void pipeline_d2h_worker(ecgpu_pipeline* p) {
  (void)hipSetDevice(p->device);  // once: this thread only ever drives this device
  for (;;) {
    ecgpu_pipeline::D2HJob job;
    {
      std::unique_lock<std::mutex> lk(p->qmu);
      p->qcv.wait(lk, [&] { return p->stop || !p->q.empty(); });
      if (p->q.empty()) return;  // stop, nothing left
      job = std::move(p->q.front());
      p->q.pop_front();
    }
    int rc = ECGPU_OK;
    bool failed_before = false;
    {
      std::lock_guard<std::mutex> lk(p->qmu);
      failed_before = p->worker_rc != ECGPU_OK;
    }
    if (!failed_before) rc = pipeline_d2h(p, job.slot, job.hp);
    std::lock_guard<std::mutex> lk(p->qmu);
    if (rc != ECGPU_OK && p->worker_rc == ECGPU_OK) {
      p->worker_rc = rc;
      p->worker_err = t_err;
    }
    p->issued_below = job.ticket + 1;
    p->qcv.notify_all();
  }
}

// Queues stripe t into ring slot t % depth: H2D of the sources (s_h2d), the
// fused apply (s_comp), then D2H of the outputs (s_d2h) -- issued here, or
// by the pipeline's D2H worker when an output is pageable.
int pipeline_enqueue(ecgpu_pipeline* p, int sl, int64_t t, char** data_ptrs, char** coding_ptrs) {
  auto host = [&](int id) { return id < p->k ? data_ptrs[id] : coding_ptrs[id - p->k]; };
  const int ns = p->nsrc(), nr = p->rows();
  const size_t bytes = size_t(p->size);
  std::vector<char*> hp;
  int rc = ECGPU_OK;
  if (nr > 0) {  // nothing to read when no shard is written
    for (int j = 0; j < ns; ++j) hp.push_back(host(p->src_ids[j]));
    if ((rc = copy_shards(true, p->slot_shard(sl, 0), p->slot_stride, hp, bytes, p->s_h2d)) != ECGPU_OK) return rc;
  }
  ECGPU_HIP(hipEventRecord(p->loaded[sl], p->s_h2d));
  ECGPU_HIP(hipStreamWaitEvent(p->s_comp, p->loaded[sl], 0));
  if (ns > 0 && nr > 0) {
    if ((rc = plan_launch(p->plans[sl], p->s_comp)) != ECGPU_OK) return rc;
  } else {
    for (int i = 0; i < nr; ++i)  // rows with no source: all-zero output
      ECGPU_HIP(hipMemsetAsync(p->slot_shard(sl, ns + i), 0, bytes, p->s_comp));
  }
  ECGPU_HIP(hipEventRecord(p->computed[sl], p->s_comp));
  hp.clear();
  for (int i = 0; i < nr; ++i) hp.push_back(host(p->out_ids[i]));
  bool pageable = false;
  for (char* h : hp) pageable = pageable || !is_pinned(h);
  std::unique_lock<std::mutex> lk(p->qmu);
  if (p->worker_rc != ECGPU_OK) return fail(p->worker_rc, p->worker_err);
  if ((pageable && pipe_d2h_worker_enabled()) || !p->q.empty()) {
    // behind any pending job, so s_d2h keeps submission order
    if (!p->worker.joinable()) p->worker = std::thread(pipeline_d2h_worker, p);
    p->q.push_back(ecgpu_pipeline::D2HJob{sl, t, std::move(hp)});
    lk.unlock();
    p->qcv.notify_all();
    return ECGPU_OK;
  }
  lk.unlock();
  if ((rc = pipeline_d2h(p, sl, hp)) != ECGPU_OK) return rc;
  lk.lock();
  p->issued_below = t + 1;
  return ECGPU_OK;
}
}  // namespace

ECGPU_API int64_t ecgpu_pipeline_submit(ecgpu_pipeline* p, char** data_ptrs, char** coding_ptrs) {
  if (!p || !data_ptrs || !coding_ptrs) return fail(ECGPU_ERR_ARG, "ecgpu_pipeline_submit: bad arguments");
  std::lock_guard<std::mutex> lk(p->mu);
  DeviceGuard g(p->device);
  const int64_t t = p->next_ticket;
  const int sl = int(t % p->depth);
  int rc = pipeline_retire(p, sl);  // the slot's previous stripe must be out
  if (rc != ECGPU_OK) return rc;
  rc = pipeline_enqueue(p, sl, t, data_ptrs, coding_ptrs);
  if (rc != ECGPU_OK) {
    // part of the stripe may already be queued against the caller's buffers:
    // let it finish before reporting, so no DMA outlives the failed call
    const std::string msg = t_err;
    for (hipStream_t s : {p->s_h2d, p->s_comp, p->s_d2h}) (void)hipStreamSynchronize(s);
    t_err = msg;
    return rc;
  }
  p->slot_ticket[sl] = t;
  p->next_ticket = t + 1;
  return t;
}

ECGPU_API int ecgpu_pipeline_wait(ecgpu_pipeline* p, int64_t ticket) {
  if (!p || ticket < 0) return fail(ECGPU_ERR_ARG, "ecgpu_pipeline_wait: bad arguments");
  std::lock_guard<std::mutex> lk(p->mu);
  if (ticket < p->done_below) return ECGPU_OK;
  if (ticket >= p->next_ticket) return fail(ECGPU_ERR_ARG, "ecgpu_pipeline_wait: ticket not submitted");
  // (event waits need no current-device switch)
  // retire every slot up to and including the ticket's (completion is in order)
  for (int64_t t = p->done_below; t <= ticket; ++t) {
    const int rc = pipeline_retire(p, int(t % p->depth));
    if (rc != ECGPU_OK) return rc;
  }
  return ECGPU_OK;
}

ECGPU_API int ecgpu_pipeline_drain(ecgpu_pipeline* p) {
  if (!p) return fail(ECGPU_ERR_ARG, "ecgpu_pipeline_drain: null");
  if (p->next_ticket == 0) return ECGPU_OK;
  return ecgpu_pipeline_wait(p, p->next_ticket - 1);
}

ECGPU_API void ecgpu_pipeline_destroy(ecgpu_pipeline* p) {
  if (!p) return;
  (void)ecgpu_pipeline_drain(p);
  pipeline_free(p);
}

// ---------------------------------------------- multi-device pipeline ----
// Stripes are independent, so a process driving several GPUs
// shards them round-robin: stripe t runs on member t % n as that member's
// local ticket t / n.  No collective and no cross-device traffic.  Each
// member is a complete single-device pipeline with its own ring and streams
// AND its own submit thread, bound to its device once (hipSetDevice at
// thread start, never again): group_submit only hands the stripe's pointer
// lists to member t % n's queue (a per-member lock; tickets come from an
// atomic counter, no group-wide lock) and returns, the worker issues the
// stripe's copies and launch, so pageable staging on one device never holds
// up another.  Waits sync on the member's events (no device switch).
namespace {
struct GroupJob {
  std::vector<char*> data, coding;
};

struct GroupMember {
  ecgpu_pipeline* p = nullptr;
  int k = 0, m = 0, cap = 1;
  std::thread worker;
  std::mutex mu;
  std::condition_variable cv_job, cv_done, cv_space;
  std::map<int64_t, GroupJob> pending;  // local ticket -> job, handed in possibly out of order
  int64_t next_local = 0;               // next local ticket the worker submits
  int64_t failed_from = -1;             // first local ticket whose submit failed (sticky)
  int failed_rc = ECGPU_OK;
  std::string failed_msg;
  bool stop = false;

  void run() {
    (void)hipSetDevice(p->device);  // once: every submit below runs on this device
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      cv_job.wait(lk, [&] { return stop || pending.count(next_local) != 0; });
      auto it = pending.find(next_local);
      if (it == pending.end()) return;  // stop, queue drained
      GroupJob job = std::move(it->second);
      pending.erase(it);
      cv_space.notify_all();
      int64_t r = 0;
      if (failed_from < 0) {
        lk.unlock();
        r = ecgpu_pipeline_submit(p, job.data.data(), job.coding.data());
        const std::string msg = r < 0 ? t_err : std::string();
        lk.lock();
        if (r < 0) {
          failed_from = next_local;
          failed_rc = int(r);
          failed_msg = msg;
        }
      }
      ++next_local;
      cv_done.notify_all();
    }
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
      {
        std::lock_guard<std::mutex> lk(mb->mu);
        mb->stop = true;
      }
      mb->cv_job.notify_all();
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
    mb->cap = std::max(1, depth);
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
  const int64_t n = int64_t(g->members.size());
  const int64_t t = g->next_ticket.fetch_add(1);
  GroupMember& mb = *g->members[size_t(t % n)];
  GroupJob job;
  job.data.assign(data_ptrs, data_ptrs + mb.k);
  job.coding.assign(coding_ptrs, coding_ptrs + mb.m);
  {
    std::unique_lock<std::mutex> lk(mb.mu);
    // back-pressure: at most `depth` stripes queued ahead of the worker
    mb.cv_space.wait(lk, [&] { return int64_t(mb.pending.size()) < mb.cap || t / n <= mb.next_local; });
    mb.pending.emplace(t / n, std::move(job));
  }
  mb.cv_job.notify_one();
  return t;
}

ECGPU_API int ecgpu_pipeline_group_wait(ecgpu_pipeline_group* g, int64_t ticket) {
  if (!g || ticket < 0) return fail(ECGPU_ERR_ARG, "ecgpu_pipeline_group_wait: bad arguments");
  if (ticket >= g->next_ticket.load()) return fail(ECGPU_ERR_ARG, "ecgpu_pipeline_group_wait: ticket not submitted");
  const int64_t n = int64_t(g->members.size());
  GroupMember& mb = *g->members[size_t(ticket % n)];
  const int64_t local = ticket / n;
  {
    std::unique_lock<std::mutex> lk(mb.mu);
    mb.cv_done.wait(lk, [&] { return mb.next_local > local; });  // the worker has queued it
    if (mb.failed_from >= 0 && local >= mb.failed_from) return fail(mb.failed_rc, mb.failed_msg);
  }
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
