// host_sync.hpp -- the host-side synchronisation of the threaded runtime,
// with no HIP in it:
//   StripePipeline<Ops>  ticket / ring-slot / D2H-worker state machine of a
//                        host pipeline (pipeline.hip, ecgpu_pipeline_*)
//   MemberQueue<Job>     per-member submit queue of a pipeline group
//                        (ecgpu_pipeline_group_*)
//   IdlePool<T>          the synchronous calls' context pool
//   PerDevice<T>         lazily created per-device objects (upload streams)
// Device work goes through an Ops object (streams, events, copies), so the
// same code runs in libecgpu with HIP and in tests/sanitize/pipeline_harness.cpp
// under ThreadSanitizer with a fake device whose streams are threads and whose
// events complete after random delays (the reference races on
// its lazy tables, galois.cpp:329-336; the replacement must not).
//
// ECGPU_MUTANT_R2_D2H and ECGPU_MUTANT_R2_WAKEUP restore the round-2 logic of
// the D2H routing and of the group back-pressure wake-up.  Only the harness
// defines them, to show that it detects those bugs (tests/test_sanitizers.py).
#pragma once

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "ecgpu.h"

namespace ecgpu {
namespace hostsync {

// ---------------------------------------------------------------------------
// StripePipeline: stripe t occupies ring slot t % depth.  submit() queues the
// stripe's H2D + apply (Ops::stage) and its D2H (Ops::d2h), and returns the
// ticket; a slot is reused only after its previous stripe has drained.
//
// Ops (duck-typed):
//   int  stage(int slot, char** data, char** coding, std::vector<char*>* out, bool* out_blocks)
//          H2D of the slot's sources, the apply, the slot's `computed` event;
//          fills the host output pointers and whether a D2H into them blocks
//          the issuing thread (pageable memory).
//   int  d2h(int slot, const std::vector<char*>& out)
//          D2H after the slot's `computed` event, then the slot's `drained` event.
//   int  sync_drained(int slot)   host wait for the slot's last `drained` record
//   void sync_all()               every stream idle (failure path)
//   void bind_thread()            once, on the D2H worker thread
//   int  fail(int rc, const std::string& msg)   sets the calling thread's error
//   std::string last_error()
//
// D2H ordering.  HIP's D2H into pageable memory blocks the issuing thread, so
// such a stripe's D2H is handed to the D2H worker; the submitting thread goes
// on with the next stripe's H2D.  D2Hs are issued in ticket order: a stripe's
// D2H is issued inline only when no earlier ticket is still unissued
// (`issued_below == t`, which covers a job the worker has popped but not yet
// issued) and the queue is empty; otherwise it queues.  A retire waits until
// its slot's own ticket has been issued (`slot_issued`) before it syncs the
// slot's `drained` event, so it never syncs a stale record.
// ---------------------------------------------------------------------------
template <class Ops>
class StripePipeline {
 public:
  StripePipeline(Ops* ops, int depth, bool d2h_worker, int test_delay_us)
      : ops_(ops), depth_(depth), worker_enabled_(d2h_worker), test_delay_us_(test_delay_us),
        slot_ticket_(size_t(depth), -1), slot_issued_(size_t(depth), -1) {}
  StripePipeline(const StripePipeline&) = delete;
  StripePipeline& operator=(const StripePipeline&) = delete;
  ~StripePipeline() { stop_worker(); }

  int depth() const { return depth_; }

  // Ticket (>= 0) or an error code (< 0).
  int64_t submit(char** data, char** coding) {
    std::lock_guard<std::mutex> lk(mu_);
    const int64_t t = next_ticket_;
    const int sl = int(t % depth_);
    int rc = retire(sl);  // the slot's previous stripe must be out
    if (rc != ECGPU_OK) return rc;
    rc = enqueue(sl, t, data, coding);
    if (rc != ECGPU_OK) {
      // part of the stripe may already be queued against the caller's
      // buffers: let it finish before reporting, so no DMA outlives the call
      const std::string msg = ops_->last_error();
      ops_->sync_all();
      return ops_->fail(rc, msg);
    }
    slot_ticket_[size_t(sl)] = t;
    next_ticket_ = t + 1;
    return t;
  }

  int wait(int64_t ticket) {
    std::lock_guard<std::mutex> lk(mu_);
    return wait_locked(ticket);
  }

  int drain() {
    std::lock_guard<std::mutex> lk(mu_);
    if (next_ticket_ == 0) return ECGPU_OK;
    return wait_locked(next_ticket_ - 1);
  }

  // Joins the D2H worker after it has issued every queued job.
  void stop_worker() {
    {
      std::lock_guard<std::mutex> lk(qmu_);
      if (!worker_.joinable()) return;
      stop_ = true;
    }
    qcv_.notify_all();
    worker_.join();
  }

 private:
  struct Job {
    int slot;
    int64_t ticket;
    std::vector<char*> out;
  };

  // caller holds mu_
  int wait_locked(int64_t ticket) {
    if (ticket < 0) return ops_->fail(ECGPU_ERR_ARG, "ecgpu_pipeline_wait: bad ticket");
    if (ticket < done_below_) return ECGPU_OK;
    if (ticket >= next_ticket_) return ops_->fail(ECGPU_ERR_ARG, "ecgpu_pipeline_wait: ticket not submitted");
    // completion is in ticket order: retire every slot up to the ticket's
    for (int64_t t = done_below_; t <= ticket; ++t) {
      const int rc = retire(int(t % depth_));
      if (rc != ECGPU_OK) return rc;
    }
    return ECGPU_OK;
  }

  // caller holds mu_
  int retire(int slot) {
    const int64_t t = slot_ticket_[size_t(slot)];
    if (t < 0) return ECGPU_OK;
    {
      // the slot's drained event means something only once ITS ticket's D2H
      // has been issued
      std::unique_lock<std::mutex> lk(qmu_);
#ifdef ECGPU_MUTANT_R2_D2H
      qcv_.wait(lk, [&] { return issued_below_ > t; });
#else
      qcv_.wait(lk, [&] { return slot_issued_[size_t(slot)] >= t; });
#endif
      if (worker_rc_ != ECGPU_OK) return ops_->fail(worker_rc_, worker_err_);
    }
    if (int rc = ops_->sync_drained(slot)) return rc;
    slot_ticket_[size_t(slot)] = -1;
    if (t + 1 > done_below_) done_below_ = t + 1;
    return ECGPU_OK;
  }

  // caller holds mu_ (so no other enqueue runs concurrently)
  int enqueue(int sl, int64_t t, char** data, char** coding) {
    std::vector<char*> out;
    bool blocks = false;
    if (int rc = ops_->stage(sl, data, coding, &out, &blocks)) return rc;
    std::unique_lock<std::mutex> lk(qmu_);
    if (worker_rc_ != ECGPU_OK) return ops_->fail(worker_rc_, worker_err_);
#ifdef ECGPU_MUTANT_R2_D2H
    const bool earlier_pending = !q_.empty();
#else
    const bool earlier_pending = !q_.empty() || issued_below_ != t;
#endif
    if ((blocks && worker_enabled_) || earlier_pending) {
      // behind every earlier ticket, so the D2H stream keeps ticket order
      if (!worker_.joinable()) worker_ = std::thread([this] { worker_main(); });
      q_.push_back(Job{sl, t, std::move(out)});
      lk.unlock();
      qcv_.notify_all();
      return ECGPU_OK;
    }
    lk.unlock();
    // every earlier ticket is issued and the worker holds no job; no other
    // enqueue can start until this one returns (mu_)
    if (int rc = ops_->d2h(sl, out)) return rc;
    lk.lock();
    mark_issued(sl, t);
    lk.unlock();
    qcv_.notify_all();
    return ECGPU_OK;
  }

  // caller holds qmu_
  void mark_issued(int slot, int64_t t) {
#ifdef ECGPU_MUTANT_R2_D2H
    issued_below_ = t + 1;
#else
    issued_below_ = std::max(issued_below_, t + 1);
#endif
    slot_issued_[size_t(slot)] = std::max(slot_issued_[size_t(slot)], t);
  }

  void worker_main() {
    ops_->bind_thread();
    for (;;) {
      Job job;
      bool failed_before = false;
      {
        std::unique_lock<std::mutex> lk(qmu_);
        qcv_.wait(lk, [&] { return stop_ || !q_.empty(); });
        if (q_.empty()) return;  // stop, nothing left
        job = std::move(q_.front());
        q_.pop_front();
        failed_before = worker_rc_ != ECGPU_OK;
      }
      if (test_delay_us_ > 0)  // widens the pop -> issue window (ECGPU_TEST_D2H_DELAY_US)
        std::this_thread::sleep_for(std::chrono::microseconds(test_delay_us_));
      // after a failure the later jobs are abandoned (their retire reports it)
      const int rc = failed_before ? ECGPU_OK : ops_->d2h(job.slot, job.out);
      const std::string msg = rc != ECGPU_OK ? ops_->last_error() : std::string();
      {
        std::lock_guard<std::mutex> lk(qmu_);
        if (rc != ECGPU_OK && worker_rc_ == ECGPU_OK) {
          worker_rc_ = rc;
          worker_err_ = msg;
        }
        mark_issued(job.slot, job.ticket);
      }
      qcv_.notify_all();
    }
  }

  Ops* ops_;
  const int depth_;
  const bool worker_enabled_;
  const int test_delay_us_;
  // submit side (mu_)
  std::mutex mu_;
  std::vector<int64_t> slot_ticket_;  // ticket occupying each slot (-1: free)
  int64_t next_ticket_ = 0;
  int64_t done_below_ = 0;  // every ticket < done_below_ has completed
  // D2H issue side (qmu_)
  std::mutex qmu_;
  std::condition_variable qcv_;
  std::deque<Job> q_;
  std::vector<int64_t> slot_issued_;  // latest ticket whose D2H (drained record) is issued, per slot
  int64_t issued_below_ = 0;          // every ticket < issued_below_ is issued
  bool stop_ = false;
  int worker_rc_ = ECGPU_OK;  // first failure of a worker-issued D2H
  std::string worker_err_;
  std::thread worker_;
};

// ---------------------------------------------------------------------------
// MemberQueue: jobs handed in by any number of threads under local tickets
// 0, 1, 2, ... (possibly out of order), consumed in ticket order by one
// worker thread.  put() blocks while `cap` jobs wait ahead of the worker,
// except for the ticket the worker needs next.
// ---------------------------------------------------------------------------
template <class Job>
class MemberQueue {
 public:
  explicit MemberQueue(int cap) : cap_(std::max(1, cap)) {}

  void put(int64_t local, Job job) {
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_space_.wait(lk, [&] { return int64_t(pending_.size()) < cap_ || local <= next_local_; });
      pending_.emplace(local, std::move(job));
    }
    cv_job_.notify_all();
  }

  // Worker loop: submit(job) returns < 0 on failure (and then its message);
  // every later ticket is reported failed with the first failure.
  void run(const std::function<int64_t(Job&, std::string*)>& submit) {
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_job_.wait(lk, [&] { return stop_ || pending_.count(next_local_) != 0; });
      auto it = pending_.find(next_local_);
      if (it == pending_.end()) return;  // stop, nothing left for this ticket
      Job job = std::move(it->second);
      pending_.erase(it);
      cv_space_.notify_all();
      if (failed_from_ < 0) {
        lk.unlock();
        std::string msg;
        const int64_t r = submit(job, &msg);
        lk.lock();
        if (r < 0) {
          failed_from_ = next_local_;
          failed_rc_ = int(r);
          failed_msg_ = msg;
        }
      }
      ++next_local_;
#ifndef ECGPU_MUTANT_R2_WAKEUP
      cv_space_.notify_all();  // admits a put() waiting for exactly this ticket
#endif
      cv_done_.notify_all();
    }
  }

  // Blocks until the worker has handled `local`; its failure code (and
  // message) if it or an earlier ticket failed to submit, else ECGPU_OK.
  int wait_handled(int64_t local, std::string* msg) {
    std::unique_lock<std::mutex> lk(mu_);
    cv_done_.wait(lk, [&] { return next_local_ > local; });
    if (failed_from_ >= 0 && local >= failed_from_) {
      *msg = failed_msg_;
      return failed_rc_;
    }
    return ECGPU_OK;
  }

  void stop() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_job_.notify_all();
  }

 private:
  const int cap_;
  std::mutex mu_;
  std::condition_variable cv_job_, cv_done_, cv_space_;
  std::map<int64_t, Job> pending_;  // local ticket -> job
  int64_t next_local_ = 0;          // next local ticket the worker takes
  int64_t failed_from_ = -1;        // first local ticket whose submit failed (sticky)
  int failed_rc_ = ECGPU_OK;
  std::string failed_msg_;
  bool stop_ = false;
};

// ---------------------------------------------------------------------------
// IdlePool: idle objects keyed by device.  acquire() hands one out (or null:
// the caller makes a new one), release() takes it back.  Objects are never
// destroyed (process lifetime).
// ---------------------------------------------------------------------------
template <class T>
class IdlePool {
 public:
  T* acquire(int device) {
    std::lock_guard<std::mutex> lk(mu_);
    for (size_t i = 0; i < idle_.size(); ++i)
      if (idle_[i].first == device) {
        T* c = idle_[i].second;
        idle_.erase(idle_.begin() + long(i));
        return c;
      }
    return nullptr;
  }
  void release(int device, T* c) {
    std::lock_guard<std::mutex> lk(mu_);
    idle_.emplace_back(device, c);
  }

 private:
  std::mutex mu_;
  std::vector<std::pair<int, T*>> idle_;
};

// ---------------------------------------------------------------------------
// PerDevice: one object per device ordinal, made on first use by make(device)
// (a failed make, returning the null value, is retried on the next get).
// ---------------------------------------------------------------------------
template <class T>
class PerDevice {
 public:
  template <class Make>
  T get(int device, Make make) {
    std::lock_guard<std::mutex> lk(mu_);
    if (size_t(device) >= objs_.size()) objs_.resize(size_t(device) + 1, T{});
    if (!objs_[size_t(device)]) objs_[size_t(device)] = make(device);
    return objs_[size_t(device)];
  }

 private:
  std::mutex mu_;
  std::vector<T> objs_;
};

}  // namespace hostsync
}  // namespace ecgpu
