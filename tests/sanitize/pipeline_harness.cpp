// pipeline_harness.cpp -- the threaded host runtime's synchronisation
// (csrc/host_sync.hpp: the host pipeline's ticket / slot / D2H-worker state
// machine, the pipeline groups' member queues, the context pool, per-device
// lazy objects) driven on a FAKE device, built with -fsanitize=thread by
// tests/test_sanitizers.py.  No HIP: host_sync.hpp is the exact code that
// libecgpu's pipeline.hip and ecgpu_runtime.hip instantiate with HIP ops.
//
// The fake device: every stream is a thread running its queue in order, each
// operation after a random delay; an event is a counter pair (recorded /
// completed) -- a host sync or a stream wait on it waits for its LAST record,
// as hipEventSynchronize / hipStreamWaitEvent do.  Copies into or out of
// "pageable" host buffers block the issuing thread until they are done (HIP's
// pageable copies do); "pinned" ones return at once.  Memory is plain host
// memory, so a slot reused while a copy still reads it, or a host buffer read
// before its D2H wrote it, is a data race TSan reports -- and the checks
// below see the wrong bytes.
//
//   pipeline_harness pipe <iterations> <seed> [s]   random pipelines, checks every
//                                                   stripe right after wait(t)
//   pipeline_harness group <iterations> <seed> [s]  member queues under racing putters
//   pipeline_harness pool <threads> 0 [s]           IdlePool / PerDevice
//
// A watchdog aborts with "HANG" (exit 3) when the phase takes more than s
// seconds (default 240); a wrong result exits 2.
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <random>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "host_sync.hpp"

using ecgpu::hostsync::IdlePool;
using ecgpu::hostsync::MemberQueue;
using ecgpu::hostsync::PerDevice;
using ecgpu::hostsync::StripePipeline;

namespace {

[[noreturn]] void die(const char* what, long a = 0, long b = 0, long c = 0) {
  std::fprintf(stderr, "FAIL: %s (%ld, %ld, %ld)\n", what, a, b, c);
  std::fflush(stderr);
  std::_Exit(2);
}

// ---- watchdog ---------------------------------------------------------------
// (polls an atomic: GCC 11's timed condition waits use pthread_cond_clockwait,
// which this TSan does not intercept)
struct Watchdog {
  std::atomic<bool> done{false};
  std::thread th;
  Watchdog(const char* phase, int seconds) {
    th = std::thread([this, phase, seconds] {
      const auto end = std::chrono::steady_clock::now() + std::chrono::seconds(seconds);
      while (!done.load()) {
        if (std::chrono::steady_clock::now() > end) {
          std::fprintf(stderr, "HANG: %s did not finish in %d s\n", phase, seconds);
          std::fflush(stderr);
          std::_Exit(3);
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(20));
      }
    });
  }
  ~Watchdog() {
    done = true;
    th.join();
  }
};

thread_local std::mt19937 t_rng{std::random_device{}()};
void jitter(int max_us) {
  if (max_us <= 0) return;
  std::uniform_int_distribution<int> d(0, max_us);
  const int us = d(t_rng);
  if (us > max_us / 2) std::this_thread::sleep_for(std::chrono::microseconds(us));
  else std::this_thread::yield();
}

// ---- fake device -----------------------------------------------------------
struct FakeEvent {
  std::mutex mu;
  std::condition_variable cv;
  int64_t recorded = 0, completed = 0;
};

class FakeStream {
 public:
  explicit FakeStream(int jitter_us) : jitter_us_(jitter_us), th_([this] { loop(); }) {}
  ~FakeStream() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    th_.join();
  }
  void push(std::function<void()> fn) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      q_.push_back(std::move(fn));
    }
    cv_.notify_all();
  }
  // the stream's work up to now has run (a fresh event, recorded and waited)
  void sync() {
    auto ev = std::make_shared<FakeEvent>();
    record(ev.get());
    push([ev] {});  // keeps the event alive until the stream is past its record
    host_wait(ev.get());
  }
  void record(FakeEvent* ev) {
    int64_t g;
    {
      std::lock_guard<std::mutex> lk(ev->mu);
      g = ++ev->recorded;
    }
    push([ev, g] {
      std::lock_guard<std::mutex> lk(ev->mu);
      ev->completed = std::max(ev->completed, g);
      ev->cv.notify_all();
    });
  }
  void wait_event(FakeEvent* ev) {  // hipStreamWaitEvent: the event's latest record
    int64_t g;
    {
      std::lock_guard<std::mutex> lk(ev->mu);
      g = ev->recorded;
    }
    push([ev, g] {
      std::unique_lock<std::mutex> lk(ev->mu);
      ev->cv.wait(lk, [&] { return ev->completed >= g; });
    });
  }
  static void host_wait(FakeEvent* ev) {  // hipEventSynchronize
    std::unique_lock<std::mutex> lk(ev->mu);
    const int64_t g = ev->recorded;
    ev->cv.wait(lk, [&] { return ev->completed >= g; });
  }

 private:
  void loop() {
    for (;;) {
      std::function<void()> fn;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
        if (q_.empty()) return;
        fn = std::move(q_.front());
        q_.pop_front();
      }
      jitter(jitter_us_);
      fn();
    }
  }
  int jitter_us_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
  bool stop_ = false;
  std::thread th_;
};

// Byte map of the fake "kernel": output row i = f(i, sources).  Any function
// of every source byte does; expected() recomputes it on the host.
inline uint8_t apply_byte(int i, const uint8_t* src, int nsrc) {
  uint8_t acc = uint8_t(0x5A + 17 * i);
  for (int j = 0; j < nsrc; ++j) acc = uint8_t((acc ^ src[j]) * 3 + j + i);
  return acc;
}

thread_local std::string t_fake_err;
std::atomic<long> g_inline_d2h{0}, g_worker_d2h{0};

// hostsync::StripePipeline's Ops on the fake device.
struct FakePipeOps {
  int k, m, depth;
  size_t size;
  std::set<const char*>* pinned;  // buffers whose copies do not block
  std::vector<std::vector<uint8_t>> ring;  // per slot: k inputs then m outputs, each `size`
  std::vector<std::unique_ptr<FakeEvent>> loaded, computed, drained;
  std::unique_ptr<FakeStream> s_h2d, s_comp, s_d2h;
  std::thread::id submitter;

  FakePipeOps(int k_, int m_, int depth_, size_t size_, std::set<const char*>* pinned_, int jitter_us)
      : k(k_), m(m_), depth(depth_), size(size_), pinned(pinned_) {
    ring.assign(size_t(depth), std::vector<uint8_t>(size_t(k + m) * size));
    for (auto* v : {&loaded, &computed, &drained})
      for (int i = 0; i < depth; ++i) v->push_back(std::make_unique<FakeEvent>());
    s_h2d = std::make_unique<FakeStream>(jitter_us);
    s_comp = std::make_unique<FakeStream>(jitter_us);
    s_d2h = std::make_unique<FakeStream>(jitter_us);
  }
  uint8_t* shard(int slot, int j) { return ring[size_t(slot)].data() + size_t(j) * size; }
  bool is_pinned(const char* p) const { return pinned->count(p) != 0; }

  // a copy on stream s; a pageable one blocks the caller until it is done
  void copy(FakeStream* s, uint8_t* dst, const uint8_t* src, bool blocking) {
    const size_t n = size;
    if (!blocking) {
      s->push([=] { std::memcpy(dst, src, n); });
      return;
    }
    auto done = std::make_shared<FakeEvent>();
    s->push([=] { std::memcpy(dst, src, n); });
    s->record(done.get());
    s->push([done] {});  // keeps the event alive until the stream is past its record
    FakeStream::host_wait(done.get());
  }

  int stage(int sl, char** data, char** coding, std::vector<char*>* out, bool* out_blocks) {
    for (int j = 0; j < k; ++j)
      copy(s_h2d.get(), shard(sl, j), reinterpret_cast<const uint8_t*>(data[j]), !is_pinned(data[j]));
    s_h2d->record(loaded[size_t(sl)].get());
    s_comp->wait_event(loaded[size_t(sl)].get());
    uint8_t* base = shard(sl, 0);
    const int kk = k, mm = m;
    const size_t n = size;
    s_comp->push([=] {
      std::vector<uint8_t> col(static_cast<size_t>(kk));
      for (size_t b = 0; b < n; ++b) {
        for (int j = 0; j < kk; ++j) col[size_t(j)] = base[size_t(j) * n + b];
        for (int i = 0; i < mm; ++i) base[size_t(kk + i) * n + b] = apply_byte(i, col.data(), kk);
      }
    });
    s_comp->record(computed[size_t(sl)].get());
    out->assign(coding, coding + m);
    bool pageable = false;
    for (char* h : *out) pageable = pageable || !is_pinned(h);
    *out_blocks = pageable;
    return ECGPU_OK;
  }

  int d2h(int sl, const std::vector<char*>& out) {
    (std::this_thread::get_id() == submitter ? g_inline_d2h : g_worker_d2h)++;
    s_d2h->wait_event(computed[size_t(sl)].get());
    for (int i = 0; i < m; ++i)
      copy(s_d2h.get(), reinterpret_cast<uint8_t*>(out[size_t(i)]), shard(sl, k + i), !is_pinned(out[size_t(i)]));
    s_d2h->record(drained[size_t(sl)].get());
    return ECGPU_OK;
  }

  int sync_drained(int sl) {
    FakeStream::host_wait(drained[size_t(sl)].get());
    return ECGPU_OK;
  }
  void sync_all() {
    s_h2d->sync();
    s_comp->sync();
    s_d2h->sync();
  }
  void bind_thread() {}
  int fail(int rc, const std::string& msg) {
    t_fake_err = msg;
    return rc;
  }
  std::string last_error() const { return t_fake_err; }
};

// One random pipeline run: `stripes` stripes of k data / m coding host
// buffers, pinned or pageable per buffer by pattern; after every submit a
// random earlier ticket may be waited, and every stripe is checked right
// after the first wait that covers it (before any later submit can reuse
// its slot).  The last stripes are drained.
void run_pipeline(std::mt19937& rng, int iter) {
  const int k = 1 + int(rng() % 6), m = 1 + int(rng() % 3), depth = 1 + int(rng() % 3);
  const size_t size = 64 + rng() % 512;
  const int stripes = 6 + int(rng() % 14);
  const int pattern = int(rng() % 4);  // 0 alternate, 1 random, 2 pageable then pinned, 3 all pinned
  const int delay_us = int(rng() % 3) * 150;  // the ECGPU_TEST_D2H_DELAY_US window
  const int jitter_us = int(rng() % 2) * 60;
  const bool worker = rng() % 8 != 0;
  std::set<const char*> pinned;
  std::vector<std::vector<std::vector<char>>> data(static_cast<size_t>(stripes)), coding(static_cast<size_t>(stripes));
  for (int s = 0; s < stripes; ++s) {
    const bool out_pinned = pattern == 0 ? s % 2 == 1
                            : pattern == 1 ? rng() % 2 == 0
                            : pattern == 2 ? s >= stripes / 2 : true;
    for (int j = 0; j < k; ++j) {
      data[size_t(s)].emplace_back(size);
      for (auto& c : data[size_t(s)].back()) c = char(rng());
      pinned.insert(data[size_t(s)].back().data());  // pinned inputs: the H2D never slows the submitter
    }
    for (int i = 0; i < m; ++i) {
      coding[size_t(s)].emplace_back(size, char(0x77));
      if (out_pinned) pinned.insert(coding[size_t(s)].back().data());
    }
  }
  auto check = [&](int s) {
    std::vector<uint8_t> col(static_cast<size_t>(k));
    for (size_t b = 0; b < size; ++b) {
      for (int j = 0; j < k; ++j) col[size_t(j)] = uint8_t(data[size_t(s)][size_t(j)][b]);
      for (int i = 0; i < m; ++i)
        if (uint8_t(coding[size_t(s)][size_t(i)][b]) != apply_byte(i, col.data(), k))
          die("stripe output wrong right after wait()", iter, s, i);
    }
  };
  FakePipeOps ops(k, m, depth, size, &pinned, jitter_us);
  ops.submitter = std::this_thread::get_id();
  {
    StripePipeline<FakePipeOps> p(&ops, depth, worker, delay_us);
    int checked = 0;
    std::vector<char*> dp(static_cast<size_t>(k)), cp(static_cast<size_t>(m));
    for (int s = 0; s < stripes; ++s) {
      for (int j = 0; j < k; ++j) dp[size_t(j)] = data[size_t(s)][size_t(j)].data();
      for (int i = 0; i < m; ++i) cp[size_t(i)] = coding[size_t(s)][size_t(i)].data();
      const int64_t t = p.submit(dp.data(), cp.data());
      if (t != s) die("submit ticket", iter, s, long(t));
      if (rng() % 3 == 0) {
        const int w = checked + int(rng() % size_t(s + 1 - checked));
        if (p.wait(w) != ECGPU_OK) die("wait failed", iter, w);
        for (; checked <= w; ++checked) check(checked);
      }
    }
    if (p.drain() != ECGPU_OK) die("drain failed", iter);
    for (; checked < stripes; ++checked) check(checked);
    if (p.wait(stripes) != ECGPU_ERR_ARG) die("wait on an unsubmitted ticket", iter);
  }
}

// Member queue: `nput` threads put local tickets 0..n-1 (claimed from an
// atomic counter, then put after a random delay, so they arrive out of
// order); the worker must see them in order; every wait_handled returns.
void run_group(std::mt19937& rng, int iter) {
  const int cap = 1 + int(rng() % 3), nput = cap + 2 + int(rng() % 4), n = 40 + int(rng() % 40);
  MemberQueue<int64_t> q(cap);
  std::vector<int64_t> seen;
  std::thread worker([&] {
    q.run([&](int64_t& job, std::string* msg) {
      jitter(80);
      seen.push_back(job);
      if (job == n + 7) {  // never: a failure path is exercised by run_group_failure
        *msg = "x";
        return int64_t(-1);
      }
      return job;
    });
  });
  std::atomic<int64_t> next{0};
  std::vector<std::thread> putters;
  for (int t = 0; t < nput; ++t)
    putters.emplace_back([&] {
      for (;;) {
        const int64_t local = next.fetch_add(1);
        if (local >= n) return;
        jitter(200);
        q.put(local, local);
      }
    });
  for (auto& th : putters) th.join();
  std::string msg;
  for (int64_t l = n - 1; l >= 0; l -= 7)
    if (q.wait_handled(l, &msg) != ECGPU_OK) die("wait_handled", iter, long(l));
  q.stop();
  worker.join();
  if (int(seen.size()) != n) die("jobs lost", iter, long(seen.size()), n);
  for (int i = 0; i < n; ++i)
    if (seen[size_t(i)] != i) die("jobs out of order", iter, i, long(seen[size_t(i)]));
}

// The lost wake-up of round 2, constructed: with cap 2, tickets 2 and 3 fill
// the queue, ticket 1 blocks in put(), then ticket 0 (always admitted) goes
// in.  The worker takes 0; ticket 1 may enter only once next_local reaches 1.
void run_group_wakeup() {
  MemberQueue<int64_t> q(2);
  std::vector<int64_t> seen;
  std::mutex smu;
  std::thread worker([&] {
    q.run([&](int64_t& job, std::string*) {
      std::this_thread::sleep_for(std::chrono::milliseconds(job == 0 ? 50 : 1));
      std::lock_guard<std::mutex> lk(smu);
      seen.push_back(job);
      return job;
    });
  });
  q.put(2, 2);
  q.put(3, 3);
  std::thread one([&] { q.put(1, 1); });
  std::this_thread::sleep_for(std::chrono::milliseconds(30));  // ticket 1 is blocked now
  q.put(0, 0);
  one.join();
  std::string msg;
  if (q.wait_handled(3, &msg) != ECGPU_OK) die("wait_handled");
  q.stop();
  worker.join();
  if (seen != std::vector<int64_t>({0, 1, 2, 3})) die("wake-up order");
}

// A failing submit: its ticket and every later one report the failure.
void run_group_failure() {
  MemberQueue<int64_t> q(2);
  std::thread worker([&] {
    q.run([&](int64_t& job, std::string* msg) {
      if (job == 3) {
        *msg = "device lost";
        return int64_t(-3);
      }
      return job;
    });
  });
  for (int64_t l = 0; l < 6; ++l) q.put(l, l);
  std::string msg;
  if (q.wait_handled(2, &msg) != ECGPU_OK) die("failure: early ticket");
  if (q.wait_handled(5, &msg) != -3 || msg != "device lost") die("failure: later ticket");
  q.stop();
  worker.join();
}

void run_pool(int threads) {
  struct Obj {
    int device;
    std::atomic<int> users{0};
  };
  IdlePool<Obj> pool;
  PerDevice<Obj*> lazy;
  std::mutex made_mu;
  std::vector<std::unique_ptr<Obj>> made;
  std::atomic<int> creations{0};
  std::vector<std::thread> ts;
  for (int t = 0; t < threads; ++t)
    ts.emplace_back([&, t] {
      std::mt19937 rng(static_cast<unsigned>(t));
      for (int i = 0; i < 2000; ++i) {
        const int dev = int(rng() % 3);
        Obj* o = pool.acquire(dev);
        if (!o) {
          std::lock_guard<std::mutex> lk(made_mu);
          made.push_back(std::make_unique<Obj>());
          made.back()->device = dev;
          o = made.back().get();
        }
        if (o->device != dev) die("pool: wrong device");
        if (o->users.fetch_add(1) != 0) die("pool: object handed out twice");
        jitter(5);
        o->users.fetch_sub(1);
        pool.release(dev, o);
        Obj* u = lazy.get(dev, [&](int d) {
          creations++;
          std::lock_guard<std::mutex> lk(made_mu);
          made.push_back(std::make_unique<Obj>());
          made.back()->device = d;
          return made.back().get();
        });
        if (u->device != dev) die("per-device: wrong object");
      }
    });
  for (auto& th : ts) th.join();
  if (creations.load() > 3) die("per-device: made more than once", creations.load());
}

}  // namespace

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "pipe";
  const int n = argc > 2 ? std::atoi(argv[2]) : 40;
  const unsigned seed = argc > 3 ? unsigned(std::atoi(argv[3])) : 1u;
  const int limit_s = argc > 4 ? std::atoi(argv[4]) : 240;  // watchdog
  std::mt19937 rng(seed);
  if (mode == "pipe") {
    Watchdog wd("pipeline runs", limit_s);
    for (int i = 0; i < n; ++i) run_pipeline(rng, i);
    std::printf("pipeline harness ok: %d runs, %ld D2H issued inline, %ld by the worker\n", n, g_inline_d2h.load(),
                g_worker_d2h.load());
  } else if (mode == "group") {
    Watchdog wd("member queues", limit_s);
    run_group_wakeup();
    run_group_failure();
    for (int i = 0; i < n; ++i) run_group(rng, i);
    std::printf("group harness ok: %d runs\n", n);
  } else if (mode == "pool") {
    Watchdog wd("pool", limit_s);
    run_pool(n);
    std::printf("pool harness ok: %d threads\n", n);
  } else {
    std::fprintf(stderr, "usage: %s pipe|group|pool [n] [seed]\n", argv[0]);
    return 1;
  }
  return 0;
}
