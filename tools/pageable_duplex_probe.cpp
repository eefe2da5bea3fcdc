// pageable_duplex_probe.cpp -- can pageable H2D and D2H copies overlap if
// they are issued from two host threads?  (HIP stages pageable copies
// through its own pinned buffers and blocks the issuing thread; a pipeline
// that issues both directions from one thread serialises them.)
// Prints JSON lines: H2D alone, D2H alone, both from one thread, both from
// two threads (each on its own stream), for the RS(10,4) 4 MiB stripe shape
// (10 x 4 MiB in, 4 x 4 MiB out, one copy per shard), medians of 9.
// Built by tools/build_tools.sh.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

namespace {

double now_us() {
  using namespace std::chrono;
  return duration<double, std::micro>(steady_clock::now().time_since_epoch()).count();
}

#define CK(x)                                                      \
  do {                                                             \
    hipError_t e_ = (x);                                           \
    if (e_ != hipSuccess) {                                        \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); \
      std::exit(1);                                                \
    }                                                              \
  } while (0)

double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

}  // namespace

int main() {
  CK(hipSetDevice(0));
  const size_t S = size_t(4) << 20;
  const int k = 10, m = 4;
  hipStream_t s_in, s_out;
  CK(hipStreamCreateWithFlags(&s_in, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s_out, hipStreamNonBlocking));
  std::vector<char*> hin(k), hout(m);
  for (auto& p : hin) {
    p = static_cast<char*>(std::malloc(S));
    std::memset(p, 3, S);
  }
  for (auto& p : hout) {
    p = static_cast<char*>(std::malloc(S));
    std::memset(p, 0, S);
  }
  char* dev = nullptr;
  CK(hipMalloc(reinterpret_cast<void**>(&dev), (k + m) * S));
  CK(hipMemset(dev, 1, (k + m) * S));

  auto h2d = [&] {
    for (int j = 0; j < k; ++j) CK(hipMemcpyAsync(dev + j * S, hin[j], S, hipMemcpyHostToDevice, s_in));
    CK(hipStreamSynchronize(s_in));
  };
  auto d2h = [&] {
    for (int i = 0; i < m; ++i) CK(hipMemcpyAsync(hout[i], dev + (k + i) * S, S, hipMemcpyDeviceToHost, s_out));
    CK(hipStreamSynchronize(s_out));
  };
  auto bench = [&](const char* name, auto&& fn) {
    fn();
    std::vector<double> t;
    for (int r = 0; r < 9; ++r) {
      const double t0 = now_us();
      fn();
      t.push_back(now_us() - t0);
    }
    const double us = median(t);
    std::printf("{\"probe\": \"pageable %s\", \"us\": %.1f, \"in_GBps\": %.1f, \"out_GBps\": %.1f}\n", name, us,
                double(k * S) / (us * 1e3), double(m * S) / (us * 1e3));
    std::fflush(stdout);
  };
  // D2H variants: stream flags, copy kind, one contiguous copy
  hipStream_t s_blk;
  CK(hipStreamCreateWithFlags(&s_blk, hipStreamDefault));
  char* hslab = static_cast<char*>(std::malloc(m * S));
  std::memset(hslab, 0, m * S);
  bench("D2H 4 x 4 MiB, blocking stream, kind Default", [&] {
    for (int i = 0; i < m; ++i) CK(hipMemcpyAsync(hout[i], dev + (k + i) * S, S, hipMemcpyDefault, s_blk));
    CK(hipStreamSynchronize(s_blk));
  });
  bench("D2H 4 x 4 MiB, blocking stream, kind DeviceToHost", [&] {
    for (int i = 0; i < m; ++i) CK(hipMemcpyAsync(hout[i], dev + (k + i) * S, S, hipMemcpyDeviceToHost, s_blk));
    CK(hipStreamSynchronize(s_blk));
  });
  bench("D2H 4 x 4 MiB, non-blocking stream, kind Default", [&] {
    for (int i = 0; i < m; ++i) CK(hipMemcpyAsync(hout[i], dev + (k + i) * S, S, hipMemcpyDefault, s_out));
    CK(hipStreamSynchronize(s_out));
  });
  bench("D2H one 16 MiB copy, non-blocking stream", [&] {
    CK(hipMemcpyAsync(hslab, dev + k * S, m * S, hipMemcpyDeviceToHost, s_out));
    CK(hipStreamSynchronize(s_out));
  });
  bench("D2H 4 x 4 MiB, blocking hipMemcpy", [&] {
    for (int i = 0; i < m; ++i) CK(hipMemcpy(hout[i], dev + (k + i) * S, S, hipMemcpyDeviceToHost));
  });
  // does a pageable range that once was an H2D source take a faster D2H path?
  for (size_t n : {size_t(1) << 20, size_t(4) << 20}) {
    char* fresh = static_cast<char*>(std::malloc(n));
    char* used = static_cast<char*>(std::malloc(n));
    std::memset(fresh, 0, n);
    std::memset(used, 0, n);
    CK(hipMemcpy(dev, used, n, hipMemcpyHostToDevice));
    char name[96];
    std::snprintf(name, sizeof(name), "D2H %zu KiB into a buffer never copied H2D", n >> 10);
    bench(name, [&] {
      CK(hipMemcpyAsync(fresh, dev, n, hipMemcpyDeviceToHost, s_blk));
      CK(hipStreamSynchronize(s_blk));
    });
    std::snprintf(name, sizeof(name), "D2H %zu KiB into a buffer once copied H2D", n >> 10);
    bench(name, [&] {
      CK(hipMemcpyAsync(used, dev, n, hipMemcpyDeviceToHost, s_blk));
      CK(hipStreamSynchronize(s_blk));
    });
    std::snprintf(name, sizeof(name), "H2D %zu KiB", n >> 10);
    bench(name, [&] {
      CK(hipMemcpyAsync(dev, used, n, hipMemcpyHostToDevice, s_blk));
      CK(hipStreamSynchronize(s_blk));
    });
    std::free(fresh);
    std::free(used);
  }
  // the H2D of one stripe split over two issuing threads (two streams)
  hipStream_t s_in2;
  CK(hipStreamCreateWithFlags(&s_in2, hipStreamNonBlocking));
  bench("H2D 10 x 4 MiB from two threads (5 shards each)", [&] {
    std::thread t([&] {
      for (int j = 5; j < k; ++j) CK(hipMemcpyAsync(dev + j * S, hin[j], S, hipMemcpyHostToDevice, s_in2));
      CK(hipStreamSynchronize(s_in2));
    });
    for (int j = 0; j < 5; ++j) CK(hipMemcpyAsync(dev + j * S, hin[j], S, hipMemcpyHostToDevice, s_in));
    CK(hipStreamSynchronize(s_in));
    t.join();
  });
  bench("H2D 10 x 4 MiB alone", h2d);
  bench("D2H 4 x 4 MiB alone", d2h);
  bench("H2D then D2H, one thread", [&] {
    h2d();
    d2h();
  });
  bench("H2D and D2H from two threads", [&] {
    std::thread t(d2h);
    h2d();
    t.join();
  });
  // the pipeline shape: stripe i's D2H from a worker while stripe i+1's H2D
  // is issued by the caller, 8 stripes
  bench("8-stripe pipeline, D2H on a worker thread (per stripe)", [&] {
    for (int st = 0; st < 8; ++st) {
      std::thread t(d2h);
      h2d();
      t.join();
    }
  });
  bench("8-stripe sequence, one thread (per stripe)", [&] {
    for (int st = 0; st < 8; ++st) {
      h2d();
      d2h();
    }
  });
  CK(hipFree(dev));
  for (auto* p : hin) std::free(p);
  for (auto* p : hout) std::free(p);
  return 0;
}
