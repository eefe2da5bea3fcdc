// hip_overheads.cpp -- per-call costs of the HIP runtime primitives a
// synchronous drop-in call is built from, and host memcpy bandwidth
// (pageable -> pinned) per thread count.  Medians in microseconds, one JSON
// line per primitive.  Used to budget the synchronous path.
//
// Built by tools/build_tools.sh.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <thread>
#include <vector>

namespace {

double now_us() {
  using namespace std::chrono;
  return duration<double, std::micro>(steady_clock::now().time_since_epoch()).count();
}

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
      std::exit(1);                                                              \
    }                                                                            \
  } while (0)

void report(const char* name, std::vector<double> v, const char* extra = "") {
  std::sort(v.begin(), v.end());
  std::printf("{\"op\": \"%s\", \"median_us\": %.2f, \"p10_us\": %.2f, \"p90_us\": %.2f%s}\n", name, v[v.size() / 2],
              v[v.size() / 10], v[v.size() * 9 / 10], extra);
  std::fflush(stdout);
}

void time_op(const char* name, int reps, const std::function<void()>& f, const char* extra = "") {
  for (int i = 0; i < 5; ++i) f();
  std::vector<double> v;
  for (int i = 0; i < reps; ++i) {
    const double t0 = now_us();
    f();
    v.push_back(now_us() - t0);
  }
  report(name, v, extra);
}

__global__ void empty_kernel(int* p) {
  if (p && threadIdx.x == 0 && blockIdx.x == 0) p[0] = 1;
}

void par_memcpy(char* dst, const char* src, size_t n, int threads) {
  if (threads <= 1) {
    std::memcpy(dst, src, n);
    return;
  }
  std::vector<std::thread> ts;
  const size_t per = (n / threads + 4095) & ~size_t(4095);
  for (int t = 0; t < threads; ++t) {
    const size_t a = std::min(n, per * t), b = std::min(n, per * (t + 1));
    if (a < b) ts.emplace_back([=] { std::memcpy(dst + a, src + a, b - a); });
  }
  for (auto& t : ts) t.join();
}

}  // namespace

int main() {
  CK(hipSetDevice(0));
  hipStream_t s, snb;
  CK(hipStreamCreateWithFlags(&s, hipStreamDefault));
  CK(hipStreamCreateWithFlags(&snb, hipStreamNonBlocking));
  void* d = nullptr;
  CK(hipMalloc(&d, 64 << 20));
  std::vector<char> pageable(64 << 20, 1);
  char* pinned = nullptr;
  CK(hipHostMalloc(reinterpret_cast<void**>(&pinned), 64 << 20, hipHostMallocDefault));

  time_op("hipStreamSynchronize (idle stream)", 500, [&] { CK(hipStreamSynchronize(s)); });
  time_op("hipPointerGetAttributes (host ptr)", 500, [&] {
    hipPointerAttribute_t a;
    (void)hipPointerGetAttributes(&a, pageable.data() + 4096);
    (void)hipGetLastError();
  });
  time_op("hipPointerGetAttributes (device ptr)", 500, [&] {
    hipPointerAttribute_t a;
    CK(hipPointerGetAttributes(&a, static_cast<char*>(d) + 4096));
  });
  time_op("hipMalloc+hipFree 4 KiB", 200, [&] {
    void* p;
    CK(hipMalloc(&p, 4096));
    CK(hipFree(p));
  });
  time_op("hipMalloc 4 KiB (no free)", 100, [&] {
    void* p;
    CK(hipMalloc(&p, 4096));
  });
  time_op("hipMallocAsync+hipFreeAsync 4 KiB + sync", 200, [&] {
    void* p;
    CK(hipMallocAsync(&p, 4096, snb));
    CK(hipFreeAsync(p, snb));
    CK(hipStreamSynchronize(snb));
  });
  time_op("hipMemcpy H2D 256 B pageable (blocking)", 500,
          [&] { CK(hipMemcpy(d, pageable.data(), 256, hipMemcpyHostToDevice)); });
  time_op("hipMemcpyAsync H2D 256 B pageable + sync", 500, [&] {
    CK(hipMemcpyAsync(d, pageable.data(), 256, hipMemcpyHostToDevice, s));
    CK(hipStreamSynchronize(s));
  });
  time_op("hipMemcpyAsync H2D 256 B pinned + sync", 500, [&] {
    CK(hipMemcpyAsync(d, pinned, 256, hipMemcpyHostToDevice, s));
    CK(hipStreamSynchronize(s));
  });
  time_op("hipMemcpyAsync H2D 256 B pageable (enqueue only)", 500, [&] {
    CK(hipMemcpyAsync(d, pageable.data(), 256, hipMemcpyHostToDevice, s));
  });
  CK(hipStreamSynchronize(s));
  time_op("hipMemcpyAsync H2D 256 B pinned (enqueue only)", 500,
          [&] { CK(hipMemcpyAsync(d, pinned, 256, hipMemcpyHostToDevice, s)); });
  CK(hipStreamSynchronize(s));
  time_op("kernel launch (enqueue only)", 500, [&] { hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, nullptr); });
  CK(hipStreamSynchronize(s));
  time_op("kernel launch + hipStreamSynchronize", 500, [&] {
    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, nullptr);
    CK(hipStreamSynchronize(s));
  });
  time_op("kernel launch + sync (non-blocking stream)", 500, [&] {
    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, snb, nullptr);
    CK(hipStreamSynchronize(snb));
  });
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  time_op("kernel + eventRecord + eventSynchronize", 500, [&] {
    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, snb, nullptr);
    CK(hipEventRecord(ev, snb));
    CK(hipEventSynchronize(ev));
  });
  time_op("kernel + eventRecord + hipEventQuery spin", 500, [&] {
    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, snb, nullptr);
    CK(hipEventRecord(ev, snb));
    while (hipEventQuery(ev) == hipErrorNotReady) {
    }
  });
  time_op("H2D 1 MiB pinned + sync", 200, [&] {
    CK(hipMemcpyAsync(d, pinned, 1 << 20, hipMemcpyHostToDevice, s));
    CK(hipStreamSynchronize(s));
  });
  time_op("H2D 1 MiB pageable + sync", 200, [&] {
    CK(hipMemcpyAsync(d, pageable.data(), 1 << 20, hipMemcpyHostToDevice, s));
    CK(hipStreamSynchronize(s));
  });
  time_op("D2H 1 MiB pinned + sync", 200, [&] {
    CK(hipMemcpyAsync(pinned, d, 1 << 20, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
  });
  time_op("H2D 6 MiB pinned + sync", 100, [&] {
    CK(hipMemcpyAsync(d, pinned, 6 << 20, hipMemcpyHostToDevice, s));
    CK(hipStreamSynchronize(s));
  });
  time_op("6 x H2D 1 MiB pinned + sync", 100, [&] {
    for (int i = 0; i < 6; ++i)
      CK(hipMemcpyAsync(static_cast<char*>(d) + (size_t(i) << 20), pinned + (size_t(i) << 20), 1 << 20,
                        hipMemcpyHostToDevice, s));
    CK(hipStreamSynchronize(s));
  });
  time_op("H2D 6 MiB pageable + sync", 100, [&] {
    CK(hipMemcpyAsync(d, pageable.data(), 6 << 20, hipMemcpyHostToDevice, s));
    CK(hipStreamSynchronize(s));
  });
  time_op("hipHostMalloc+hipHostFree 1 MiB", 50, [&] {
    void* p;
    CK(hipHostMalloc(&p, 1 << 20, hipHostMallocDefault));
    CK(hipHostFree(p));
  });
  time_op("hipHostRegister+Unregister 1 MiB", 50, [&] {
    CK(hipHostRegister(pageable.data() + (8 << 20), 1 << 20, hipHostRegisterDefault));
    CK(hipHostUnregister(pageable.data() + (8 << 20)));
  });
  std::vector<char> src2(64 << 20, 3);
  for (int th : {1, 2, 4, 8, 16}) {
    for (size_t n : {size_t(1) << 20, size_t(6) << 20, size_t(32) << 20}) {
      char name[128], extra[64];
      std::vector<double> v;
      for (int i = 0; i < 30; ++i) {
        const double t0 = now_us();
        par_memcpy(pinned, src2.data() + (i & 1) * (16 << 20) * 0, n, th);
        v.push_back(now_us() - t0);
      }
      std::sort(v.begin(), v.end());
      std::snprintf(name, sizeof name, "memcpy pageable->pinned %zu KiB, %d threads", n >> 10, th);
      std::snprintf(extra, sizeof extra, ", \"GBps\": %.1f", double(n) / (v[v.size() / 2] * 1e3));
      report(name, v, extra);
    }
  }
  return 0;
}
