// zero_copy_probe.cpp -- can a synchronous call on caller (pageable)
// buffers skip the staging copies?  Measures, on the GPU box:
//   * hipHostRegister / hipHostUnregister of fresh, already-touched malloc
//     ranges (the reference callers' buffers), per size;
//   * DMA from a freshly registered range;
//   * "zero-copy": a kernel reading host memory and/or writing host memory
//     directly over PCIe (registered pageable and hipHostMalloc pinned),
//     16 B per lane -- reads and writes go in opposite directions of the link,
//     so a kernel that reads k shards and writes m shards can overlap them.
// Every pointer a kernel touches is inside a range registered (or
// hipHostMalloc'd) just before the launch; registration is checked with
// hipPointerGetAttributes first and the probe exits on any failure.
// Built by tools/build_tools.sh.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// dst[i] = src[i] over n16 16-B words (either side may be host memory)
__global__ void copy16(const u32x4* __restrict__ src, u32x4* __restrict__ dst, int64_t n16) {
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n16; i += int64_t(gridDim.x) * blockDim.x)
    dst[i] = src[i];
}

// read a (host) and write b (host) in one kernel: b[i] = a[i % na] ^ c[i]
__global__ void duplex16(const u32x4* __restrict__ a, int64_t na, const u32x4* __restrict__ c, u32x4* __restrict__ b,
                         int64_t nb) {
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  const int64_t n = na > nb ? na : nb;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    u32x4 v = {0u, 0u, 0u, 0u};
    if (i < na) v = a[i];
    if (i < nb) b[i] = v ^ c[i];
  }
}

double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

void check_host_mapped(const void* p) {
  hipPointerAttribute_t attr;
  CK(hipPointerGetAttributes(&attr, p));
  if (attr.type != hipMemoryTypeHost) {
    std::fprintf(stderr, "not registered host memory: %p\n", p);
    std::exit(1);
  }
}

}  // namespace

int main() {
  CK(hipSetDevice(0));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const size_t pool = size_t(512) << 20;
  char* host = static_cast<char*>(std::malloc(pool));
  std::memset(host, 7, pool);  // touched, like a caller's filled buffers
  char* dev = nullptr;
  CK(hipMalloc(reinterpret_cast<void**>(&dev), 64 << 20));
  CK(hipMemset(dev, 1, 64 << 20));
  char* pinned = nullptr;
  CK(hipHostMalloc(reinterpret_cast<void**>(&pinned), 64 << 20, hipHostMallocDefault));
  std::memset(pinned, 5, 64 << 20);

  // 0. what HIP reports for host allocations the GPU can address in place:
  //    range start / size of the allocation a pointer lies in, device address
  auto range = [&](const char* name, const void* p) {
    hipPointerAttribute_t attr;
    const hipError_t e0 = hipPointerGetAttributes(&attr, p);
    void* start = nullptr;
    size_t rsize = 0;
    const hipError_t e1 = hipPointerGetAttribute(&start, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, (hipDeviceptr_t)p);
    const hipError_t e2 = hipPointerGetAttribute(&rsize, HIP_POINTER_ATTRIBUTE_RANGE_SIZE, (hipDeviceptr_t)p);
    void* dp = nullptr;
    const hipError_t e3 = hipHostGetDevicePointer(&dp, const_cast<void*>(p), 0);
    (void)hipGetLastError();
    std::printf("{\"probe\": \"range %s\", \"type\": %d, \"rc\": [%d, %d, %d, %d], \"offset_in_range\": %lld, "
                "\"range_size\": %zu, \"dev_equals_host\": %d}\n",
                name, e0 == hipSuccess ? int(attr.type) : -1, int(e0), int(e1), int(e2), int(e3),
                (long long)(static_cast<const char*>(p) - static_cast<const char*>(start)), rsize, int(dp == p));
    std::fflush(stdout);
  };
  range("hipHostMalloc base", pinned);
  range("hipHostMalloc +12345", pinned + 12345);
  {
    char* reg = host + 100003;  // not page aligned
    CK(hipHostRegister(reg, 3 << 20, hipHostRegisterDefault));
    range("registered base (unaligned)", reg);
    range("registered +1 MiB", reg + (1 << 20));
    range("registered last byte", reg + (3 << 20) - 1);
    range("just past registered", reg + (3 << 20) + 8192);
    CK(hipHostUnregister(reg));
  }
  range("pageable", host + 12345);

  // 1. registration cost on fresh ranges (never registered before)
  size_t off = 0;
  for (size_t n : {size_t(64) << 10, size_t(349525), size_t(1) << 20, size_t(6) << 20, size_t(16) << 20}) {
    std::vector<double> reg, unreg, dma;
    for (int i = 0; i < 12; ++i) {
      char* p = host + off;
      off += (n + (size_t(1) << 20)) & ~size_t(4095);
      if (off + n > pool) off = 0;
      const double t0 = now_us();
      CK(hipHostRegister(p, n, hipHostRegisterDefault));
      const double t1 = now_us();
      check_host_mapped(p);
      CK(hipMemcpyAsync(dev, p, n, hipMemcpyHostToDevice, s));
      CK(hipStreamSynchronize(s));
      const double t2 = now_us();
      CK(hipHostUnregister(p));
      const double t3 = now_us();
      if (i >= 2) {
        reg.push_back(t1 - t0);
        dma.push_back(t2 - t1);
        unreg.push_back(t3 - t2);
      }
    }
    std::printf("{\"probe\": \"register fresh range\", \"bytes\": %zu, \"register_us\": %.2f, \"h2d_us\": %.2f, "
                "\"unregister_us\": %.2f}\n",
                n, median(reg), median(dma), median(unreg));
    std::fflush(stdout);
  }

  // 2. zero-copy kernel bandwidth
  auto zc = [&](const char* name, const char* src, char* dst, size_t n) {
    std::vector<double> t;
    const int64_t n16 = int64_t(n / 16);
    const int grid = int(std::min<int64_t>((n16 + 255) / 256, 2048));
    for (int i = 0; i < 12; ++i) {
      const double t0 = now_us();
      hipLaunchKernelGGL(copy16, dim3(grid), dim3(256), 0, s, reinterpret_cast<const u32x4*>(src),
                         reinterpret_cast<u32x4*>(dst), n16);
      CK(hipStreamSynchronize(s));
      if (i >= 2) t.push_back(now_us() - t0);
    }
    const double us = median(t);
    std::printf("{\"probe\": \"zero-copy kernel %s\", \"bytes\": %zu, \"us\": %.2f, \"GBps\": %.1f}\n", name, n, us,
                double(n) / (us * 1e3));
    std::fflush(stdout);
  };
  for (size_t n : {size_t(64) << 10, size_t(1) << 20, size_t(6) << 20, size_t(32) << 20}) {
    zc("read pinned -> device", pinned, dev, n);
    zc("write device -> pinned", dev, pinned, n);
    char* p = host + (size_t(256) << 20);
    CK(hipHostRegister(p, n, hipHostRegisterDefault));
    check_host_mapped(p);
    void* dp = nullptr;
    CK(hipHostGetDevicePointer(&dp, p, 0));
    if (dp != p) std::printf("{\"note\": \"registered device pointer differs from host pointer\"}\n");
    zc("read registered pageable -> device", static_cast<char*>(dp), dev, n);
    zc("write device -> registered pageable", dev, static_cast<char*>(dp), n);
    CK(hipHostUnregister(p));
  }
  // 3. duplex: read 2n from pinned, write n to pinned, one kernel (C2-like 6:3)
  for (size_t n : {size_t(1) << 20, size_t(3) << 20, size_t(16) << 20}) {
    std::vector<double> t;
    const int64_t na = int64_t(2 * n / 16), nb = int64_t(n / 16);
    for (int i = 0; i < 12; ++i) {
      const double t0 = now_us();
      hipLaunchKernelGGL(duplex16, dim3(2048), dim3(256), 0, s, reinterpret_cast<const u32x4*>(pinned), na,
                         reinterpret_cast<const u32x4*>(dev), reinterpret_cast<u32x4*>(pinned + (32 << 20)), nb);
      CK(hipStreamSynchronize(s));
      if (i >= 2) t.push_back(now_us() - t0);
    }
    const double us = median(t);
    std::printf("{\"probe\": \"zero-copy duplex read 2n + write n (pinned)\", \"n\": %zu, \"us\": %.2f, "
                "\"read_GBps\": %.1f, \"write_GBps\": %.1f}\n",
                n, us, double(2 * n) / (us * 1e3), double(n) / (us * 1e3));
    std::fflush(stdout);
  }
  // 4. queued back-to-back 4 MiB reads of pinned memory (the ECX accumulator's
  //    per-block traffic): kernel reads at several grid sizes / words in
  //    flight per lane vs DMA, 20 in a row, one sync at the end
  {
    const size_t n = size_t(4) << 20;
    const int reps = 20;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto queued = [&](const char* name, auto&& one) {
      for (int w = 0; w < 3; ++w) one();
      CK(hipStreamSynchronize(s));
      std::vector<double> t;
      for (int r = 0; r < 5; ++r) {
        CK(hipEventRecord(e0, s));
        for (int i = 0; i < reps; ++i) one();
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        t.push_back(double(ms) * 1e3 / reps);
      }
      const double us = median(t);
      std::printf("{\"probe\": \"queued 4 MiB pinned read: %s\", \"us_per_block\": %.2f, \"GBps\": %.1f}\n", name, us,
                  double(n) / (us * 1e3));
      std::fflush(stdout);
    };
    const int64_t n16 = int64_t(n / 16);
    for (int grid : {256, 512, 1024, 2048, 4096}) {
      char name[64];
      std::snprintf(name, sizeof(name), "kernel grid %d x 256", grid);
      queued(name, [&] {
        hipLaunchKernelGGL(copy16, dim3(grid), dim3(256), 0, s, reinterpret_cast<const u32x4*>(pinned),
                           reinterpret_cast<u32x4*>(dev), n16);
      });
    }
    queued("DMA hipMemcpyAsync", [&] { CK(hipMemcpyAsync(dev, pinned, n, hipMemcpyHostToDevice, s)); });
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
  }
  CK(hipHostFree(pinned));
  CK(hipFree(dev));
  std::free(host);
  return 0;
}
