// sdma_d2h_probe.cpp -- MEASUREMENT TOOL (not the product): is a device ->
// pinned-host copy faster on an SDMA engine than HIP's own D2H, which HIP
// runs as a blit kernel (`__amd_rocclr_copyBuffer`, profiles/r06_pipe_copy_engines.json)?
// DESIGN.md §11 item 5 left this "not attempted": the pipelines' encode gives
// back 2-4 % with 1-D D2H copies.  Copies here go below HIP, through
// hsa_amd_memory_async_copy_on_engine on an engine the status query reports
// free, and are timed against hipMemcpyAsync on the same buffers:
//   d2h       one 16 MiB (the encode's 4 parity shards) or 4 MiB D2H, alone
//   duplex    24 x (40 MiB H2D by hipMemcpyAsync || 16 MiB D2H: HIP 1-D, HIP
//             2-D, or an SDMA engine), the encode
//             pipeline's copy pattern without the kernel: GiB/s of H2D data
// One JSON line per measurement on stdout.
//
// Build: hipcc -O2 --offload-arch=gfx950 tools/sdma_d2h_probe.cpp -lhsa-runtime64 -o tools/sdma_d2h_probe.bin
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace {

#define CHECK_HIP(x)                                                                    \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                                     \
    }                                                                                   \
  } while (0)
#define CHECK_HSA(x)                                                                    \
  do {                                                                                  \
    hsa_status_t s_ = (x);                                                              \
    if (s_ != HSA_STATUS_SUCCESS) {                                                     \
      std::fprintf(stderr, "%s:%d %s: hsa status 0x%x\n", __FILE__, __LINE__, #x, unsigned(s_)); \
      std::exit(3);                                                                     \
    }                                                                                   \
  } while (0)

struct Agents {
  hsa_agent_t gpu{}, cpu{};
  bool have_gpu = false, have_cpu = false;
};

hsa_status_t pick_agent(hsa_agent_t a, void* data) {
  auto* ag = static_cast<Agents*>(data);
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
  if (t == HSA_DEVICE_TYPE_GPU && !ag->have_gpu) {
    ag->gpu = a;
    ag->have_gpu = true;
  } else if (t == HSA_DEVICE_TYPE_CPU && !ag->have_cpu) {
    ag->cpu = a;
    ag->have_cpu = true;
  }
  return HSA_STATUS_SUCCESS;
}

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

}  // namespace

int main() {
  constexpr size_t kMiB = size_t(1) << 20;
  constexpr size_t kIn = 40 * kMiB, kOut = 16 * kMiB;
  constexpr int kStripes = 24, kReps = 7;
  CHECK_HIP(hipSetDevice(0));
  CHECK_HIP(hipFree(nullptr));  // HIP (and under it HSA) initialised
  CHECK_HSA(hsa_init());        // a reference on the runtime HIP already opened
  Agents ag;
  CHECK_HSA(hsa_iterate_agents(pick_agent, &ag));
  if (!ag.have_gpu || !ag.have_cpu) {
    std::fprintf(stderr, "no GPU / CPU agent\n");
    return 4;
  }
  uint32_t d2h_mask = 0, h2d_mask = 0;
  CHECK_HSA(hsa_amd_memory_copy_engine_status(ag.cpu, ag.gpu, &d2h_mask));
  CHECK_HSA(hsa_amd_memory_copy_engine_status(ag.gpu, ag.cpu, &h2d_mask));
  std::printf("{\"probe\": \"engines\", \"d2h_free_mask\": %u, \"h2d_free_mask\": %u}\n", d2h_mask, h2d_mask);

  uint8_t *d_in = nullptr, *d_out = nullptr, *h_in = nullptr, *h_out = nullptr;
  CHECK_HIP(hipMalloc(&d_in, kIn * 2));  // two slots: H2D alternates, like the ring
  CHECK_HIP(hipMalloc(&d_out, kOut));
  CHECK_HIP(hipHostMalloc(&h_in, kIn, hipHostMallocDefault));
  CHECK_HIP(hipHostMalloc(&h_out, kOut, hipHostMallocDefault));
  std::vector<uint8_t> pattern(kOut);
  for (size_t i = 0; i < kOut; ++i) pattern[i] = uint8_t(i * 131u + 7u);
  CHECK_HIP(hipMemcpy(d_out, pattern.data(), kOut, hipMemcpyHostToDevice));
  std::memset(h_in, 0x5A, kIn);
  hipStream_t s_h2d, s_d2h;
  CHECK_HIP(hipStreamCreateWithFlags(&s_h2d, hipStreamNonBlocking));
  CHECK_HIP(hipStreamCreateWithFlags(&s_d2h, hipStreamNonBlocking));
  hsa_signal_t sig;
  CHECK_HSA(hsa_signal_create(1, 0, nullptr, &sig));

  // engines to try for the D2H: every one the status query reports free
  std::vector<uint32_t> engines;
  for (uint32_t b = 0; b < 16; ++b)
    if (d2h_mask & (1u << b)) engines.push_back(1u << b);

  auto sdma_d2h = [&](uint32_t eng, size_t bytes) {
    hsa_signal_store_relaxed(sig, 1);
    CHECK_HSA(hsa_amd_memory_async_copy_on_engine(h_out, ag.cpu, d_out, ag.gpu, bytes, 0, nullptr, sig,
                                                  hsa_amd_sdma_engine_id_t(eng), true));
  };
  auto sdma_wait = [&] {
    while (hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED) != 0) {
    }
  };
  auto verify = [&](size_t bytes) { return std::memcmp(h_out, pattern.data(), bytes) == 0; };

  for (size_t bytes : {kOut, 4 * kMiB}) {
    // HIP's D2H alone
    std::vector<double> t;
    for (int r = 0; r < kReps + 1; ++r) {
      std::memset(h_out, 0, bytes);
      const double t0 = now_ms();
      CHECK_HIP(hipMemcpyAsync(h_out, d_out, bytes, hipMemcpyDeviceToHost, s_d2h));
      CHECK_HIP(hipStreamSynchronize(s_d2h));
      if (r) t.push_back(now_ms() - t0);
    }
    std::printf("{\"probe\": \"d2h\", \"path\": \"hip\", \"bytes\": %zu, \"median_ms\": %.4f, \"GBps\": %.1f, \"ok\": %s}\n",
                bytes, median(t), bytes / median(t) / 1e6, verify(bytes) ? "true" : "false");
    t.clear();
    for (int r = 0; r < kReps + 1; ++r) {
      std::memset(h_out, 0, bytes);
      const double t0 = now_ms();
      CHECK_HIP(hipMemcpy2DAsync(h_out, bytes / 4, d_out, bytes / 4, bytes / 4, 4, hipMemcpyDeviceToHost, s_d2h));
      CHECK_HIP(hipStreamSynchronize(s_d2h));
      if (r) t.push_back(now_ms() - t0);
    }
    std::printf("{\"probe\": \"d2h\", \"path\": \"hip_2d\", \"bytes\": %zu, \"median_ms\": %.4f, \"GBps\": %.1f, \"ok\": %s}\n",
                bytes, median(t), bytes / median(t) / 1e6, verify(bytes) ? "true" : "false");
    for (uint32_t eng : engines) {
      t.clear();
      for (int r = 0; r < kReps + 1; ++r) {
        std::memset(h_out, 0, bytes);
        const double t0 = now_ms();
        sdma_d2h(eng, bytes);
        sdma_wait();
        if (r) t.push_back(now_ms() - t0);
      }
      std::printf("{\"probe\": \"d2h\", \"path\": \"sdma\", \"engine_mask\": %u, \"bytes\": %zu, \"median_ms\": %.4f, "
                  "\"GBps\": %.1f, \"ok\": %s}\n",
                  eng, bytes, median(t), bytes / median(t) / 1e6, verify(bytes) ? "true" : "false");
    }
  }

  // duplex: the encode pipeline's copies without the kernel
  auto duplex = [&](int eng) {  // eng 0: HIP's 1-D D2H, -1: HIP's 2-D D2H (4 rows of 4 MiB, pitch = width)
    std::vector<double> t;
    for (int r = 0; r < kReps + 1; ++r) {
      const double t0 = now_ms();
      for (int s = 0; s < kStripes; ++s) {
        CHECK_HIP(hipMemcpyAsync(d_in + kIn * size_t(s & 1), h_in, kIn, hipMemcpyHostToDevice, s_h2d));
        if (eng == 0) {
          CHECK_HIP(hipMemcpyAsync(h_out, d_out, kOut, hipMemcpyDeviceToHost, s_d2h));
        } else if (eng < 0) {
          CHECK_HIP(hipMemcpy2DAsync(h_out, kOut / 4, d_out, kOut / 4, kOut / 4, 4, hipMemcpyDeviceToHost, s_d2h));
        } else {
          if (s) sdma_wait();  // one SDMA copy in flight at a time, like the ring's D2H stream
          sdma_d2h(uint32_t(eng), kOut);
        }
      }
      CHECK_HIP(hipStreamSynchronize(s_h2d));
      if (eng <= 0) CHECK_HIP(hipStreamSynchronize(s_d2h));
      else sdma_wait();
      if (r) t.push_back(now_ms() - t0);
    }
    const double ms = median(t);
    std::printf("{\"probe\": \"duplex\", \"d2h_path\": \"%s\", \"engine_mask\": %d, \"stripes\": %d, \"median_ms\": %.3f, "
                "\"h2d_data_GiBps\": %.2f, \"d2h_GBps\": %.1f}\n",
                eng > 0 ? "sdma" : eng < 0 ? "hip_2d" : "hip", eng, kStripes, ms, double(kIn) * kStripes / (ms / 1e3) / double(1 << 30),
                double(kOut) * kStripes / ms / 1e6);
  };
  duplex(0);
  duplex(-1);
  for (uint32_t eng : engines)
    if (eng <= 8) duplex(int(eng));  // engines 4-15 ran 7-12 GB/s alone (profiles/r06_sdma_d2h.jsonl)
  duplex(0);
  duplex(-1);

  CHECK_HSA(hsa_signal_destroy(sig));
  CHECK_HIP(hipHostFree(h_in));
  CHECK_HIP(hipHostFree(h_out));
  CHECK_HIP(hipFree(d_in));
  CHECK_HIP(hipFree(d_out));
  CHECK_HSA(hsa_shut_down());
  std::printf("{\"probe\": \"done\"}\n");
  return 0;
}
