// ecgpu_runtime.hip -- device side of include/ecgpu.h: plans, kernel
// dispatch, staging of host buffers, and the hot-path C ABI.  The ECX
// accumulators (accum.hip), host pipelines (pipeline.hip) and GF(2) packet
// coding (packets.hip) build on the helpers this file exports to them
// through runtime.hpp.
//
// Execution model (MI355X-first, not the reference's byte loops):
//   * every hot-path call is planned on the host into ONE fused
//     rows x nsrc GF(2^8) matrix apply (planner.hpp) and runs as one
//     streaming launch per <= 4 output rows;
//   * buffers are classified per pointer: device memory is used in place,
//     host memory is staged through a per-context HBM slab with
//     hipMemcpyAsync on that context's own stream (ordered after the null stream);
//   * contexts (stream + staging + plan cache) come from a process-wide
//     pool, so concurrent callers (the reference's encode pthreads,
//     client_main.cpp:1074-1164) never share a stream or a lock on the
//     submit path; tables are built once (std::call_once in gf_host).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <list>
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
#include "gf_kernels.hpp"
#include "gf_spec.hpp"
#include "host_sync.hpp"
#include "knobs.hpp"
#include "matrix_host.hpp"
#include "planner.hpp"
#include "runtime.hpp"

using namespace ecgpu;
using namespace ecgpu::rt;
using dev::ApplyArgs;
using dev::u32x4;

ECGPU_RT_BEGIN

// t_err / fail / ecgpu_last_error live in capi_host.cpp (host code, so the
// host-only checks -- buffer contract, knobs -- report through them too)


// ------------------------------------------------------- kernel tables ----
using KernelFn = void (*)(ApplyArgs);

// Production kernels: gf_apply<K, R, UNITS> specialised at compile time
// (gf_spec.hpp, one translation unit per R): one 16-B column per lane,
// 3-bit-slice v_perm multiply, XOR3 via v_bitop3, unit-coefficient
// structure fixed per launch, non-temporal loads; store policy per launch.
// Which compile-time unit structure holds exactly for rows [r0, r0+R).
int unit_variant(const std::vector<uint32_t>& coef, int K, int r0, int R) {
  bool all = true, col0 = true, row0 = true;
  for (int r = 0; r < R; ++r)
    for (int j = 0; j < K; ++j) {
      const bool one = coef[size_t(r0 + r) * K + j] == 1;
      all &= one;
      if (j == 0) col0 &= one;
      if (r == 0) row0 &= one;
    }
  if (all) return 4;
  return (col0 ? 1 : 0) | (row0 ? 2 : 0);
}

KernelFn generic_fn(int R) {
  switch (R) {
    case 1: return &dev::gf_apply_perm_generic<1>;
    case 2: return &dev::gf_apply_perm_generic<2>;
    case 3: return &dev::gf_apply_perm_generic<3>;
    default: return &dev::gf_apply_perm_generic<4>;
  }
}

hipError_t launch(KernelFn fn, dim3 grid, dim3 block, ApplyArgs& a, hipStream_t s, unsigned lds_bytes = 0) {
  void* args[] = {&a};
  return hipLaunchKernel(reinterpret_cast<const void*>(fn), grid, block, args, lds_bytes, s);
}

// Residency cap for the streaming kernels.  Fewer resident workgroups per CU
// means fewer DRAM pages open at once across the chip: with each lane reading
// K shards and writing R, the uncapped kernel (VGPR-limited to 7 blocks/CU)
// keeps ~28k distinct 4 KiB shard chunks in flight.  What matters is the
// number of shard streams per lane, K + R: a sweep over eight encode and
// decode shapes (K + R = 5..16, 64 KiB..16 MiB shards, 3 interleaved rounds,
// profiles/r02_residency_sweep.json) has 4 blocks/CU best or within 0.3 % of
// the best for K + R <= 9 and 3 blocks/CU for K + R >= 10; never capping is
// the worst or near it everywhere (-1.5 % to -7 %).  A launch dense in GF
// multiplies (decode{0,1,2,3}: 40 non-unit coefficients over 14 shards)
// needs the occupancy to hide its VALU work and loses 7 %, so such launches
// stay uncapped (cap_for).  The cap is an unused dynamic LDS allocation of
// LDS_per_CU / blocks (rounded down to 512 B).  A kernel with static LDS of
// its own (the LDS engine's tables) gets that much less and a further 4 KiB
// margin, rounded down to 4 KiB: RS(10,4) at "3 per CU" with 1,280 B of
// tables, dynamic 52,736 B (1.8 KiB spare) ran at 2 per CU's speed (989 us),
// 40,960-49,152 B at 902-905 (tools/encode_lab.hip --lds 2).
// ECGPU_BLOCKS_PER_CU fixes the block count (0 = never cap).
unsigned residency_lds_bytes(int device, int streams, unsigned static_bytes = 0) {
  static std::once_flag once;
  static int per_cu = 0;
  std::call_once(once, [&] {
    if (hipDeviceGetAttribute(&per_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, device) != hipSuccess)
      per_cu = 0;
  });
  const int fixed = knob(Knob::kBlocksPerCu);
  const int blocks = fixed >= 0 ? fixed : (streams <= 9 ? 4 : 3);
  if (blocks <= 0 || per_cu <= 0) return 0;
  const unsigned total = unsigned(per_cu / blocks) & ~511u;
  const unsigned reserve = static_bytes ? static_bytes + 4096u : 0u;
  if (total <= reserve) return 0;
  const unsigned b = (total - reserve) & (static_bytes ? ~4095u : ~511u);
  return b + static_bytes > unsigned(per_cu / (blocks + 1)) ? b : 0u;
}

// Per-launch policy of the production kernel (A/B on MI355X in the bench's
// back-to-back context, DESIGN.md §5, profiles/r01_policy_ab.json):
//   * stores non-temporal (loads always are): bench step +4 %, RS(10,4)
//     encode 0.947 -> 0.889 ms, dense decode +9 %, RS(12,4) +6 %;
//   * residency cap unless the launch is dense in GF multiplies (more than
//     2.5 non-unit coefficients per shard touched): decode{0} +9 %, RS(6,3)
//     +6 %; the 40-multiply decode{0,1,2,3} needs the occupancy (-7 % capped).
// The store policy is the plan's `nt` field (0 plain, 1 nt -- the default;
// ECGPU_NT, ecgpu_plan_set_kernel); the cap knob (ECGPU_CAP: 0 = never,
// 1 = always) overrides the cap rule.
bool cap_for(int K, int R, int mul_terms) {
  const int v = knob(Knob::kCap);
  return v < 0 ? 2 * mul_terms <= 5 * (K + R) : (v != 0);
}

// Per-coefficient tables.  PERM: word p holds c*(e << 2p) in byte e.  LDS:
// 16 low-nibble products then 16 high-nibble products.
// P3 (production, gf_kernels.hpp mul3): T0[e] = c*e and T1[e] = c*(e << 3)
// for e < 8 as dword pairs (low dword = entries 0..3), T2[e] = c*(e << 6).
void build_tables(int c, u32x4* q, uint32_t* p3, uint8_t* nib) {
  const auto& T = gf8().mul[c & 0xFF];
  uint32_t w[4];
  for (int p = 0; p < 4; ++p) {
    w[p] = 0;
    for (int e = 0; e < 4; ++e) w[p] |= uint32_t(T[e << (2 * p)]) << (8 * e);
  }
  *q = u32x4{w[0], w[1], w[2], w[3]};
  for (int i = 0; i < dev::kP3Words; ++i) p3[i] = 0;
  for (int e = 0; e < 8; ++e) {
    p3[e >> 2] |= uint32_t(T[e]) << (8 * (e & 3));
    p3[2 + (e >> 2)] |= uint32_t(T[e << 3]) << (8 * (e & 3));
  }
  for (int e = 0; e < 4; ++e) p3[4] |= uint32_t(T[e << 6]) << (8 * e);
  for (int x = 0; x < 16; ++x) {
    nib[x] = T[x];
    nib[16 + x] = T[x << 4];
  }
}

// Wide-word tables (gf_kernels.hpp, "wide words"): for coefficient c of
// GF(2^(8W)), the v_perm table pairs of every (rotation d, slice p[, lane
// pair h]).  lane_table(o, b, p) byte e = byte o of c * ((e << 2p) << 8b).
void build_wide_tables(uint32_t c, int W, uint32_t* t) {
  const int w = 8 * W;
  auto lane_table = [&](int o, int b, int p) {
    uint32_t v = 0;
    for (int e = 0; e < 4; ++e) {
      const uint32_t x = uint32_t(e) << (2 * p) << (8 * b);
      v |= ((gf_mul_poly(x, c, w) >> (8 * o)) & 0xFFu) << (8 * e);
    }
    return v;
  };
  if (W == 2) {
    for (int d = 0; d < 2; ++d)
      for (int p = 0; p < 4; ++p) {
        const int i = d * 4 + p;
        t[2 * i] = lane_table(1, (1 + d) % 2, p);  // odd lanes (selectors 4..7)
        t[2 * i + 1] = lane_table(0, d % 2, p);    // even lanes (selectors 0..3)
      }
  } else {
    for (int d = 0; d < 4; ++d)
      for (int p = 0; p < 4; ++p)
        for (int h = 0; h < 2; ++h) {
          const int i = (d * 4 + p) * 2 + h, lo = 2 * h, hi = 2 * h + 1;
          t[2 * i] = lane_table(hi, (hi + d) % 4, p);
          t[2 * i + 1] = lane_table(lo, (lo + d) % 4, p);
        }
  }
}

// LDS nibble tables of gf_apply_wide_nib: T_t[v] = c*(v << 4t) at w = 32; at
// w = 16 tables 0..3 serve the low word of a dword and 4..7 the high word
// (entries shifted into bits 16..31).
void build_wide_nib_tables(uint32_t c, int w, uint32_t* t) {
  for (int tt = 0; tt < 8; ++tt)
    for (uint32_t v = 0; v < 16; ++v)
      t[tt * 16 + int(v)] = w == 32  ? gf_mul_poly(v << (4 * tt), c, 32)
                            : tt < 4 ? gf_mul_poly(v << (4 * tt), c, 16)
                                     : gf_mul_poly(v << (4 * (tt - 4)), c, 16) << 16;
}

int wide_words_per_coef(int w) { return w == 16 ? 2 * dev::Wide<2>::kPerms : 2 * dev::Wide<4>::kPerms; }

ECGPU_RT_END

ECGPU_RT_BEGIN


// One non-blocking stream per device for coefficient-table uploads: a plan's
// creation does not wait for its tables (one blocking copy cost ~12 us,
// tools/hip_overheads.cpp); its launches wait on the upload's event instead.
hipStream_t upload_stream(int device) {
  static hostsync::PerDevice<hipStream_t> streams;
  return streams.get(device, [](int dev) {
    DeviceGuard g(dev);
    hipStream_t s = nullptr;
    return hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess ? s : nullptr;
  });
}

// Allocates p->d_tabs and uploads `host` into it without waiting (the plan
// keeps `host` alive until the upload has completed).
int plan_upload_tables(ecgpu_plan* p, std::vector<uint8_t>&& host) {
  DeviceGuard g(p->device);
  ECGPU_HIP(hipMalloc(reinterpret_cast<void**>(&p->d_tabs), host.size()));
  p->host_tabs = std::move(host);
  const hipStream_t s = upload_stream(p->device);
  if (!s) {  // no stream: a blocking copy
    ECGPU_HIP(hipMemcpy(p->d_tabs, p->host_tabs.data(), p->host_tabs.size(), hipMemcpyHostToDevice));
    return ECGPU_OK;
  }
  ECGPU_HIP(hipEventCreateWithFlags(&p->uploaded, hipEventDisableTiming));
  ECGPU_HIP(hipMemcpyAsync(p->d_tabs, p->host_tabs.data(), p->host_tabs.size(), hipMemcpyHostToDevice, s));
  ECGPU_HIP(hipEventRecord(p->uploaded, s));
  p->upload_pending = true;
  return ECGPU_OK;
}

// Waits for the plan's table upload on the host (a no-op once it completed).
int plan_sync_tables(ecgpu_plan* p) {
  if (!p->upload_pending) return ECGPU_OK;
  ECGPU_HIP(hipEventSynchronize(p->uploaded));
  p->upload_pending = false;
  std::vector<uint8_t>().swap(p->host_tabs);
  return ECGPU_OK;
}

// Orders `stream` after the plan's table upload (a no-op once it completed).
// A blocking bind has already waited for it, so a bound plan launches inside
// a stream capture without touching the event; a plan bound on a stream
// (the synchronous calls) may not be captured before its upload completed.
int plan_wait_tables(ecgpu_plan* p, hipStream_t stream) {
  if (!p->upload_pending) return ECGPU_OK;
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &cap) == hipSuccess && cap != hipStreamCaptureStatusNone)
    return fail(ECGPU_ERR, "plan tables still uploading: bind the plan without a stream before capturing it");
  (void)hipGetLastError();
  const hipError_t q = hipEventQuery(p->uploaded);
  if (q == hipSuccess) {
    p->upload_pending = false;
    std::vector<uint8_t>().swap(p->host_tabs);
    return ECGPU_OK;
  }
  if (q != hipErrorNotReady) return fail(ECGPU_ERR_HIP, std::string("table upload: ") + hipGetErrorString(q));
  (void)hipGetLastError();  // not ready is not an error
  ECGPU_HIP(hipStreamWaitEvent(stream, p->uploaded, 0));
  return ECGPU_OK;
}

void plan_free(ecgpu_plan* p) {
  if (!p) return;
  DeviceGuard g(p->device);
  if (p->uploaded) {
    (void)hipEventSynchronize(p->uploaded);  // the table upload may still read host_tabs
    (void)hipEventDestroy(p->uploaded);
  }
  if (p->d_tabs) (void)hipFree(p->d_tabs);
  if (p->d_ptrs) (void)hipFree(p->d_ptrs);
  delete p;
}

int plan_init(ecgpu_plan* p, int rows, int nsrc, const int* coefs, int device, int w) {
  p->device = device;
  p->rows = rows;
  p->nsrc = nsrc;
  p->w = w;
  p->kind = knob(Knob::kKernel);
  p->nt = std::min(kStorePolicies - 1, std::max(0, knob(Knob::kNt)));
  const size_t n = size_t(rows) * nsrc;
  p->coef.resize(n);
  if (w != 8) {
    const uint32_t mask = w == 32 ? 0xFFFFFFFFu : (1u << w) - 1u;
    const int nw = wide_words_per_coef(w);
    std::vector<uint32_t> t(n * size_t(nw));
    std::vector<uint8_t> cls(n);
    std::vector<uint32_t> nib(n * size_t(dev::kNibWords));
    for (size_t i = 0; i < n; ++i) {
      p->coef[i] = uint32_t(coefs[i]) & mask;
      cls[i] = p->coef[i] == 0 ? 2 : p->coef[i] == 1 ? 1 : 0;
      build_wide_tables(p->coef[i], w / 8, &t[i * size_t(nw)]);
      build_wide_nib_tables(p->coef[i], w, &nib[i * size_t(dev::kNibWords)]);
    }
    // [wide tables | nibble tables | classes] in one allocation, one upload
    const size_t tb = t.size() * sizeof(uint32_t), nb = nib.size() * sizeof(uint32_t);
    std::vector<uint8_t> host(tb + nb + n);
    std::memcpy(host.data(), t.data(), tb);
    std::memcpy(host.data() + tb, nib.data(), nb);
    std::memcpy(host.data() + tb + nb, cls.data(), n);
    if (int rc = plan_upload_tables(p, std::move(host))) return rc;
    p->d_w = reinterpret_cast<uint32_t*>(p->d_tabs);
    p->d_wnib = reinterpret_cast<uint32_t*>(p->d_tabs + tb);
    p->d_wcls = p->d_tabs + tb + nb;
    return ECGPU_OK;
  }
  for (size_t i = 0; i < n; ++i) p->coef[i] = uint32_t(coefs[i]) & 0xFFu;
  std::vector<u32x4> q(n);
  std::vector<uint32_t> p3(n * dev::kP3Words);
  std::vector<uint8_t> nib(n * 32);
  for (size_t i = 0; i < n; ++i) build_tables(coefs[i], &q[i], &p3[i * dev::kP3Words], &nib[i * 32]);
  // [2-bit tables | 3-bit tables | nibble tables] in one allocation, ONE
  // asynchronous upload (plan_upload_tables; three blocking copies cost ~12 us
  // each, tools/hip_overheads.cpp)
  const size_t qb = n * sizeof(u32x4), pb = p3.size() * sizeof(uint32_t), nb = n * 32;
  std::vector<uint8_t> host(qb + pb + nb);
  std::memcpy(host.data(), q.data(), qb);
  std::memcpy(host.data() + qb, p3.data(), pb);
  std::memcpy(host.data() + qb + pb, nib.data(), nb);
  if (int rc = plan_upload_tables(p, std::move(host))) return rc;
  p->d_q = reinterpret_cast<u32x4*>(p->d_tabs);
  p->d_p3 = reinterpret_cast<uint32_t*>(p->d_tabs + qb);
  p->d_nib = p->d_tabs + qb + pb;
  return ECGPU_OK;
}

// With a stream the pointer tables are uploaded asynchronously on it; unless
// `keep_alive` (the caller keeps src/dst alive until it synchronises the
// stream, as execute() does) the call waits for the upload.
int plan_bind(ecgpu_plan* p, int stripes, const uint8_t* const* src, uint8_t* const* dst, int64_t size,
              hipStream_t stream, bool keep_alive) {
  const size_t ns = size_t(stripes) * p->nsrc, nd = size_t(stripes) * p->rows;
  DeviceGuard g(p->device);
  // a blocking bind settles the table upload too (it overlapped the table
  // build-up to here); a bind on a stream leaves it to the launch
  if (!stream)
    if (int rc = plan_sync_tables(p)) return rc;
  if (ns + nd > p->cap_ptrs) {
    if (p->d_ptrs) ECGPU_HIP(hipFree(p->d_ptrs));
    p->d_ptrs = nullptr;
    p->cap_ptrs = 0;
    ECGPU_HIP(hipMalloc(reinterpret_cast<void**>(&p->d_ptrs), (ns + nd) * sizeof(void*)));
    p->cap_ptrs = ns + nd;
  }
  p->d_src = static_cast<const uint8_t**>(static_cast<void*>(p->d_ptrs));
  p->d_dst = static_cast<uint8_t**>(static_cast<void*>(p->d_ptrs + ns));
  bool aligned = true;
  for (size_t i = 0; i < ns; ++i) aligned &= (reinterpret_cast<uintptr_t>(src[i]) & 15u) == 0;
  for (size_t i = 0; i < nd; ++i) aligned &= (reinterpret_cast<uintptr_t>(dst[i]) & 15u) == 0;
  if (stream && keep_alive) {
    // the caller's arrays outlive the stream sync: no wait here
    ECGPU_HIP(hipMemcpyAsync(p->d_src, src, ns * sizeof(void*), hipMemcpyHostToDevice, stream));
    ECGPU_HIP(hipMemcpyAsync(p->d_dst, dst, nd * sizeof(void*), hipMemcpyHostToDevice, stream));
  } else {
    // one upload of [sources | destinations]
    std::vector<const void*> host(ns + nd);
    std::memcpy(host.data(), src, ns * sizeof(void*));
    std::memcpy(host.data() + ns, dst, nd * sizeof(void*));
    if (stream) {
      ECGPU_HIP(hipMemcpyAsync(p->d_ptrs, host.data(), (ns + nd) * sizeof(void*), hipMemcpyHostToDevice, stream));
      ECGPU_HIP(hipStreamSynchronize(stream));  // the host table dies on return
    } else {
      ECGPU_HIP(hipMemcpy(p->d_ptrs, host.data(), (ns + nd) * sizeof(void*), hipMemcpyHostToDevice));
    }
  }
  p->stripes = stripes;
  p->size = size;
  p->aligned = aligned;
  return ECGPU_OK;
}

// CU count (the launch device; the pool is homogeneous).
int multiprocessors(int device) {
  static std::once_flag once;
  static int n = 0;
  std::call_once(once, [&] {
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || n <= 0) n = 256;
  });
  return n;
}

// Resident workgroups per CU of a kernel at kBlock threads and `lds` bytes
// of dynamic LDS (cached; the launch shapes are few).
int resident_blocks(KernelFn fn, unsigned lds) {
  static std::mutex mu;
  static std::vector<std::pair<std::pair<const void*, unsigned>, int>> cache;
  std::lock_guard<std::mutex> lk(mu);
  const auto key = std::make_pair(reinterpret_cast<const void*>(fn), lds);
  for (const auto& e : cache)
    if (e.first == key) return e.second;
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void*>(fn), dev::kBlock, lds) !=
          hipSuccess ||
      n <= 0)
    n = 4;
  cache.emplace_back(key, n);
  return n;
}

// w = 16 / 32: 16-B column kernel over the aligned part, word kernel for the
// rest; size must be a whole number of words (checked by the callers).  The
// column kernel is gf_apply_wide_nib (LDS nibble tables) when a launch's
// tables fit in kNibMaxLds, else gf_apply_wide (v_perm); ECGPU_WIDE=1 forces
// v_perm (A/B, tools/bench_surface.py).
int plan_launch_wide(ecgpu_plan* p, hipStream_t stream) {
  const int K = p->nsrc, W = p->w / 8, nw = wide_words_per_coef(p->w);
  const int64_t nvec = p->aligned ? p->size / 16 : 0;
  const int64_t byte0 = nvec * 16;
  const dim3 block(dev::kBlock);
  constexpr int kMaxGridY = 65535;
  const bool force_perm = knob(Knob::kWidePerm) == 1;
  for (int r0 = 0; r0 < p->rows; r0 += dev::kMaxRows) {
    const int R = std::min(dev::kMaxRows, p->rows - r0);
    // w = 16 packs two rows per LDS dword (gf_apply_wide_nib16, half the LDS bytes)
    const bool pack16 = W == 2 && knob(Knob::kNib16) != 0;
    // the unit structure (gf_apply_wide_nib<R, 1>, gf_apply_wide_nib16<R, 1>):
    // the launch's row 0 and column 0 all ones, as in every Vandermonde encode
    bool unit_rc = R >= 2 && knob(pack16 ? Knob::kWide16Units : Knob::kWideUnits) != 0;
    for (int j = 0; j < K && unit_rc; ++j) unit_rc = p->coef[size_t(r0) * K + j] == 1u;
    for (int r = 0; r < R && unit_rc; ++r) unit_rc = p->coef[size_t(r0 + r) * K] == 1u;
    const unsigned nib_lds =
        pack16 ? unsigned(K - (unit_rc ? 1 : 0)) * unsigned(dev::nib16_source_bytes(R - (unit_rc ? 1 : 0)))
               : unsigned(dev::nib_lds_bytes(K, R, unit_rc ? 1 : 0));
    const bool nib = !force_perm && nib_lds <= unsigned(dev::kNibMaxLds);
    KernelFn vec_fn = nullptr, word_fn = W == 2 ? &dev::gf_apply_wide_words<2> : &dev::gf_apply_wide_words<4>;
    if (nib && pack16 && unit_rc) {
      switch (R) {
        case 2: vec_fn = &dev::gf_apply_wide_nib16<2, 1>; break;
        case 3: vec_fn = &dev::gf_apply_wide_nib16<3, 1>; break;
        default: vec_fn = &dev::gf_apply_wide_nib16<4, 1>; break;
      }
    } else if (nib && pack16) {
      switch (R) {
        case 1: vec_fn = &dev::gf_apply_wide_nib16<1>; break;
        case 2: vec_fn = &dev::gf_apply_wide_nib16<2>; break;
        case 3: vec_fn = &dev::gf_apply_wide_nib16<3>; break;
        default: vec_fn = &dev::gf_apply_wide_nib16<4>; break;
      }
    } else if (nib && unit_rc) {
      switch (R) {
        case 2: vec_fn = &dev::gf_apply_wide_nib<2, 1>; break;
        case 3: vec_fn = &dev::gf_apply_wide_nib<3, 1>; break;
        default: vec_fn = &dev::gf_apply_wide_nib<4, 1>; break;
      }
    } else if (nib) {
      switch (R) {
        case 1: vec_fn = &dev::gf_apply_wide_nib<1>; break;
        case 2: vec_fn = &dev::gf_apply_wide_nib<2>; break;
        case 3: vec_fn = &dev::gf_apply_wide_nib<3>; break;
        default: vec_fn = &dev::gf_apply_wide_nib<4>; break;
      }
    } else {
      switch (R) {
        case 1: vec_fn = W == 2 ? &dev::gf_apply_wide<2, 1> : &dev::gf_apply_wide<4, 1>; break;
        case 2: vec_fn = W == 2 ? &dev::gf_apply_wide<2, 2> : &dev::gf_apply_wide<4, 2>; break;
        case 3: vec_fn = W == 2 ? &dev::gf_apply_wide<2, 3> : &dev::gf_apply_wide<4, 3>; break;
        default: vec_fn = W == 2 ? &dev::gf_apply_wide<2, 4> : &dev::gf_apply_wide<4, 4>; break;
      }
    }
    // The pipelined form of the same kernels (gf_apply_wide_pipe: compile-time
    // K, the next chunk's loads in flight during this chunk's lookups) for
    // launches of whole 256-column blocks, where it measured faster: the
    // w = 32 unit form with K = 7..10 sources (RS(K,4) 64 MiB, in one process:
    // K = 7 148 -> 139 us, 8 162 -> 149, 10 197 -> 191; K = 5, 11 equal or
    // slower, and so were the general w = 32 and the w = 16 forms outside
    // K = 10 -- profiles/r03_wide_lab.jsonl, "r03 pipe K sweep") and, since
    // round 4, K = 12 in six chunks (227.6 -> 216.8 us,
    // profiles/r04_wide_lab_k12.jsonl; K = 11 stays level, 210.9 vs 211.0).
    // ECGPU_WIDE_PIPE: 1 that rule (default), 0 never, 2 every whole-block
    // launch of every mode (tests, A/B).
    const int pipe = knob(Knob::kWidePipe);
    // (the pipelined w = 16 form has no unit structure: it packs every row)
    const bool pipe_shape = pipe == 2 || (pipe == 1 && !pack16 && unit_rc && ((K >= 7 && K <= 10) || K == 12));
    bool piped = false;
    if (nib && nvec > 0 && nvec % dev::kBlock == 0 && pipe_shape)
      if (KernelFn f = wide_pipe_kernel(K, R, pack16 ? dev::kPipeW16 : unit_rc ? dev::kPipeW32Unit : dev::kPipeW32)) {
        vec_fn = f;
        piped = true;
      }
    const unsigned launch_lds =
        piped && pack16 && unit_rc ? unsigned(K) * unsigned(dev::nib16_source_bytes(R)) : nib_lds;
    for (int s0 = 0; s0 < p->stripes; s0 += kMaxGridY) {
      const int ns = std::min(kMaxGridY, p->stripes - s0);
      ApplyArgs a{};
      a.wtab = nib ? p->d_wnib + size_t(r0) * K * dev::kNibWords : p->d_w + size_t(r0) * K * nw;
      a.wcls = p->d_wcls + size_t(r0) * K;
      a.src = p->d_src + size_t(s0) * K;
      a.dst = p->d_dst + size_t(s0) * p->rows;
      a.nvec = nvec;
      a.size = p->size;
      a.byte0 = byte0;
      a.src_stride = K;
      a.dst_stride = p->rows;
      a.row0 = r0;
      a.K = K;
      a.R = R;
      a.nt = p->nt;
      if (nvec > 0) {
        const int64_t nblk = (nvec + dev::kBlock - 1) / dev::kBlock;
        if (nib) {
          // exactly one resident round of workgroups (occupancy x CUs), each
          // looping over column blocks: a second, partial round would run
          // on part of the chip
          // The w = 16 packed kernel (LDS at half the w = 32 cycles, HBM-bound)
          // runs fewer workgroups per CU than fit, like the w = 8 residency
          // cap: 3 per CU beat the 6 the occupancy allows for RS(10,4) 64 MiB
          // (171.5 vs 181.6 us), RS(5,4) 64 MiB (107.3 vs 116.0) and RS(12,4)
          // 16 MiB (55.1 vs 56.3; tools/wide_lab.hip grid sweep,
          // profiles/r03_wide_lab.jsonl); the LDS-bound w = 32 kernel wants
          // every wave it can get (3 per CU: 242 vs 192 us).
          // ECGPU_WIDE16_BPCU overrides (0: the occupancy).
          int bpcu = resident_blocks(vec_fn, launch_lds);
          if (pack16) {
            const int cap16 = knob(Knob::kWide16Bpcu);
            if (cap16 > 0) bpcu = std::min(bpcu, cap16);
          }
          const int64_t per_stripe = std::max<int64_t>(1, int64_t(multiprocessors(p->device)) * bpcu / ns);
          const dim3 grid(unsigned(std::min(nblk, per_stripe)), unsigned(ns));
          ECGPU_HIP(launch(vec_fn, grid, block, a, stream, launch_lds));
        } else {
          ECGPU_HIP(launch(vec_fn, dim3(unsigned(nblk), unsigned(ns)), block, a, stream));
        }
      }
      const int64_t words = (p->size - byte0) / W;
      if (words > 0) {
        // the word kernel reads the v_perm tables
        a.wtab = p->d_w + size_t(r0) * K * nw;
        const dim3 grid(unsigned((words + dev::kBlock - 1) / dev::kBlock), unsigned(ns));
        ECGPU_HIP(launch(word_fn, grid, block, a, stream));
      }
    }
  }
  return ECGPU_OK;
}

int plan_launch(ecgpu_plan* p, hipStream_t stream) {
  if (p->stripes <= 0 || p->size <= 0 || p->rows <= 0) return ECGPU_OK;
  DeviceGuard g(p->device);
  if (int rc = plan_wait_tables(p, stream)) return rc;
  if (p->w != 8) return plan_launch_wide(p, stream);
  const int K = p->nsrc;
  const int64_t nvec = p->aligned ? p->size / 16 : 0;
  const int64_t byte0 = nvec * 16;
  const dim3 block(dev::kBlock);
  constexpr int kMaxGridY = 65535;
  for (int r0 = 0; r0 < p->rows; r0 += dev::kMaxRows) {
    const int R = std::min(dev::kMaxRows, p->rows - r0);
    const bool spec = K <= dev::kMaxSpecK;
    int mul_terms = 0;  // coefficients that are neither 0 nor 1
    for (int r = 0; r < R; ++r)
      for (int j = 0; j < K; ++j) mul_terms += p->coef[size_t(r0 + r) * K + j] > 1u;
    // The v_perm engine unless ECGPU_KERNEL / ecgpu_plan_set_kernel asks for the
    // LDS nibble-table engine.  (Dense launches on the LDS engine were tried:
    // an in-process interleaved A/B has v_perm 2.5 % faster on C4 decode
    // {0,1,2,3} and even on RS(12,4) {0,1,2,3}, profiles/r02_engine_ab_inprocess.json.)
    const bool use_lds = p->kind == ECGPU_KERNEL_LDS;
    KernelFn vec_fn = spec ? spec_kernel(use_lds, K, R, unit_variant(p->coef, K, r0, R), p->nt) : generic_fn(R);
    const int vec = 1;
    // Both engines follow the cap rule; the LDS engine's allocation leaves room
    // for its K * 128 B of tables (tools/encode_lab.hip --lds: RS(10,4) encode
    // 1008 us uncapped, 902 at 3 per CU, v_perm 890).
    const bool cap = cap_for(K, R, mul_terms);
    const unsigned static_lds = use_lds && spec ? unsigned(K) * 32u * 4u : 0u;
    uint64_t unit = 0, zero = 0;
    if (spec)
      for (int r = 0; r < R; ++r)
        for (int j = 0; j < K; ++j) {
          const uint32_t c = p->coef[size_t(r0 + r) * K + j];
          if (c == 1) unit |= uint64_t(1) << (r * K + j);
          if (c == 0) zero |= uint64_t(1) << (r * K + j);
        }
    for (int s0 = 0; s0 < p->stripes; s0 += kMaxGridY) {
      const int ns = std::min(kMaxGridY, p->stripes - s0);
      ApplyArgs a{};
      a.qtab = p->d_q + size_t(r0) * K;
      a.ptab = p->d_p3 + size_t(r0) * K * dev::kP3Words;
      a.ntab = p->d_nib + size_t(r0) * K * 32;
      a.src = p->d_src + size_t(s0) * K;
      a.dst = p->d_dst + size_t(s0) * p->rows;
      a.nvec = nvec;
      a.size = p->size;
      a.byte0 = byte0;
      a.src_stride = K;
      a.dst_stride = p->rows;
      a.row0 = r0;
      a.K = K;
      a.R = R;
      a.nt = p->nt;
      a.unit_mask = unit;
      a.zero_mask = zero;
      if (nvec > 0) {
        const int64_t per_block = int64_t(dev::kBlock) * vec;
        const dim3 grid(unsigned((nvec + per_block - 1) / per_block), unsigned(ns));
        const unsigned lds = cap ? residency_lds_bytes(p->device, K + R, static_lds) : 0u;
        ECGPU_HIP(launch(vec_fn, grid, block, a, stream, lds));
      }
      if (byte0 < p->size) {
        const dim3 grid(unsigned((p->size - byte0 + dev::kBlock - 1) / dev::kBlock), unsigned(ns));
        ECGPU_HIP(launch(&dev::gf_apply_bytes, grid, block, a, stream));
      }
    }
  }
  return ECGPU_OK;
}

// ------------------------------------------------------ context pool ----

hostsync::IdlePool<Ctx> g_pool;  // idle contexts (process lifetime)

int current_device() {
  const int forced = knob(Knob::kDevice);
  if (forced >= 0) return forced;
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess) d = 0;
  return d;
}

Ctx* acquire_ctx(int device, int* rc) {
  if (Ctx* c = g_pool.acquire(device)) {
    *rc = ECGPU_OK;
    return c;
  }
  auto* c = new Ctx();
  c->device = device;
  DeviceGuard g(device);
  // A blocking stream: a synchronous call on device buffers is ordered after
  // work the caller queued on the null stream (PyTorch's default stream,
  // e.g. the fill of a freshly allocated output), and that stream's later
  // work after the call.  Calls from different threads still run on
  // different contexts, unordered against each other.
  hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamDefault);
  if (e != hipSuccess) {
    *rc = fail(ECGPU_ERR_HIP, std::string("hipStreamCreateWithFlags: ") + hipGetErrorString(e));
    delete c;
    return nullptr;
  }
  *rc = ECGPU_OK;
  return c;
}

void release_ctx(Ctx* c) { g_pool.release(c->device, c); }


int ctx_plan(Ctx* c, int rows, int nsrc, const std::vector<uint32_t>& coef, int w, ecgpu_plan** out) {
  PlanKey key{rows, nsrc, w, coef};
  for (auto it = c->plans.begin(); it != c->plans.end(); ++it)
    if (it->first == key) {
      c->plans.splice(c->plans.begin(), c->plans, it);
      *out = it->second;
      return ECGPU_OK;
    }
  auto* p = new ecgpu_plan();
  std::vector<int> ci(coef.begin(), coef.end());
  int rc = plan_init(p, rows, nsrc, ci.data(), c->device, w);
  if (rc != ECGPU_OK) {
    plan_free(p);
    return rc;
  }
  c->plans.emplace_front(std::move(key), p);
  if (c->plans.size() > 64) {
    plan_free(c->plans.back().second);
    c->plans.pop_back();
  }
  *out = p;
  return ECGPU_OK;
}

// How a synchronous call moves host (pageable or pinned) buffers, by the
// bytes it stages (measured on MI355X, tools/hip_overheads.cpp,
// tools/zero_copy_probe.cpp): every DMA costs ~10 us of setup
// and a launch + sync ~11 us, so
//   * up to zc_max() staged bytes: NO DMA.  The calling thread copies the
//     host side into coherent pinned memory and the kernel reads its sources
//     and writes its outputs there directly over PCIe (zero-copy; reads and
//     writes travel opposite directions of the link): one launch per call.
//   * up to bounce_max(): the host side is copied by the CPU through a pinned
//     mirror of the staging slab and crosses PCIe as one H2D DMA plus one D2H
//     DMA per run of adjacent outputs.
//   * above: HIP's own pageable copies (a 6 MiB pageable DMA runs at the
//     pinned rate, 120 us), one 2-D copy per run of evenly spaced shards
//     (copy_shards).  Staging large calls through a pinned ring filled by
//     this thread instead lost 10-40 % (a single thread copies cold memory at
//     ~35 GB/s, below the link; profiles/r02_dropin_ab.txt).
size_t bounce_max() { return size_t(std::max(0, knob(Knob::kBounceKib))) << 10; }  // 2 MiB by default

size_t zc_max() { return size_t(std::max(0, knob(Knob::kZcKib))) << 10; }

// A call above bounce_max() whose staged outputs total at most zc_out_max()
// bytes, each at most zc_out_shard_max(), has the kernel write its outputs
// into coherent pinned memory (see execute).  A pageable D2H costs 67 us per
// 1 MiB shard but runs at link rate from 4 MiB (86 us): drop-in C2 encode 333
// -> 296 us, C3 decode{0} (one 4 MiB output) 871 -> 1005 us if it took this
// path (profiles/r02_zc_out_ab.txt).
size_t zc_out_max() { return size_t(std::max(0, knob(Knob::kZcOutKib))) << 10; }

size_t zc_out_shard_max() { return size_t(std::max(0, knob(Knob::kZcOutShardKib))) << 10; }

bool zero_copy_pinned() { return knob(Knob::kZcPinned) != 0; }

bool inline_enabled() { return knob(Knob::kInline) != 0; }

int ensure_bounce(Ctx* c, size_t bytes) {
  if (bytes <= c->bounce_cap) return ECGPU_OK;
  DeviceGuard g(c->device);
  if (c->bounce) ECGPU_HIP(hipHostFree(c->bounce));
  c->bounce = nullptr;
  c->bounce_cap = 0;
  ECGPU_HIP(hipHostMalloc(reinterpret_cast<void**>(&c->bounce), bytes, hipHostMallocDefault));
  c->bounce_cap = bytes;
  return ECGPU_OK;
}

// Coherent (fine-grained) pinned memory: the GPU does not cache it, so CPU
// writes before a launch and GPU writes before its completion are visible to
// the other side without cache maintenance.  Grows geometrically.
int ensure_zc(Ctx* c, size_t bytes) {
  if (bytes <= c->zc_cap) return ECGPU_OK;
  DeviceGuard g(c->device);
  if (c->zc) ECGPU_HIP(hipHostFree(c->zc));
  c->zc = nullptr;
  c->zc_cap = 0;
  const size_t want = std::max(bytes, size_t(256) << 10);
  ECGPU_HIP(hipHostMalloc(reinterpret_cast<void**>(&c->zc), want, hipHostMallocMapped | hipHostMallocCoherent));
  c->zc_cap = want;
  return ECGPU_OK;
}

int ensure_stage(Ctx* c, size_t bytes) {
  if (bytes <= c->stage_cap) return ECGPU_OK;
  DeviceGuard g(c->device);
  if (c->stage) ECGPU_HIP(hipFree(c->stage));
  c->stage = nullptr;
  c->stage_cap = 0;
  ECGPU_HIP(hipMalloc(reinterpret_cast<void**>(&c->stage), bytes));
  c->stage_cap = bytes;
  return ECGPU_OK;
}

// Is p device memory of `device` (usable in place)?  Host memory (pageable or
// pinned) is staged; device memory of another GPU is rejected.
int classify(const void* p, int device, bool* on_device) {
  hipPointerAttribute_t attr;
  hipError_t e = hipPointerGetAttributes(&attr, p);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    *on_device = false;
    return ECGPU_OK;
  }
  if (attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged) {
    if (attr.device != device)
      return fail(ECGPU_ERR_ARG, "buffer lives on device " + std::to_string(attr.device) + ", call runs on " +
                                     std::to_string(device));
    *on_device = true;
    return ECGPU_OK;
  }
  *on_device = false;
  return ECGPU_OK;
}

// Host memory the GPU addresses in place -- hipHostMalloc'd, or registered
// with hipHostRegister -- when [p, p + bytes) lies inside ONE such
// allocation (HIP's range attributes; a range that leaves it would fault).
// *dev = the device address of p.
bool host_mapped(const void* p, size_t bytes, void** dev) {
  hipPointerAttribute_t attr;
  if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  if (attr.type != hipMemoryTypeHost) return false;
  void* start = nullptr;
  size_t range = 0;
  if (hipPointerGetAttribute(&start, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, hipDeviceptr_t(p)) != hipSuccess ||
      hipPointerGetAttribute(&range, HIP_POINTER_ATTRIBUTE_RANGE_SIZE, hipDeviceptr_t(p)) != hipSuccess ||
      hipHostGetDevicePointer(dev, const_cast<void*>(p), 0) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  const char* c = static_cast<const char*>(p);
  const char* s0 = static_cast<const char*>(start);
  return c >= s0 && bytes <= range && size_t(c - s0) <= range - bytes;
}

bool is_pinned(const void* p) {
  hipPointerAttribute_t attr;
  if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return attr.type == hipMemoryTypeHost;
}

// ------------------------------------------------------ stats counters ----
std::mutex g_stats_mu;
double g_stats[3] = {0, 0, 0};  // xor, gf, memcpy -- jerasure.cpp:1145-1147 order

void add_stats(const FusedOp& op) {
  std::lock_guard<std::mutex> lk(g_stats_mu);
  g_stats[0] += op.xor_bytes;
  g_stats[1] += op.gf_bytes;
  g_stats[2] += op.memcpy_bytes;
}

// Moves n shards of `bytes` between host pointers hp[i] and device shards
// d0 + i * dstride.  Every run of >= 2 evenly spaced host shards (a stripe
// laid out in one host slab, as the reference client's stripe buffer is,
// client_main.cpp:1619-1647) goes as ONE 2-D copy, the rest one copy per
// shard.  ECGPU_PIPE_2D=0 always copies per shard.  Used by the pipelines and
// by synchronous calls on large host buffers.
int copy_shards(bool h2d, uint8_t* d0, size_t dstride, const std::vector<char*>& hp, size_t bytes, hipStream_t s) {
  const bool two_d = knob(Knob::kPipe2d) != 0;
  const size_t n = hp.size();
  for (size_t a = 0; a < n;) {
    size_t b = a + 1;  // [a, b): maximal run with one pitch >= bytes
    const ptrdiff_t pitch = b < n ? hp[b] - hp[a] : 0;
    // pageable memory only when the run is contiguous (pitch == bytes): a
    // pageable 2-D copy with gaps between rows ran 15x slower than per-shard
    // copies (RS(6,3) 1 MiB, shards malloc'd one by one, 16 B apart)
    bool ok = two_d && pitch > 0 && size_t(pitch) >= bytes;
    if (ok && size_t(pitch) != bytes) ok = is_pinned(hp[a]);  // pinned or registered
    if (ok)
      while (b < n && hp[b] - hp[b - 1] == pitch) ++b;
    // a gapped run must be pinned at both ends (one registration or
    // allocation spans it; HIP rejects a span across separately registered
    // buffers at enqueue, which falls back below)
    if (b - a >= 2 && size_t(pitch) != bytes && !is_pinned(hp[b - 1] + bytes - 1)) b = a + 1;
    uint8_t* d = d0 + a * dstride;
    if (b - a >= 2) {
      const hipError_t e =
          h2d ? hipMemcpy2DAsync(d, dstride, hp[a], size_t(pitch), bytes, b - a, hipMemcpyHostToDevice, s)
              : hipMemcpy2DAsync(hp[a], size_t(pitch), d, dstride, bytes, b - a, hipMemcpyDeviceToHost, s);
      if (e == hipSuccess) {
        a = b;
        continue;
      }
      // not enqueued: fall back to one copy per shard (the error is not sticky)
      (void)hipGetLastError();
    }
    for (size_t i = a; i < b; ++i) {
      if (h2d)
        ECGPU_HIP(hipMemcpyAsync(d0 + i * dstride, hp[i], bytes, hipMemcpyDefault, s));
      else
        ECGPU_HIP(hipMemcpyAsync(hp[i], d0 + i * dstride, bytes, hipMemcpyDefault, s));
    }
    a = b;
  }
  return ECGPU_OK;
}

// P3 tables of one coefficient (see build_tables).
void build_p3(uint32_t c, uint32_t* p3) {
  const auto& T = gf8().mul[c & 0xFF];
  for (int i = 0; i < dev::kP3Words; ++i) p3[i] = 0;
  for (int e = 0; e < 8; ++e) {
    p3[e >> 2] |= uint32_t(T[e]) << (8 * (e & 3));
    p3[2 + (e >> 2)] |= uint32_t(T[e << 3]) << (8 * (e & 3));
  }
  for (int e = 0; e < 4; ++e) p3[4] |= uint32_t(T[e << 6]) << (8 * e);
}

// Can a fused op run as gf_apply_inl launches (everything in the kernel
// arguments, no table or pointer upload)?  w = 8, 1..16 sources, the
// production engine, and no output that is also a source when the rows need
// more than one launch.
bool inline_ok(const FusedOp& op, int64_t size) {
  const int rows = int(op.dsts.size()), nsrc = int(op.srcs.size());
  // The inline kernels with 15-16 sources and a full 4-row launch hold more
  // coefficient tables than the SGPR file and spill them to VGPR lanes (the
  // plan kernel loads them as it goes): a dense RS(16,4) 64 MiB encode ran
  // 574 us inline against 229 us as a plan launch (tools/probe_inline.py,
  // profiles/r03_inline_vs_plan.csv); K = 14 and below are equal.  Large
  // such calls take the plan; small ones stay inline, where the table upload
  // a plan needs would cost more than the spills.
  const bool spills = nsrc >= 15 && rows >= dev::kMaxRows && size > (int64_t(1) << 20);
  return inline_enabled() && op.w == 8 && nsrc >= 1 && nsrc <= dev::kMaxSpecK && rows >= 1 && !spills &&
         knob(Knob::kKernel) == ECGPU_KERNEL_PERM && !(op.dst_is_src && rows > dev::kMaxRows);
}

// Workgroups of an inline launch that reads or writes host memory in place
// (zero-copy): queued 4 MiB pinned reads ran at 52.5 GB/s with 256
// grid-stride workgroups and 41 GB/s with 1024+ (too many PCIe requests in
// flight; tools/zero_copy_probe.cpp); through the drop-in, 32-64 workgroups
// were best (C3 pinned encode 0.83 ms vs 0.93-0.96 uncapped,
// profiles/r02_zc_grid_sweep.txt).  0 = uncapped.
int64_t zc_grid() { return knob(Knob::kZcGrid); }

// One gf_apply_inl launch per <= 4 output rows over `size` bytes.  host_io:
// some pointer is host memory the kernel reads / writes over PCIe (grid
// capped at zc_grid()).
int launch_inline(const FusedOp& op, const std::vector<const uint8_t*>& sp, const std::vector<uint8_t*>& dp,
                  int64_t size, hipStream_t s, bool host_io) {
  const int K = int(sp.size()), rows = int(dp.size());
  bool aligned = true;
  for (auto* p : sp) aligned &= (reinterpret_cast<uintptr_t>(p) & 15u) == 0;
  for (auto* p : dp) aligned &= (reinterpret_cast<uintptr_t>(p) & 15u) == 0;
  const int64_t nvec = aligned ? size / 16 : 0, byte0 = nvec * 16;
  int64_t nbv = (nvec + dev::kBlock - 1) / dev::kBlock;
  if (host_io && zc_grid() > 0) nbv = std::min(nbv, zc_grid());
  const int64_t nbb = (size - byte0 + dev::kBlock - 1) / dev::kBlock;
  for (int r0 = 0; r0 < rows; r0 += dev::kMaxRows) {
    const int R = std::min(dev::kMaxRows, rows - r0);
    // the grid-stride form only where the grid is capped (host memory in place)
    const bool zc = nbv * dev::kBlock < nvec;
    const InlineKernelFn fn = inline_kernel(K, R, unit_variant(op.coef, K, r0, R), zc);
    if (!fn) return fail(ECGPU_ERR, "no inline kernel for K = " + std::to_string(K));
    dev::InlineArgs a{};
    for (int j = 0; j < K; ++j) a.src[j] = sp[size_t(j)];
    for (int r = 0; r < R; ++r) a.dst[r] = dp[size_t(r0 + r)];
    a.nvec = nvec;
    a.size = size;
    a.byte0 = byte0;
    a.nblk_vec = int(nbv);
    int mul_terms = 0;  // coefficients that are neither 0 nor 1
    for (int r = 0; r < R; ++r)
      for (int j = 0; j < K; ++j) {
        const uint32_t c = op.coef[size_t(r0 + r) * K + j];
        build_p3(c, &a.ptab[(r * K + j) * dev::kP3Words]);
        mul_terms += c > 1u;
      }
    // device buffers: the plan launches' residency cap (cap_for) -- a large
    // one-stripe call streams K + R shards per lane like a batched launch
    // (RS(10,4) 64 MiB encode, separately allocated shards: 275 us uncapped)
    const unsigned lds =
        !host_io && nvec > 0 && cap_for(K, R, mul_terms) ? residency_lds_bytes(current_device(), K + R) : 0u;
    void* args[] = {&a};
    ECGPU_HIP(hipLaunchKernel(reinterpret_cast<const void*>(fn), dim3(unsigned(nbv + nbb)), dim3(dev::kBlock), args,
                              lds, s));
  }
  return ECGPU_OK;
}

// Where every distinct buffer of one synchronous call lives: sources first
// (as op.srcs), then the outputs that are not also sources.  devp[i] is the
// device address the kernel uses (the buffer itself, its mapping in place, or
// a staging slot); staged[i] marks host memory that must be copied.
struct CallMap {
  std::vector<void*> bufs;
  std::vector<uint8_t*> devp;
  std::vector<char> staged;
  size_t nstage = 0;
  size_t slot = 0;   // staging slot bytes (size rounded to 256)
  int64_t size = 0;
  int rows = 0, nsrc = 0;
  bool host_io = false;  // some buffer is host memory the kernel uses in place
  size_t index(const void* p) const { return size_t(std::find(bufs.begin(), bufs.end(), p) - bufs.begin()); }
  std::vector<const uint8_t*> sources() const { return {devp.begin(), devp.begin() + nsrc}; }
  std::vector<uint8_t*> outputs(const FusedOp& op) const {
    std::vector<uint8_t*> dp(static_cast<size_t>(rows));
    for (int r = 0; r < rows; ++r) dp[size_t(r)] = devp[index(op.dsts[size_t(r)])];
    return dp;
  }
};

int map_buffers(const FusedOp& op, int64_t size, int device, bool inl, CallMap* m) {
  m->bufs = op.srcs;
  for (void* d : op.dsts)
    if (std::find(m->bufs.begin(), m->bufs.end(), d) == m->bufs.end()) m->bufs.push_back(d);
  m->size = size;
  m->slot = (size_t(size) + 255) & ~size_t(255);
  m->rows = int(op.dsts.size());
  m->nsrc = int(op.srcs.size());
  m->devp.assign(m->bufs.size(), nullptr);
  m->staged.assign(m->bufs.size(), 0);
  for (size_t i = 0; i < m->bufs.size(); ++i) {
    bool on_dev = false;
    if (int rc = classify(m->bufs[i], device, &on_dev)) return rc;
    if (on_dev) {
      m->devp[i] = static_cast<uint8_t*>(m->bufs[i]);
    } else {
      m->staged[i] = 1;
      ++m->nstage;
    }
  }
  if (inl && zero_copy_pinned()) {
    // pinned / registered host buffers are read and written by the kernel in
    // place over PCIe: no staging copy, no DMA setup, and a call's reads and
    // writes overlap on the two directions of the link
    for (size_t i = 0; i < m->bufs.size(); ++i) {
      void* d = nullptr;
      if (m->staged[i] && host_mapped(m->bufs[i], size_t(size), &d)) {
        m->staged[i] = 0;
        --m->nstage;
        m->devp[i] = static_cast<uint8_t*>(d);
        m->host_io = true;
      }
    }
  }
  return ECGPU_OK;
}

int launch_and_sync(Ctx* c, const FusedOp& op, const CallMap& m, bool host_io) {
  if (int rc = launch_inline(op, m.sources(), m.outputs(op), m.size, c->stream, host_io)) return rc;
  ECGPU_HIP(hipStreamSynchronize(c->stream));
  ECGPU_HIP(hipGetLastError());
  return ECGPU_OK;
}

// Small calls: every staged buffer goes through coherent pinned memory the
// kernel reads and writes in place -- host copies and ONE launch, no DMA.
int exec_zero_copy(Ctx* c, const FusedOp& op, CallMap& m) {
  if (int rc = ensure_zc(c, m.nstage * m.slot)) return rc;
  size_t next = 0;
  for (size_t i = 0; i < m.bufs.size(); ++i)
    if (m.staged[i]) m.devp[i] = c->zc + (next++) * m.slot;
  for (int j = 0; j < m.nsrc; ++j)
    if (m.staged[size_t(j)]) std::memcpy(m.devp[size_t(j)], op.srcs[size_t(j)], size_t(m.size));
  if (int rc = launch_and_sync(c, op, m, /*host_io=*/true)) return rc;
  for (int r = 0; r < m.rows; ++r) {
    const size_t i = m.index(op.dsts[size_t(r)]);
    if (m.staged[i]) std::memcpy(op.dsts[size_t(r)], m.devp[i], size_t(m.size));
  }
  return ECGPU_OK;
}

// Larger calls with few output bytes: sources cross by HIP's copies (a
// contiguous pageable run goes as one pinned blit at link rate), the kernel
// writes the outputs straight into coherent pinned memory and the calling
// thread copies them out: no per-output pageable D2H (67 us per 1 MiB shard,
// tools/pageable_duplex_probe.cpp).  Returns ECGPU_OK with *done = false when
// the call does not qualify (an output that is also a source, or outputs
// above zc_out_max() / zc_out_shard_max()).
int exec_outputs_zero_copy(Ctx* c, const FusedOp& op, CallMap& m, bool* done) {
  *done = false;
  size_t nout = 0;
  std::vector<char> is_out(m.bufs.size(), 0);
  for (int r = 0; r < m.rows; ++r) {
    const size_t i = m.index(op.dsts[size_t(r)]);
    if (!m.staged[i] || is_out[i]) continue;
    if (i < size_t(m.nsrc)) return ECGPU_OK;  // aliased: keep the staged path
    is_out[i] = 1;
    ++nout;
  }
  if (nout == 0 || nout * size_t(m.size) > zc_out_max() || size_t(m.size) > zc_out_shard_max()) return ECGPU_OK;
  const size_t nin = m.nstage - nout;
  if (int rc = ensure_zc(c, nout * m.slot)) return rc;
  if (int rc = ensure_stage(c, std::max<size_t>(nin, 1) * m.slot)) return rc;
  size_t ni = 0, no = 0;
  std::vector<char*> staged_hp;
  for (size_t i = 0; i < m.bufs.size(); ++i) {
    if (!m.staged[i]) continue;
    if (is_out[i]) {
      m.devp[i] = c->zc + (no++) * m.slot;
    } else {
      m.devp[i] = c->stage + (ni++) * m.slot;
      staged_hp.push_back(static_cast<char*>(m.bufs[i]));
    }
  }
  if (int rc = copy_shards(true, c->stage, m.slot, staged_hp, size_t(m.size), c->stream)) return rc;
  if (int rc = launch_and_sync(c, op, m, /*host_io=*/true)) return rc;
  for (size_t i = 0; i < m.bufs.size(); ++i)
    if (m.staged[i] && is_out[i]) std::memcpy(m.bufs[i], m.devp[i], size_t(m.size));
  *done = true;
  return ECGPU_OK;
}

// Everything else: staged buffers go through the context's HBM slab, by the
// pinned bounce (mid-size) or HIP's copies (large); non-inline ops (w = 16 /
// 32, > 16 sources, the LDS engine) run a cached bound plan.
int exec_staged(Ctx* c, const FusedOp& op, CallMap& m, bool inl) {
  const size_t slot = m.slot, size = size_t(m.size);
  const int rows = m.rows, nsrc = m.nsrc;
  // With several launches (> 4 rows) an output that is also a source must
  // not be overwritten before the last launch reads it: write to temps.
  const bool via_temp = op.dst_is_src && rows > dev::kMaxRows;
  const size_t ntemp = via_temp ? size_t(rows) : 0;
  if (int rc = ensure_stage(c, (m.nstage + ntemp) * slot)) return rc;
  size_t next = 0;
  for (size_t i = 0; i < m.bufs.size(); ++i)
    if (m.staged[i]) m.devp[i] = c->stage + (next++) * slot;
  // Staged sources take the first staging slots (bufs lists sources first),
  // so with the pinned bounce they go up as one contiguous DMA.
  const bool bounce = m.nstage > 0 && m.nstage * slot <= bounce_max();
  if (bounce)
    if (int rc = ensure_bounce(c, m.nstage * slot)) return rc;
  auto bounce_of = [&](size_t i) { return c->bounce + (m.devp[i] - c->stage); };
  std::vector<char*> staged_hp;
  for (size_t j = 0; j < op.srcs.size(); ++j)
    if (m.staged[j]) {
      staged_hp.push_back(static_cast<char*>(op.srcs[j]));
      if (bounce) std::memcpy(bounce_of(j), op.srcs[j], size);
    }
  if (bounce && !staged_hp.empty()) {
    ECGPU_HIP(hipMemcpyAsync(c->stage, c->bounce, staged_hp.size() * slot, hipMemcpyHostToDevice, c->stream));
  } else if (int rc = copy_shards(true, c->stage, slot, staged_hp, size, c->stream)) {
    return rc;
  }

  const std::vector<const uint8_t*> sp = m.sources();
  std::vector<uint8_t*> dp = m.outputs(op);
  if (via_temp)
    for (int r = 0; r < rows; ++r) dp[size_t(r)] = c->stage + (m.nstage + size_t(r)) * slot;
  if (nsrc == 0) {
    // Every output is identically zero (e.g. region multiply by 0 without
    // add, galois.cpp:447-451): nothing to read.
    for (int r = 0; r < rows; ++r) ECGPU_HIP(hipMemsetAsync(dp[size_t(r)], 0, size, c->stream));
  } else if (inl) {
    if (int rc = launch_inline(op, sp, dp, m.size, c->stream, m.host_io)) return rc;
  } else {
    ecgpu_plan* p = nullptr;
    if (int rc = ctx_plan(c, rows, nsrc, op.coef, op.w, &p)) return rc;
    // sp/dp outlive the stream sync below
    if (int rc = plan_bind(p, 1, sp.data(), dp.data(), m.size, c->stream, /*keep_alive=*/true)) return rc;
    if (int rc = plan_launch(p, c->stream)) return rc;
  }
  // staged outputs, in slot order
  std::vector<std::pair<uint8_t*, char*>> outs;  // (device slot, host pointer)
  for (int r = 0; r < rows; ++r) {
    const size_t i = m.index(op.dsts[size_t(r)]);
    if (via_temp)
      ECGPU_HIP(hipMemcpyAsync(m.devp[i], dp[size_t(r)], size, hipMemcpyDeviceToDevice, c->stream));
    if (m.staged[i]) outs.emplace_back(m.devp[i], static_cast<char*>(op.dsts[size_t(r)]));
  }
  std::sort(outs.begin(), outs.end());
  if (bounce) {
    // one D2H per run of adjacent slots (the bounce mirrors the slab)
    for (size_t a = 0; a < outs.size();) {
      size_t b = a + 1;
      while (b < outs.size() && outs[b].first == outs[b - 1].first + slot) ++b;
      const size_t off = size_t(outs[a].first - c->stage);
      ECGPU_HIP(hipMemcpyAsync(c->bounce + off, outs[a].first, (b - a - 1) * slot + size, hipMemcpyDeviceToHost,
                               c->stream));
      a = b;
    }
    ECGPU_HIP(hipStreamSynchronize(c->stream));
    ECGPU_HIP(hipGetLastError());
    for (const auto& o : outs) std::memcpy(o.second, c->bounce + (o.first - c->stage), size);
    return ECGPU_OK;
  }
  // outputs in consecutive slots: one 2-D copy per evenly spaced run of host outputs
  bool consecutive = true;
  for (size_t i = 1; i < outs.size() && consecutive; ++i) consecutive = outs[i].first == outs[0].first + i * slot;
  if (consecutive && !outs.empty()) {
    std::vector<char*> hp;
    for (const auto& o : outs) hp.push_back(o.second);
    if (int rc = copy_shards(false, outs[0].first, slot, hp, size, c->stream)) return rc;
  } else {
    for (const auto& o : outs) ECGPU_HIP(hipMemcpyAsync(o.second, o.first, size, hipMemcpyDeviceToHost, c->stream));
  }
  ECGPU_HIP(hipStreamSynchronize(c->stream));
  ECGPU_HIP(hipGetLastError());
  return ECGPU_OK;
}

// Runs a fused op synchronously over `size` bytes of every buffer on
// `device`: maps the buffers, then the cheapest staging mode for the host
// ones (§8 of DESIGN.md; the thresholds are measured, see bounce_max / zc_max
// / zc_out_max).
int execute_on(const FusedOp& op, int64_t size, int device) {
  CtxLease lease(device);
  if (!lease.c) return lease.rc;
  Ctx* c = lease.c;
  DeviceGuard g(device);
  const bool inl = inline_ok(op, size);
  CallMap m;
  if (int rc = map_buffers(op, size, device, inl, &m)) return rc;
  if (inl && m.nstage > 0 && m.nstage * size_t(size) <= zc_max()) return exec_zero_copy(c, op, m);
  if (inl && m.nstage > 0 && m.nstage * m.slot > bounce_max()) {
    bool done = false;
    if (int rc = exec_outputs_zero_copy(c, op, m, &done)) return rc;
    if (done) return ECGPU_OK;
  }
  return exec_staged(c, op, m, inl);
}

// ------------------------------------------------------- split calls ----
// A synchronous call on host memory can be cut into contiguous 16-B-aligned
// byte ranges that run concurrently, each on its own context (thread, stream,
// staging) and device.  Every byte column of a fused op is independent -- a
// column's outputs depend on that column of the sources only, identical
// buffers included -- so the ranges' bytes are the call's.  This is the
// reference client's own split (encode_mul_thread, client_main.cpp:1074-1164)
// done inside one call, and SURVEY §8e's "one huge stripe: contiguous byte
// ranges of S/N" over the visible GPUs: each range crosses its own PCIe link.
// ECGPU_SPLIT: 0 off (default), -1 one range per visible device, N > 0 N
// ranges over the devices in turn (N > 1 on one GPU: N contexts on it);
// ranges are at least ECGPU_SPLIT_MIN_KIB.  Calls with a device buffer stay
// whole (the buffer fixes the device).
int split_ways(const FusedOp& op, int64_t size, int* ndev) {
  const int v = knob(Knob::kSplit);
  if (v == 0) return 1;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
    (void)hipGetLastError();
    return 1;
  }
  *ndev = n;
  const int64_t min_bytes = int64_t(std::max(16, knob(Knob::kSplitMinKib))) << 10;
  const int ways = int(std::min<int64_t>(v < 0 ? n : v, size / min_bytes));
  if (ways <= 1) return 1;
  auto on_host = [](const void* p) {
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
      (void)hipGetLastError();
      return true;  // unregistered pageable memory
    }
    return attr.type != hipMemoryTypeDevice && attr.type != hipMemoryTypeManaged;
  };
  for (void* p : op.srcs)
    if (!on_host(p)) return 1;
  for (void* p : op.dsts)
    if (!on_host(p)) return 1;
  return ways;
}

FusedOp shifted(const FusedOp& op, int64_t off) {
  FusedOp s;
  for (void* p : op.srcs) s.srcs.push_back(static_cast<char*>(p) + off);
  for (void* p : op.dsts) s.dsts.push_back(static_cast<char*>(p) + off);
  s.coef = op.coef;
  s.w = op.w;
  s.dst_is_src = op.dst_is_src;
  return s;
}

int execute_split(const FusedOp& op, int64_t size, int ways, int ndev) {
  const int64_t per = (size / ways) & ~int64_t(15);  // whole words at w = 16 / 32
  const int first = current_device();
  std::vector<int> rc(size_t(ways), ECGPU_OK);
  std::vector<std::string> msg(static_cast<size_t>(ways));
  auto run = [&](int i) {
    const int64_t off = per * i, len = i + 1 < ways ? per : size - off;
    rc[size_t(i)] = execute_on(shifted(op, off), len, (first + i) % ndev);
    if (rc[size_t(i)]) msg[size_t(i)] = t_err;
  };
  std::vector<std::thread> workers;
  int next = 1;
  try {
    for (; next < ways; ++next) workers.emplace_back(run, next);
  } catch (const std::system_error&) {  // no thread: the rest run here, in turn
  }
  run(0);
  for (int i = next; i < ways; ++i) run(i);
  for (auto& t : workers) t.join();
  for (int i = 0; i < ways; ++i)
    if (rc[size_t(i)])
      return fail(rc[size_t(i)], msg[size_t(i)] + " (byte range " + std::to_string(per * i) + " of a call split " +
                                     std::to_string(ways) + " ways)");
  return ECGPU_OK;
}

// A synchronous call over `size` bytes of every buffer of the fused op.
int execute(const FusedOp& op, int64_t size, const char* call) {
  if (op.w != 8 && size % (op.w / 8) != 0)
    return fail(ECGPU_ERR_ARG, "w = " + std::to_string(op.w) + ": size must be a multiple of the word size");
  // identical or disjoint buffers, checked before anything touches the GPU
  if (int rc = check_op_buffers(call, op, size)) return rc;
  add_stats(op);
  if (op.dsts.empty() || size <= 0) return ECGPU_OK;
  int ndev = 1;
  const int ways = split_ways(op, size, &ndev);
  if (ways > 1) return execute_split(op, size, ways, ndev);
  return execute_on(op, size, current_device());
}

ECGPU_RT_END
// ================================================================ C ABI ====
extern "C" {


ECGPU_API ecgpu_plan* ecgpu_plan_create(int rows, int nsrc, const int* coefs, int device) {
  if (rows <= 0 || nsrc <= 0 || !coefs) {
    fail(ECGPU_ERR_ARG, "ecgpu_plan_create: rows, nsrc > 0 and coefs required");
    return nullptr;
  }
  if (device < 0) device = current_device();
  auto* p = new ecgpu_plan();
  if (plan_init(p, rows, nsrc, coefs, device) != ECGPU_OK) {
    plan_free(p);
    return nullptr;
  }
  return p;
}

ECGPU_API int ecgpu_plan_bind(ecgpu_plan* p, int stripes, const uint8_t* const* src_ptrs, uint8_t* const* dst_ptrs,
                              int64_t size) {
  if (!p || stripes < 0 || size < 0 || (stripes && (!src_ptrs || !dst_ptrs)))
    return fail(ECGPU_ERR_ARG, "ecgpu_plan_bind: bad arguments");
  if (int rc = ecgpu_plan_check_buffers(p->rows, p->nsrc, stripes, src_ptrs, dst_ptrs, size)) return rc;
  return plan_bind(p, stripes, src_ptrs, dst_ptrs, size, nullptr);
}

ECGPU_API int ecgpu_plan_set_kernel(ecgpu_plan* p, int kind, int nontemporal) {
  if (!p || (kind != ECGPU_KERNEL_PERM && kind != ECGPU_KERNEL_LDS))
    return fail(ECGPU_ERR_ARG, "ecgpu_plan_set_kernel: bad arguments");
  p->kind = kind;
  p->nt = std::min(kStorePolicies - 1, std::max(0, nontemporal));
  return ECGPU_OK;
}

ECGPU_API int ecgpu_plan_launch(ecgpu_plan* p, void* stream) {
  if (!p) return fail(ECGPU_ERR_ARG, "ecgpu_plan_launch: null plan");
  return plan_launch(p, static_cast<hipStream_t>(stream));
}

ECGPU_API void ecgpu_plan_destroy(ecgpu_plan* p) { plan_free(p); }

ECGPU_API int ecgpu_device_pci_bus_id(int device, char* buf, int len) {
  if (!buf || len < 13) return fail(ECGPU_ERR_ARG, "ecgpu_device_pci_bus_id: buffer of >= 13 bytes required");
  ECGPU_HIP(hipDeviceGetPCIBusId(buf, len, device));
  return ECGPU_OK;
}

ECGPU_API int ecgpu_host_register(void* ptr, int64_t bytes) {
  if (!ptr || bytes <= 0) return fail(ECGPU_ERR_ARG, "ecgpu_host_register: bad arguments");
  ECGPU_HIP(hipHostRegister(ptr, size_t(bytes), hipHostRegisterDefault));
  return ECGPU_OK;
}

ECGPU_API int ecgpu_host_unregister(void* ptr) {
  if (!ptr) return fail(ECGPU_ERR_ARG, "ecgpu_host_unregister: null");
  ECGPU_HIP(hipHostUnregister(ptr));
  return ECGPU_OK;
}

ECGPU_API int ecgpu_encode_batch(int k, int m, const int* matrix, int stripes, const uint8_t* const* data,
                                 uint8_t* const* coding, int64_t size, void* stream) {
  if (k <= 0 || m <= 0 || !matrix || stripes < 0 || size < 0 || (stripes && (!data || !coding)))
    return fail(ECGPU_ERR_ARG, "ecgpu_encode_batch: bad arguments");
  if (int rc = ecgpu_plan_check_buffers(m, k, stripes, data, coding, size)) return rc;
  ecgpu_plan* p = ecgpu_plan_create(m, k, matrix, -1);
  if (!p) return ECGPU_ERR_HIP;
  int rc = plan_bind(p, stripes, data, coding, size, static_cast<hipStream_t>(stream));
  if (rc == ECGPU_OK) rc = plan_launch(p, static_cast<hipStream_t>(stream));
  if (rc == ECGPU_OK && stream) {
    hipError_t e = hipStreamSynchronize(static_cast<hipStream_t>(stream));
    if (e != hipSuccess) rc = fail(ECGPU_ERR_HIP, hipGetErrorString(e));
  } else if (rc == ECGPU_OK) {
    hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) rc = fail(ECGPU_ERR_HIP, hipGetErrorString(e));
  }
  plan_free(p);
  return rc;
}

namespace {
bool valid_w(int w) { return w == 8 || w == 16 || w == 32; }
}  // namespace

ECGPU_API int ecgpu_jerasure_matrix_encode(int k, int m, int w, int* matrix, char** data_ptrs, char** coding_ptrs,
                                           int size) {
  if (!valid_w(w)) return fail(ECGPU_ERR_ARG, "ecgpu_jerasure_matrix_encode: w must be 8, 16 or 32");
  LinearTracker t(w);
  plan_encode(t, k, m, matrix, data_ptrs, coding_ptrs, size);
  return execute(t.finish(), size, "jerasure_matrix_encode");
}

ECGPU_API int ecgpu_jerasure_matrix_decode(int k, int m, int w, int* matrix, int row_k_ones, int* erasures,
                                           char** data_ptrs, char** coding_ptrs, int size) {
  if (!valid_w(w)) return ECGPU_ERR;  // jerasure.cpp:165: any other w returns -1
  LinearTracker t(w);
  if (plan_decode(t, k, m, matrix, row_k_ones, erasures, data_ptrs, coding_ptrs, size) < 0) return ECGPU_ERR;
  return execute(t.finish(), size, "jerasure_matrix_decode");
}

ECGPU_API int ecgpu_jerasure_matrix_dotprod(int k, int w, int* matrix_row, int* src_ids, int dest_id,
                                            char** data_ptrs, char** coding_ptrs, int size) {
  if (w == 1) {
    // jerasure.cpp:561-620 at w = 1: coefficient 1 copies (first) or XORs the
    // source; any other non-zero coefficient has no region multiply at w = 1
    // (the reference's switch has no case for it) but still counts its bytes
    // as gf and marks the destination initialised.  So the map is the XOR of
    // the unit-coefficient sources -- the XOR-only kernel over GF(2^8)
    // bytes, where 1 * x = x.
    LinearTracker t(8);
    auto buf = [&](int i) -> void* {
      const int id = src_ids ? src_ids[i] : i;
      return id < k ? static_cast<void*>(data_ptrs[id]) : static_cast<void*>(coding_ptrs[id - k]);
    };
    void* dst = dest_id < k ? static_cast<void*>(data_ptrs[dest_id]) : static_cast<void*>(coding_ptrs[dest_id - k]);
    bool init = false;
    for (int i = 0; i < k; ++i) {
      if (matrix_row[i] != 1) continue;
      if (!init) {
        t.copy(dst, buf(i));
        t.count(0, 0, double(size));
        init = true;
      } else {
        t.xor3(buf(i), dst, dst);
        t.count(double(size), 0, 0);
      }
    }
    for (int i = 0; i < k; ++i)
      if (matrix_row[i] != 0 && matrix_row[i] != 1) t.count(0, double(size), 0);
    return execute(t.finish(), size, "jerasure_matrix_dotprod");
  }
  if (!valid_w(w)) return fail(ECGPU_ERR_ARG, "ecgpu_jerasure_matrix_dotprod: w must be 1, 8, 16 or 32");
  LinearTracker t(w);
  t.dotprod(k, matrix_row, src_ids, dest_id, data_ptrs, coding_ptrs, size);
  return execute(t.finish(), size, "jerasure_matrix_dotprod");
}

ECGPU_API int ecgpu_jerasure_do_parity(int k, char** data_ptrs, char* parity_ptr, int size) {
  LinearTracker t;
  t.copy(parity_ptr, data_ptrs[0]);
  for (int i = 1; i < k; ++i) t.xor3(data_ptrs[i], parity_ptr, parity_ptr);
  t.count(double(size) * (k - 1), 0, double(size));
  return execute(t.finish(), size, "jerasure_do_parity");
}

ECGPU_API int ecgpu_galois_w08_region_multiply(char* region, int multby, int nbytes, char* r2, int add) {
  LinearTracker t;
  if (r2 == nullptr)
    t.mul(region, multby, region, false);  // galois.cpp:429,447: in place, add ignored
  else
    t.mul(region, multby, r2, add != 0);
  return execute(t.finish(), nbytes, "galois_w08_region_multiply");
}

// galois.cpp:469-542: nbytes/2 words; multby 0 zeroes (no add) or does
// nothing (add); in place (r2 NULL) ignores add.
ECGPU_API int ecgpu_galois_w16_region_multiply(char* region, int multby, int nbytes, char* r2, int add) {
  LinearTracker t(16);
  char* dst = r2 ? r2 : region;
  if (multby == 0) {
    if (!add) t.mul(region, 0, dst, false);
  } else {
    t.mul(region, multby, dst, r2 != nullptr && add != 0);
  }
  return execute(t.finish(), nbytes & ~1, "galois_w16_region_multiply");
}

// galois.cpp:666-727: nbytes/4 words; add applies even in place.
ECGPU_API int ecgpu_galois_w32_region_multiply(char* region, int multby, int nbytes, char* r2, int add) {
  LinearTracker t(32);
  t.mul(region, multby, r2 ? r2 : region, add != 0);
  return execute(t.finish(), nbytes & ~3, "galois_w32_region_multiply");
}

ECGPU_API int ecgpu_galois_region_xor(char* r1, char* r2, char* r3, int nbytes) {
  LinearTracker t;
  t.xor3(r1, r2, r3);
  return execute(t.finish(), nbytes, "galois_region_xor");
}

ECGPU_API int ecgpu_reed_sol_galois_w08_region_multby_2(char* region, int nbytes) {
  LinearTracker t;
  t.mul(region, 2, region, false);
  return execute(t.finish(), nbytes);
}

// reed_sol.cpp:158-198 / :90-106 (whole words).
ECGPU_API int ecgpu_reed_sol_galois_w16_region_multby_2(char* region, int nbytes) {
  LinearTracker t(16);
  t.mul(region, 2, region, false);
  return execute(t.finish(), nbytes & ~1);
}

ECGPU_API int ecgpu_reed_sol_galois_w32_region_multby_2(char* region, int nbytes) {
  LinearTracker t(32);
  t.mul(region, 2, region, false);
  return execute(t.finish(), nbytes & ~3);
}

// reed_sol.cpp:200-225: P = XOR of data; Q = Horner sum of 2^j d_j.
// Returns 1, or 0 for a w the reference does not handle.
ECGPU_API int ecgpu_reed_sol_r6_encode(int k, int w, char** data_ptrs, char** coding_ptrs, int size) {
  if (!valid_w(w)) return 0;
  LinearTracker t(w);
  t.copy(coding_ptrs[0], data_ptrs[0]);
  for (int i = 1; i < k; ++i) t.xor3(coding_ptrs[0], data_ptrs[i], coding_ptrs[0]);
  t.copy(coding_ptrs[1], data_ptrs[k - 1]);
  for (int i = k - 2; i >= 0; --i) {
    t.mul(coding_ptrs[1], 2, coding_ptrs[1], false);
    t.xor3(coding_ptrs[1], data_ptrs[i], coding_ptrs[1]);
  }
  const int rc = execute(t.finish(), size, "reed_sol_r6_encode");
  return rc == ECGPU_OK ? 1 : rc;
}

ECGPU_API int ecgpu_jerasure_get_stats(double* fill_in) {
  std::lock_guard<std::mutex> lk(g_stats_mu);
  for (int i = 0; i < 3; ++i) {
    fill_in[i] = g_stats[i];
    g_stats[i] = 0;
  }
  return ECGPU_OK;
}

}  // extern "C"
