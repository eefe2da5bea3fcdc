// dispatch_w8.hip -- how a w = 8 plan launches: the production v_perm engine
// or the LDS nibble-table engine (gf_kernels_w8.hpp, specialised in
// gf_spec.hip), the unit-coefficient structure of each launch, its residency
// cap and store policy, the coefficient tables a plan uploads.  With
// gf_kernels_w8.hpp and gf_spec.* this file is the w = 8 kernel build ID
// (ecgpu_build_id(1), erasure_coding_test_amd/build.py): what a rocprofv3 PMC
// record of the bench's encode / decode launches is valid for.  The
// synchronous calls' staging and the C ABI live in ecgpu_runtime.hip, the
// w = 16 / 32 dispatch in dispatch_wide.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "ecgpu.h"
#include "gf_host.hpp"
#include "gf_kernels.hpp"
#include "knobs.hpp"
#include "runtime.hpp"
#include "gf_spec.hpp"

using namespace ecgpu;
using namespace ecgpu::rt;
using dev::ApplyArgs;
using dev::u32x4;

ECGPU_RT_BEGIN

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
unsigned residency_lds_bytes(int device, int streams, unsigned static_bytes) {
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

// The w = 8 part of plan_init: [2-bit | 3-bit-slice | nibble] tables of
// every coefficient, one upload.
int plan_init_w8(ecgpu_plan* p, const int* coefs) {
  const size_t n = p->coef.size();
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

// Specialised w = 8 column launches per engine (ECGPU_KERNEL_PERM / _LDS),
// for tests that a knob switch reached the launches (ecgpu_engine_launches).
std::atomic<int64_t> g_engine_launches[2];

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
    if (spec && nvec > 0) g_engine_launches[use_lds ? 1 : 0].fetch_add(1, std::memory_order_relaxed);
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

ECGPU_RT_END

extern "C" ECGPU_API int64_t ecgpu_engine_launches(int kind) {
  return kind == 0 || kind == 1 ? ecgpu::rt::g_engine_launches[kind].load(std::memory_order_relaxed) : -1;
}
