// dispatch_wide.hip -- how a w = 16 / 32 plan launches (gf_kernels_wide.hpp,
// the pipelined forms specialised in wide_spec.hip): the LDS nibble-table or
// v_perm engine per launch, unit structure, persistent grid size, word
// tails, and the tables a plan uploads.  Its own build ID
// (ecgpu_build_id(2)): an edit here leaves the w = 8 kernels' ID unchanged.
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
#include "wide_spec.hpp"

using namespace ecgpu;
using namespace ecgpu::rt;
using dev::ApplyArgs;

ECGPU_RT_BEGIN

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

// The w = 16 / 32 part of plan_init: [v_perm tables | nibble tables |
// coefficient classes], one upload.
int plan_init_wide(ecgpu_plan* p, const int* coefs) {
  const size_t n = p->coef.size();
  const int w = p->w;
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

ECGPU_RT_END
