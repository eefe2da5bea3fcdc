// gf_spec.hip -- one R's share of the specialised kernel table (gf_spec.hpp).
// Built four times: -DECGPU_SPEC_R=1..4.
#include <hip/hip_runtime.h>

#include "gf_spec.hpp"

#ifndef ECGPU_SPEC_R
#error "build with -DECGPU_SPEC_R=<1..4>"
#endif

namespace ecgpu {
namespace {

constexpr int kR = ECGPU_SPEC_R;
constexpr int kUnitVariants[5] = {dev::kUnitNone, dev::kUnitCol0, dev::kUnitRow0, dev::kUnitCol0 | dev::kUnitRow0,
                                  dev::kUnitAll};

// NT bits: loads always non-temporal (bit 0), stores per policy (bit 1)
template <int K, int U, int STORE_NT>
constexpr SpecKernelFn apply_fn() { return &dev::gf_apply<K, kR, kUnitVariants[U], 1, 3, 1 | (STORE_NT << 1)>; }

template <int K>
struct Row {
  static constexpr SpecKernelFn apply[2][5] = {
      {apply_fn<K, 0, 0>(), apply_fn<K, 1, 0>(), apply_fn<K, 2, 0>(), apply_fn<K, 3, 0>(), apply_fn<K, 4, 0>()},
      {apply_fn<K, 0, 1>(), apply_fn<K, 1, 1>(), apply_fn<K, 2, 1>(), apply_fn<K, 3, 1>(), apply_fn<K, 4, 1>()}};
  static constexpr SpecKernelFn lds = &dev::gf_apply_lds<K, kR>;
};

template <int... Ks>
SpecKernelFn pick(bool lds, int K, int u, int store_nt) {
  SpecKernelFn out = nullptr;
  ((K == Ks ? (out = lds ? Row<Ks>::lds : Row<Ks>::apply[store_nt ? 1 : 0][u], 0) : 0), ...);
  return out;
}

}  // namespace

#define ECGPU_CAT2(a, b) a##b
#define ECGPU_CAT(a, b) ECGPU_CAT2(a, b)
SpecKernelFn ECGPU_CAT(spec_kernel_r, ECGPU_SPEC_R)(bool lds, int K, int unit_variant, int store_nt) {
  if (unit_variant < 0 || unit_variant > 4) return nullptr;
  return pick<1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16>(lds, K, unit_variant, store_nt);
}

}  // namespace ecgpu
