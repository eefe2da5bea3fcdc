// gf_spec.hip -- one R's share of the specialised w = 8 kernel table
// (gf_spec.hpp).  Built four times: -DECGPU_SPEC_R=1..4.
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

// NT: loads always non-temporal (bit 0), NT >> 1 = store policy
// (gf_kernels.hpp store16t: 0 plain, 1 nt)
template <int K, int U, int STORE>
constexpr SpecKernelFn apply_fn() { return &dev::gf_apply<K, kR, kUnitVariants[U], 1, 3, 1 | (STORE << 1)>; }

template <int K, int S>
struct Pol {
  static constexpr SpecKernelFn apply[5] = {apply_fn<K, 0, S>(), apply_fn<K, 1, S>(), apply_fn<K, 2, S>(),
                                            apply_fn<K, 3, S>(), apply_fn<K, 4, S>()};
};

template <int K, int U, bool ZC>
constexpr InlineKernelFn inl_fn() { return &dev::gf_apply_inl<K, kR, kUnitVariants[U], ZC>; }

template <int K>
struct Row {
  static constexpr InlineKernelFn inl[2][5] = {
      {inl_fn<K, 0, false>(), inl_fn<K, 1, false>(), inl_fn<K, 2, false>(), inl_fn<K, 3, false>(), inl_fn<K, 4, false>()},
      {inl_fn<K, 0, true>(), inl_fn<K, 1, true>(), inl_fn<K, 2, true>(), inl_fn<K, 3, true>(), inl_fn<K, 4, true>()}};
  static constexpr const SpecKernelFn* apply[kStorePolicies] = {Pol<K, 0>::apply, Pol<K, 1>::apply};
  static constexpr SpecKernelFn lds = &dev::gf_apply_lds<K, kR>;
};

template <int... Ks>
SpecKernelFn pick(bool lds, int K, int u, int store_pol) {
  SpecKernelFn out = nullptr;
  ((K == Ks ? (out = lds ? Row<Ks>::lds : Row<Ks>::apply[store_pol][u], 0) : 0), ...);
  return out;
}

template <int... Ks>
InlineKernelFn pick_inl(int K, int u, bool zc) {
  InlineKernelFn out = nullptr;
  ((K == Ks ? (out = Row<Ks>::inl[zc ? 1 : 0][u], 0) : 0), ...);
  return out;
}

}  // namespace

#define ECGPU_CAT2(a, b) a##b
#define ECGPU_CAT(a, b) ECGPU_CAT2(a, b)
SpecKernelFn ECGPU_CAT(spec_kernel_r, ECGPU_SPEC_R)(bool lds, int K, int unit_variant, int store_pol) {
  if (unit_variant < 0 || unit_variant > 4 || store_pol < 0 || store_pol >= kStorePolicies) return nullptr;
  return pick<1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16>(lds, K, unit_variant, store_pol);
}

InlineKernelFn ECGPU_CAT(inline_kernel_r, ECGPU_SPEC_R)(int K, int unit_variant, bool zc) {
  if (unit_variant < 0 || unit_variant > 4) return nullptr;
  return pick_inl<1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16>(K, unit_variant, zc);
}

}  // namespace ecgpu
