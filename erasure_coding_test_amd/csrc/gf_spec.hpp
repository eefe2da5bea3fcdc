// gf_spec.hpp -- the compile-time-specialised production kernels
// (gf_kernels.hpp gf_apply<K, R, UNITS, 1, 3, NT> and gf_apply_lds<K, R>)
// for K = 1..kMaxSpecK sources.  Instantiated in four translation units, one
// per output-row count R (gf_spec.hip built with -DECGPU_SPEC_R=1..4), so
// the build compiles them in parallel.
#pragma once
#include "gf_kernels.hpp"

namespace ecgpu {

using SpecKernelFn = void (*)(dev::ApplyArgs);
using InlineKernelFn = void (*)(dev::InlineArgs);
constexpr int kStorePolicies = 2;

// store_pol: store cache policy of the production kernel, 0 plain, 1 nt
// (gf_kernels.hpp store16t; loads are always
// non-temporal).  lds: the LDS nibble-table kernel instead.
// unit_variant indexes kUnitVariants (ecgpu_runtime.hip).  nullptr if K is
// outside 1..kMaxSpecK.
SpecKernelFn spec_kernel_r1(bool lds, int K, int unit_variant, int store_pol);
SpecKernelFn spec_kernel_r2(bool lds, int K, int unit_variant, int store_pol);
SpecKernelFn spec_kernel_r3(bool lds, int K, int unit_variant, int store_pol);
SpecKernelFn spec_kernel_r4(bool lds, int K, int unit_variant, int store_pol);

// gf_apply_inl<K, R, UNITS, ZC> (one stripe, everything in the kernel
// arguments; zc: the grid-stride form for host memory used in place);
// nullptr if K is outside 1..kMaxSpecK.
InlineKernelFn inline_kernel_r1(int K, int unit_variant, bool zc);
InlineKernelFn inline_kernel_r2(int K, int unit_variant, bool zc);
InlineKernelFn inline_kernel_r3(int K, int unit_variant, bool zc);
InlineKernelFn inline_kernel_r4(int K, int unit_variant, bool zc);

inline InlineKernelFn inline_kernel(int K, int R, int unit_variant, bool zc) {
  switch (R) {
    case 1: return inline_kernel_r1(K, unit_variant, zc);
    case 2: return inline_kernel_r2(K, unit_variant, zc);
    case 3: return inline_kernel_r3(K, unit_variant, zc);
    case 4: return inline_kernel_r4(K, unit_variant, zc);
    default: return nullptr;
  }
}

inline SpecKernelFn spec_kernel(bool lds, int K, int R, int unit_variant, int store_pol) {
  switch (R) {
    case 1: return spec_kernel_r1(lds, K, unit_variant, store_pol);
    case 2: return spec_kernel_r2(lds, K, unit_variant, store_pol);
    case 3: return spec_kernel_r3(lds, K, unit_variant, store_pol);
    case 4: return spec_kernel_r4(lds, K, unit_variant, store_pol);
    default: return nullptr;
  }
}

}  // namespace ecgpu
