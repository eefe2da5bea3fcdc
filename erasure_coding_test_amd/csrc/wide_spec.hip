// wide_spec.hip -- one R's share of the pipelined w = 16 / 32 kernel table
// (wide_spec.hpp).  Built four times: -DECGPU_SPEC_R=1..4.
#include <hip/hip_runtime.h>

#include "wide_spec.hpp"

#ifndef ECGPU_SPEC_R
#error "build with -DECGPU_SPEC_R=<1..4>"
#endif

namespace ecgpu {
namespace {

constexpr int kR = ECGPU_SPEC_R;

template <int K>
constexpr SpecKernelFn wide_unit_fn() {
  if constexpr (kR >= 2) return &dev::gf_apply_wide_pipe<K, kR, dev::kPipeW32Unit>;
  else return nullptr;  // the unit form needs a row besides the unit row
}

template <int K>
struct WidePipe {
  static constexpr SpecKernelFn fn[3] = {&dev::gf_apply_wide_pipe<K, kR, dev::kPipeW32>, wide_unit_fn<K>(),
                                         &dev::gf_apply_wide_pipe<K, kR, dev::kPipeW16>};
};

template <int... Ks>
SpecKernelFn pick_wide_pipe(int K, int mode) {
  SpecKernelFn out = nullptr;
  ((K == Ks ? (out = WidePipe<Ks>::fn[mode], 0) : 0), ...);
  return out;
}

}  // namespace

#define ECGPU_CAT2(a, b) a##b
#define ECGPU_CAT(a, b) ECGPU_CAT2(a, b)
SpecKernelFn ECGPU_CAT(wide_pipe_kernel_r, ECGPU_SPEC_R)(int K, int mode) {
  if (mode < 0 || mode > 2) return nullptr;
  return pick_wide_pipe<1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16>(K, mode);
}

}  // namespace ecgpu
