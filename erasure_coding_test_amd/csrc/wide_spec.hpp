// wide_spec.hpp -- the compile-time-specialised pipelined w = 16 / 32
// kernels (gf_kernels_wide.hpp gf_apply_wide_pipe<K, R, mode>) for K =
// 1..kMaxSpecK sources, instantiated in four translation units, one per
// output-row count R (wide_spec.hip built with -DECGPU_SPEC_R=1..4).
#pragma once
#include "gf_spec.hpp"

namespace ecgpu {

// mode: dev::WidePipeMode; nullptr if K is outside 1..kMaxSpecK or the mode
// needs more rows (the unit form: R >= 2).
SpecKernelFn wide_pipe_kernel_r1(int K, int mode);
SpecKernelFn wide_pipe_kernel_r2(int K, int mode);
SpecKernelFn wide_pipe_kernel_r3(int K, int mode);
SpecKernelFn wide_pipe_kernel_r4(int K, int mode);

inline SpecKernelFn wide_pipe_kernel(int K, int R, int mode) {
  switch (R) {
    case 1: return wide_pipe_kernel_r1(K, mode);
    case 2: return wide_pipe_kernel_r2(K, mode);
    case 3: return wide_pipe_kernel_r3(K, mode);
    case 4: return wide_pipe_kernel_r4(K, mode);
    default: return nullptr;
  }
}

}  // namespace ecgpu
