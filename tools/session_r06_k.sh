#!/bin/bash
# Round 6: the small-call crossover when the CPU executor runs without GFNI --
# the AVX2 nibble path (ECGPU_CPU_SIMD=1, full grid) and scalar (0, quick
# sizes) -- so the default threshold can follow the host's SIMD level.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06k
mkdir -p $O
ECGPU_CPU_SIMD=1 timeout -k 10 500 ./tools/crossover.bin > $O/crossover_avx2.jsonl 2> $O/crossover_avx2.err
echo avx2_ok
ECGPU_CPU_SIMD=0 timeout -k 10 500 ./tools/crossover.bin --quick > $O/crossover_scalar.jsonl 2> $O/crossover_scalar.err
echo session_ok
