#!/bin/bash
# Round 6: bisection of the N = 2 rehearsal's e2e encode collapse, part 2.
# Without the configs block and C5 leg the two ranks' encode pipelines share
# the link at 44.3 GiB/s (session D); with them, 26.7-27.3.  Here: the full
# rehearsal with the e2e leg repeated (transient or persistent), with the
# zero-copy pipeline, and with only one of the two blocks.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06e
mkdir -p $O
r() {  # r <tag> [env...]
  local tag=$1; shift
  env ECGPU_BENCH_ONE_DEVICE=1 "$@" timeout -k 10 300 python3 -u bench.py --gpus 2 --steps 5 --warmup 2 \
      --cpu-seconds 0 > $O/n2_$tag.json 2> $O/n2_$tag.err
  echo "$tag done"
}
r full_repeat ECGPU_BENCH_E2E_REPEAT=3
r full_zc2 ECGPU_PIPE_ZC=2 ECGPU_BENCH_E2E_REPEAT=2
r skip_c5 ECGPU_BENCH_SKIP=c5
r skip_configs ECGPU_BENCH_SKIP=configs
echo session_ok
