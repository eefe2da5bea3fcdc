#!/bin/bash
# Round-5 N = 2 rehearsal on the final bench (C1's shape in the configs block,
# the scheme-aware stride): both ranks on the one GPU, then smoke().
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05p
mkdir -p $O
ECGPU_BENCH_ONE_DEVICE=1 timeout -k 10 400 python3 bench.py --gpus 2 --steps 10 --warmup 2 > $O/bench_rehearsal_n2.json 2> $O/bench_rehearsal_n2.err
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo session_ok
