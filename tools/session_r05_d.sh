#!/bin/bash
# Round-5 final check on the last library build: the whole -m gpu suite, the
# N = 2 line rehearsed with both ranks on one GPU (per-rank e2e and its
# aggregate), and smoke().  Each step has its own time limit; the chain stops
# at the first failure.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05d
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > $O/gputest.log 2>&1
ECGPU_BENCH_ONE_DEVICE=1 timeout -k 10 400 python3 bench.py --gpus 2 --steps 10 --warmup 2 > $O/bench_rehearsal_n2.json 2> $O/bench_rehearsal_n2.err
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo session_ok
