#!/bin/bash
# Round 6: the N = 2 bench rehearsal test with the mean-launch roofline check.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06ab
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests/test_multirank_gpu.py -m gpu -x -v --timeout 450 --timeout-method thread \
  -k bench_gpus2 > $O/test.txt 2>&1
tail -3 $O/test.txt
echo session_ok
