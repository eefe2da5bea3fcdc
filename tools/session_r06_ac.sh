#!/bin/bash
# Round 6: the per-launch encode times of the driver's 20-step window, twice.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06ac
mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-configs --e2e-stripes 0 --cpu-seconds 0 \
    > $O/bench_$i.json 2> $O/bench_$i.err
done
echo session_ok
