#!/bin/bash
# Round 6: sustained rate -- the bench's timed step over 20 / 500 / 5,000
# steps (0.03 / 0.8 / 8 s of back-to-back encode + decode), configs block,
# e2e and CPU baseline off, to show the 20-step value is not a burst figure.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06z
mkdir -p $O
for s in 20 500 5000; do
  timeout -k 10 300 python3 -u bench.py --steps $s --warmup 5 --no-configs --e2e-stripes 0 --cpu-seconds 0 \
    > $O/bench_steps$s.json 2> $O/bench_steps$s.err
done
echo session_ok
