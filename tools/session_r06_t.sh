#!/bin/bash
# Round 6: the link rule (ECGPU_LINK_CALLS=1: a large host-memory call that
# finds another holding the device's link runs on the CPU executor): the GPU
# suite, concurrent callers with the library defaults (and the rule off),
# the single-thread latency table, the default bench line.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06t
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.txt 2>&1
tail -1 $O/gputest.txt
timeout -k 10 200 ./tools/dropin_latency.bin --threads > $O/threads_lib.jsonl 2> $O/threads_lib.err
ECGPU_LINK_CALLS=0 timeout -k 10 200 ./tools/dropin_latency.bin --threads > $O/threads_nolink.jsonl 2> $O/threads_nolink.err
timeout -k 10 200 ./tools/dropin_latency.bin > $O/dropin_latency.jsonl 2> $O/dropin_latency.err
timeout -k 10 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err
echo session_ok
