#!/bin/bash
# Round 6: after the decoding-matrix cache (and the host-side overhead cuts: static GF(2^8) tables,
# allocation-free planner ops): the GPU suite, the fixed host cost per
# CPU-routed call (tools/host_overhead.cpp), the drop-in latency table, the
# default bench line.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06q
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.txt 2>&1
tail -1 $O/gputest.txt
timeout -k 10 120 ./tools/host_overhead.bin > $O/host_overhead.jsonl 2> $O/host_overhead.err
timeout -k 10 200 ./tools/dropin_latency.bin > $O/dropin_latency.jsonl 2> $O/dropin_latency.err
timeout -k 10 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err
echo session_ok
