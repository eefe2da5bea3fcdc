#!/bin/bash
# Round 6, first call on the new runtime (CPU executor for small host-memory
# calls, knob-only test injection, widened fallback window, sticky-error
# fixes): the GPU suite, then the CPU/GPU crossover per call shape, the
# drop-in latencies in both modes and the CPU executor's rate on the box's
# host.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06a
mkdir -p $O
lscpu > $O/lscpu.txt 2>&1 || true
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.txt 2>&1
tail -3 $O/gputest.txt
timeout -k 10 500 ./tools/crossover.bin > $O/crossover.jsonl 2> $O/crossover.err
timeout -k 10 300 ./tools/dropin_latency.bin > $O/dropin_latency.jsonl 2> $O/dropin_latency.err
timeout -k 10 200 python3 tools/cpu_exec_rate.py > $O/cpu_exec_rate.json 2> $O/cpu_exec_rate.err
echo session_ok
