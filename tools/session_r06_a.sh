#!/bin/bash
# Round 6, first call on the new runtime (CPU executor for small host-memory
# calls, knob-only test injection, widened fallback window, sticky-error
# fixes, ECGPU_PIPE_ZC): the GPU suite, then the CPU/GPU crossover per call shape, the drop-in latencies in both
# modes and the CPU executor's rate on the box's host; then
# the two-process e2e probe and the bench line (tools/session_r06_b.sh).
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06a
mkdir -p $O
lscpu > $O/lscpu.txt 2>&1 || true
# the GPU suite first (67 s in round 5): test failures (rc 1) are recorded and
# the measurements still run; a crash, abort or time limit ends the call
rc=0
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.txt 2>&1 || rc=$?
tail -3 $O/gputest.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ]
timeout -k 10 420 ./tools/crossover.bin > $O/crossover.jsonl 2> $O/crossover.err
timeout -k 10 200 ./tools/dropin_latency.bin > $O/dropin_latency.jsonl 2> $O/dropin_latency.err
timeout -k 10 150 python3 tools/cpu_exec_rate.py > $O/cpu_exec_rate.json 2> $O/cpu_exec_rate.err
echo crossover_ok
bash tools/session_r06_b.sh
