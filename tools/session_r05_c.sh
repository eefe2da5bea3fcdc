#!/bin/bash
# Round-5 host-path session: every host-memory path (tools/bench_e2e.py), the
# C++ drop-in latency table (both after the runtime's failure-contract and
# device-list changes), the CPU fallback's rate on this host's cores
# (injected sticky error: every call on the CPU), and the GPU tests touched
# since the closing pass (fallback, schedules).  Each step has its own time
# limit; the chain stops at the first failure.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05c
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_cpu_fallback.py tests/test_surface_cpu.py -k "fallback or schedule or split" > $O/gputest.log 2>&1
timeout -k 10 300 python3 tools/bench_e2e.py > $O/e2e.json 2> $O/e2e.err
timeout -k 10 300 ./tools/dropin_latency.bin > $O/dropin_latency.jsonl 2> $O/dropin_latency.err
ECGPU_CPU_FALLBACK=1 ECGPU_TEST_INJECT_HIP=2 timeout -k 10 120 python3 tools/fallback_rate.py > $O/fallback_rate.json 2> $O/fallback_rate.err
echo session_ok
