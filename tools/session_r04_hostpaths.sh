#!/bin/bash
# Round-4 host-path and surface session on the GPU box: every host-memory path
# (bench_e2e), the C++ drop-in latency table, the off-north-star surface calls
# under a kernel trace, and the long fuzz runs (plain 20,000 cases; aliased /
# shifted 3,000).  Each step has its own time limit; the chain stops at the
# first failure.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python3 tools/bench_e2e.py > $O/r04_e2e.json 2> $O/r04_e2e.err
timeout -k 10 300 ./tools/dropin_latency.bin > $O/r04_dropin_latency.jsonl 2> $O/r04_dropin_latency.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/surf -o run -- python3 tools/bench_surface.py > $O/r04_surface.json 2> $O/r04_surface.err
cp $O/surf/run_kernel_stats.csv $O/r04_surface_kernel_stats.csv 2>/dev/null || cp $(find $O/surf -name 'run_kernel_stats.csv' -print -quit) $O/r04_surface_kernel_stats.csv
rm -rf $O/surf
ECGPU_FUZZ_CASES=20000 ECGPU_FUZZ_ALIAS_CASES=3000 timeout -k 10 900 python3 -u -m pytest -x -q -m gpu --timeout 800 --timeout-method thread tests/test_fuzz_gpu.py > $O/r04_fuzz_long.txt 2>&1
echo session_ok
