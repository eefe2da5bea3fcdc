#!/bin/bash
# Round-4 closing pass on the GPU box: the whole -m gpu suite, the profile
# pass (kernel trace + PMC + bench, tools/profile_round.sh) on the final
# kernel build, and the bench with the LDS nibble-table engine as the timed
# kernel.  Every step has its own time limit; the chain stops at the first
# failure.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 450 --timeout-method thread tests > gpurun_out/r04_gputest_final.log 2>&1
bash tools/profile_round.sh r04 > gpurun_out/profile_r04_final.log 2>&1
timeout -k 10 200 python3 bench.py --kernel lds > gpurun_out/r04_bench_lds.json 2> gpurun_out/r04_bench_lds.err
echo session_ok
