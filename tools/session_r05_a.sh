#!/bin/bash
# Round-5 first GPU pass on the new build: the whole -m gpu suite (CPU
# fallback, device list, engine-knob plan cache, N > 1 e2e rehearsal
# included), the default bench line and smoke().  Each step has its own time
# limit; the chain stops at the first failure.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05a
timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > gpurun_out/r05a/gputest.log 2>&1
timeout -k 10 300 python3 bench.py > gpurun_out/r05a/bench.json 2> gpurun_out/r05a/bench.err
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05a/smoke.log 2>&1
echo session_ok
