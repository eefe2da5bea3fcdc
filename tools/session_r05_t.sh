#!/bin/bash
# Round-5 driver rehearsal on the final tree: smoke() and the default bench
# line, as the round-end driver runs them.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05t
mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err
echo session_ok
