#!/bin/bash
# Round 6: the driver's round-end steps rehearsed on the final tree --
# pytest -m gpu, smoke(), the default bench line -- plus the drop-in latency
# table with the per-level threshold default.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06u
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.txt 2>&1
tail -2 $O/gputest.txt
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
tail -1 $O/smoke.txt
timeout -k 10 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 200 ./tools/dropin_latency.bin > $O/dropin_latency.jsonl 2> $O/dropin_latency.err
echo session_ok
