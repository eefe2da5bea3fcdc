#!/bin/bash
# Round 6: the driver's round-end steps on the final tree (the library rebuilt after the
# closed D2H-on-compute experiment, same sources and build ID) -- pytest -m gpu, smoke(),
# the bench as the driver runs it.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06ae
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.txt 2>&1
tail -2 $O/gputest.txt
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
tail -1 $O/smoke.txt
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
echo session_ok
