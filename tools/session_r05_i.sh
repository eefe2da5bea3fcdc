#!/bin/bash
# Round-5 small-shard stride change (shard_stride.hpp kNoSkewUpTo): the -m gpu
# suite on the new layout, the library-path A/B of the new stride against the
# old +10 KiB (tools/probe_small_stride.py), and the default bench line (which
# now carries C1's shape device-resident).
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05i
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > $O/gputest.log 2>&1
timeout -k 10 400 python3 -u tools/probe_small_stride.py > $O/small_stride.jsonl 2> $O/small_stride.err
timeout -k 10 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err
echo session_ok
