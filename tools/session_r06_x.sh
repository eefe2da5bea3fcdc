#!/bin/bash
# Round 6: the default bench line after roofline.achieved moved to the mean
# of the timed encode launches (the contract's average; the median beside it).
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06x
mkdir -p $O
timeout -k 10 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err
echo session_ok
