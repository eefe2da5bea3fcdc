#!/bin/bash
# Round-5 scheme-aware stride (ecgpu_recommended_shard_stride_km): the -m gpu
# suite, the library-path A/B at 256 / 512 KiB for four schemes against the
# round-4 table (RS(10,4) has the same layout in both: the noise check), and
# the default bench line.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05m
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > $O/gputest.log 2>&1
timeout -k 10 400 python3 -u tools/probe_small_stride.py --sizes 256,512 --shapes '4,2;6,3;10,4;12,4' > $O/stride_km.jsonl 2> $O/stride_km.err
timeout -k 10 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err
echo session_ok
