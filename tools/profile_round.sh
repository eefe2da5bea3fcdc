#!/bin/bash
# Full measurement pass on the GPU box (run under gpurun from the repo root):
#   rocprofv3 kernel trace + stats of the default bench command, two separate
#   PMC passes (FETCH_SIZE, WRITE_SIZE) of the same command, the summary into
#   profiles/, then the bench again so its roofline.traffic comes from this
#   box's counters.
#   bash tools/profile_round.sh r02
set -e
TAG=${1:-r02}
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_trace -o run -- python3 bench.py > $O/prof_trace.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof_fetch -o run -- python3 bench.py > $O/prof_fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof_write -o run -- python3 bench.py > $O/prof_write.log 2>&1
for d in prof_trace prof_fetch prof_write; do
  f=$(find $O/$d -name 'run_*.csv' -print -quit); dd=$(dirname "$f"); [ "$dd" = "$O/$d" ] || cp "$dd"/run_*.csv $O/$d/
done
python3 profiles/summarize.py --tag $TAG --trace $O/prof_trace --fetch $O/prof_fetch --write $O/prof_write > $O/summary.log
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err
cp profiles/${TAG}_rocprof_summary.json profiles/${TAG}_kernel_stats.csv profiles/pmc_encode.json profiles/pmc_decode.json $O/
