#!/bin/bash
# Round-6 profile pass on the final tree (w = 8 kernels unchanged, build
# 4f58ba055f334a19; host paths of round 6): kernel trace + stats and the two
# PMC passes of the default bench command, the summary, and the bench line
# reading this box's counters (tools/profile_round.sh), so the round-6 line has
# a round-6 rocprof record.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06w
bash tools/profile_round.sh r06 > gpurun_out/r06w/profile_r06.log 2>&1
# the raw traces exceed what gpurun copies back (64 MiB): keep the summaries
cp gpurun_out/bench.json gpurun_out/bench.err gpurun_out/summary.log gpurun_out/r06_rocprof_summary.json \
   gpurun_out/r06_kernel_stats.csv gpurun_out/pmc_encode.json gpurun_out/pmc_decode.json gpurun_out/r06w/
for d in prof_trace prof_fetch prof_write; do
  f=$(find gpurun_out/$d -name '*kernel_stats.csv' -print -quit); [ -n "$f" ] && cp "$f" gpurun_out/r06w/$d.kernel_stats.csv
done
rm -rf gpurun_out/prof_trace gpurun_out/prof_fetch gpurun_out/prof_write
echo session_ok
