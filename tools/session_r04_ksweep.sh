#!/bin/bash
# Round-4 re-check: the w = 32 pipelined-form rule (K = 7..10) at the library's
# shard stride (the round-3 sweep used a fixed +10 KiB), and the pageable host
# pipeline measured three times beside the pinned one.  Every step has its own
# time limit; the chain stops at the first failure.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
: > $O/r04_wide_lab_k7_10.jsonl
for k in 7 8 9 10; do
  timeout -k 10 180 ./tools/wide_lab.bin --w 32 --k $k --rounds 7 --only prod_u1,prod_pipe >> $O/r04_wide_lab_k7_10.jsonl 2>> $O/r04_wide_lab_k7_10.err
done
: > $O/r04_e2e_pageable_repeat.txt
for i in 1 2 3; do
  timeout -k 10 240 python3 tools/bench_e2e.py --parts e2e_pipeline_pinned,e2e_pipeline_pageable >> $O/r04_e2e_pageable_repeat.txt 2>> $O/r04_e2e_pageable_repeat.err
done
echo session_ok
