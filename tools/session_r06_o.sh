#!/bin/bash
# Round 6: the contiguous-slot pipelines give back 4 % alone (pinned) and 13 %
# (pageable) to the skewed slots.  Candidates: the 4-shard D2H as one copy
# per shard (ECGPU_PIPE_D2H_SPLIT=1), flat runs kept on hipMemcpy2DAsync
# (ECGPU_PIPE_FLAT=0); one and two processes, pinned (e2e_pair) and pageable
# (tools/bench_e2e.py), then the N = 2 rehearsal for each.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06o
mkdir -p $O
L=pipe_encode,pipe_decode,pipe_encode_skew,pipe_encode,pipe_decode,pipe_encode_skew
port=29720
for cfg in "base:ECGPU_PIPE_FLAT=1" "split:ECGPU_PIPE_D2H_SPLIT=1" "noflat:ECGPU_PIPE_FLAT=0" "split_noflat:ECGPU_PIPE_D2H_SPLIT=1,ECGPU_PIPE_FLAT=0"; do
  tag=${cfg%%:*}; kv=${cfg#*:}
  KN=""
  for x in ${kv//,/ }; do KN="$KN --knob $x"; done
  port=$((port + 1))
  timeout -k 10 200 python3 -u tools/e2e_pair.py --world 1 --port $port --tag one_$tag --passes 5 --legs $L $KN \
      >> $O/pair.jsonl 2> $O/one_$tag.err
  port=$((port + 1))
  timeout -k 10 240 python3 -u tools/e2e_pair.py --rank 0 --world 2 --port $port --tag two_$tag --passes 5 --legs $L $KN \
      >> $O/pair.jsonl 2> $O/two_${tag}_0.err & a=$!
  timeout -k 10 240 python3 -u tools/e2e_pair.py --rank 1 --world 2 --port $port --tag two_$tag --passes 5 --legs $L $KN \
      > /dev/null 2> $O/two_${tag}_1.err & b=$!
  ra=0; rb=0
  wait $a || ra=$?
  wait $b || rb=$?
  [ $ra -eq 0 ] && [ $rb -eq 0 ]
  env ${kv//,/ } timeout -k 10 200 python3 -u tools/bench_e2e.py --parts e2e_pipeline_pinned,e2e_pipeline_pageable,e2e_read_pipeline_4 \
      > $O/e2e_$tag.json 2> $O/e2e_$tag.err
  echo "$tag ok"
done
for cfg in "split:ECGPU_PIPE_D2H_SPLIT=1" "noflat:ECGPU_PIPE_FLAT=0"; do
  tag=${cfg%%:*}; kv=${cfg#*:}
  env ECGPU_BENCH_ONE_DEVICE=1 $kv timeout -k 10 300 python3 -u bench.py --gpus 2 --steps 5 --warmup 2 --cpu-seconds 0 \
      > $O/n2_$tag.json 2> $O/n2_$tag.err
done
echo session_ok
