#!/bin/bash
# Round 6: bisection of the N = 2 e2e encode collapse, part 3.  Session E
# put it on bench.py's sharded_c5 leg (configs alone: 43.8 GiB/s; C5 alone:
# 27.2) and showed it persists over repeated passes, and that the zero-copy
# pipeline avoids it (46.3).  Here: sharded_c5's work reproduced inside
# tools/e2e_pair.py; an HBM alloc / free churn instead; per-shard 1-D copies
# (ECGPU_PIPE_2D=0) in the collapsed state, in the pair and in the bench;
# then both states under rocprofv3 --kernel-trace --memory-copy-trace with
# the 1-D copies, so every copy is in the trace.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06f
mkdir -p $O
pair() {  # pair <tag> <port> [env assignments --] args...
  local tag=$1 port=$2; shift 2
  timeout -k 10 240 env $ENVS python3 -u tools/e2e_pair.py --rank 0 --world 2 --port $port --tag $tag "$@" \
      >> $O/pair.jsonl 2> $O/pair_${tag}_0.err & local a=$!
  timeout -k 10 240 env $ENVS python3 -u tools/e2e_pair.py --rank 1 --world 2 --port $port --tag $tag "$@" \
      > /dev/null 2> $O/pair_${tag}_1.err & local b=$!
  local ra=0 rb=0
  wait $a || ra=$?
  wait $b || rb=$?
  [ $ra -eq 0 ] && [ $rb -eq 0 ]
}
ENVS="ECGPU_PIPE_2D=1"
pair c5 29651 --legs pipe_encode,pipe_decode,pipe_encode_zc2,pipe_encode_zc1 --c5
pair churn6 29652 --legs pipe_encode,pipe_decode --churn-gib 6
ENVS="ECGPU_PIPE_2D=0"
pair c5_1d 29653 --legs pipe_encode,pipe_decode --c5
pair fresh_1d 29654 --legs pipe_encode,pipe_decode
echo pairs_ok
env ECGPU_BENCH_ONE_DEVICE=1 ECGPU_BENCH_SKIP=configs ECGPU_PIPE_2D=0 timeout -k 10 300 python3 -u bench.py --gpus 2 \
    --steps 5 --warmup 2 --cpu-seconds 0 > $O/n2_skip_configs_1d.json 2> $O/n2_skip_configs_1d.err
echo bench_ok
port=29660
for state in fresh c5; do
  port=$((port + 1))
  extra=""
  [ $state = c5 ] && extra="--c5"
  P=$O/prof_$state
  ECGPU_PIPE_2D=0 timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $P/r0 -o r0 -- \
      python3 -u tools/e2e_pair.py --rank 0 --world 2 --port $port --legs pipe_encode --passes 2 --tag prof_$state $extra \
      > $O/prof_$state.jsonl 2> $O/prof_${state}_0.err & a=$!
  ECGPU_PIPE_2D=0 timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $P/r1 -o r1 -- \
      python3 -u tools/e2e_pair.py --rank 1 --world 2 --port $port --legs pipe_encode --passes 2 --tag prof_$state $extra \
      > /dev/null 2> $O/prof_${state}_1.err & b=$!
  ra=0; rb=0
  wait $a || ra=$?
  wait $b || rb=$?
  [ $ra -eq 0 ] && [ $rb -eq 0 ]
  python3 tools/copy_overlap.py $P/r0 $P/r1 --h2d-bytes $((4 << 20)) --d2h-bytes $((4 << 20)) > $O/overlap_$state.json
done
echo session_ok
