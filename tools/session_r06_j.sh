#!/bin/bash
# Round 6: where the contiguous-slot pipeline's single-process encode loses
# its ~3 % to the skewed slots' 2-D copies: the same legs with every shard
# copied on its own (ECGPU_PIPE_2D=0) and as runs, one and two processes,
# legs interleaved, 5 passes each, twice.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06j
mkdir -p $O
L=pipe_encode,pipe_encode_skew,pipe_decode,pipe_decode_skew
L=$L,$L
port=29700
for v in 1 0; do
  port=$((port + 1))
  timeout -k 10 200 python3 -u tools/e2e_pair.py --world 1 --port $port --tag one_2d$v --passes 5 --legs $L \
      --knob ECGPU_PIPE_2D=$v >> $O/pair.jsonl 2> $O/one_2d$v.err
  port=$((port + 1))
  timeout -k 10 240 python3 -u tools/e2e_pair.py --rank 0 --world 2 --port $port --tag two_2d$v --passes 5 --legs $L \
      --knob ECGPU_PIPE_2D=$v >> $O/pair.jsonl 2> $O/two_2d${v}_0.err & a=$!
  timeout -k 10 240 python3 -u tools/e2e_pair.py --rank 1 --world 2 --port $port --tag two_2d$v --passes 5 --legs $L \
      --knob ECGPU_PIPE_2D=$v > /dev/null 2> $O/two_2d${v}_1.err & b=$!
  ra=0; rb=0
  wait $a || ra=$?
  wait $b || rb=$?
  [ $ra -eq 0 ] && [ $rb -eq 0 ]
done
echo session_ok
