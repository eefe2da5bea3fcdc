#!/bin/bash
# Round 6: the pipelines' D2H on an SDMA engine (ECGPU_D2H_NOCU=1: the flat
# device -> pinned copies as hipMemcpyDeviceToDeviceNoCU) against HIP's blit
# kernel: the pipeline GPU tests with it on, one and two processes, and one
# traced two-process pass to see which engine ran the copies.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06m
mkdir -p $O
ECGPU_D2H_NOCU=1 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "pipeline" \
    --timeout 120 --timeout-method thread > $O/gputest_pipeline_nocu.txt 2>&1
tail -1 $O/gputest_pipeline_nocu.txt
L=pipe_encode,pipe_decode,pipe_encode_skew,pipe_encode,pipe_decode,pipe_encode_skew
port=29710
for v in 0 1; do
  port=$((port + 1))
  timeout -k 10 200 python3 -u tools/e2e_pair.py --world 1 --port $port --tag one_nocu$v --passes 5 --legs $L \
      --knob ECGPU_D2H_NOCU=$v >> $O/pair.jsonl 2> $O/one_nocu$v.err
  port=$((port + 1))
  timeout -k 10 240 python3 -u tools/e2e_pair.py --rank 0 --world 2 --port $port --tag two_nocu$v --passes 5 --legs $L \
      --knob ECGPU_D2H_NOCU=$v >> $O/pair.jsonl 2> $O/two_nocu${v}_0.err & a=$!
  timeout -k 10 240 python3 -u tools/e2e_pair.py --rank 1 --world 2 --port $port --tag two_nocu$v --passes 5 --legs $L \
      --knob ECGPU_D2H_NOCU=$v > /dev/null 2> $O/two_nocu${v}_1.err & b=$!
  ra=0; rb=0
  wait $a || ra=$?
  wait $b || rb=$?
  [ $ra -eq 0 ] && [ $rb -eq 0 ]
done
echo pairs_ok
P=$O/prof_nocu
port=$((port + 1))
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $P/r0 -o r0 -- \
    python3 -u tools/e2e_pair.py --rank 0 --world 2 --port $port --legs pipe_encode --passes 2 --tag prof_nocu \
    --knob ECGPU_D2H_NOCU=1 > $O/prof_nocu.jsonl 2> $O/prof_nocu_0.err & a=$!
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $P/r1 -o r1 -- \
    python3 -u tools/e2e_pair.py --rank 1 --world 2 --port $port --legs pipe_encode --passes 2 --tag prof_nocu \
    --knob ECGPU_D2H_NOCU=1 > /dev/null 2> $O/prof_nocu_1.err & b=$!
ra=0; rb=0
wait $a || ra=$?
wait $b || rb=$?
[ $ra -eq 0 ] && [ $rb -eq 0 ]
echo session_ok
