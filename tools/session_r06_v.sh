#!/bin/bash
# Round 6: the pipelines' D2H by the library's own copy kernel
# (ECGPU_PIPE_D2H_GRID workgroups) instead of HIP's 1-D blit, to take back the
# 2-4 % the 1-D copies give up alone without the 2-D copies' collapse when
# shared: pipeline GPU tests with it on, one and two processes per grid,
# then the N = 2 rehearsal at two grids.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06v
mkdir -p $O
ECGPU_PIPE_D2H_GRID=256 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "pipeline" \
    --timeout 120 --timeout-method thread > $O/gputest_pipeline_d2hk.txt 2>&1
tail -1 $O/gputest_pipeline_d2hk.txt
L=pipe_encode,pipe_decode,pipe_encode_skew,pipe_encode,pipe_decode,pipe_encode_skew
port=29730
for g in 0 64 256 1024; do
  port=$((port + 1))
  timeout -k 10 200 python3 -u tools/e2e_pair.py --world 1 --port $port --tag one_g$g --passes 5 --legs $L \
      --knob ECGPU_PIPE_D2H_GRID=$g >> $O/pair.jsonl 2> $O/one_g$g.err
  port=$((port + 1))
  timeout -k 10 240 python3 -u tools/e2e_pair.py --rank 0 --world 2 --port $port --tag two_g$g --passes 5 --legs $L \
      --knob ECGPU_PIPE_D2H_GRID=$g >> $O/pair.jsonl 2> $O/two_g${g}_0.err & a=$!
  timeout -k 10 240 python3 -u tools/e2e_pair.py --rank 1 --world 2 --port $port --tag two_g$g --passes 5 --legs $L \
      --knob ECGPU_PIPE_D2H_GRID=$g > /dev/null 2> $O/two_g${g}_1.err & b=$!
  ra=0; rb=0
  wait $a || ra=$?
  wait $b || rb=$?
  [ $ra -eq 0 ] && [ $rb -eq 0 ]
done
echo pairs_ok
for g in 256 1024; do
  env ECGPU_BENCH_ONE_DEVICE=1 ECGPU_PIPE_D2H_GRID=$g timeout -k 10 300 python3 -u bench.py --gpus 2 --steps 5 --warmup 2 \
      --cpu-seconds 0 > $O/n2_g$g.json 2> $O/n2_g$g.err
done
echo session_ok
