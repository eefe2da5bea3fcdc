#!/bin/bash
# Round 6: the pipeline default, decided on repeats -- DMA into contiguous
# slots (1-D copies), DMA into skewed slots (2-D, round 5), zero-copy
# (ECGPU_PIPE_ZC=2), one and two processes, 5 passes each, the legs
# interleaved twice; then bench.py N = 1 and the N = 2 rehearsal with the
# zero-copy pipelines.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06h
mkdir -p $O
L=pipe_encode,pipe_encode_zc2,pipe_encode_skew,pipe_decode,pipe_decode_zc2,pipe_decode_skew
L2=$L,$L
timeout -k 10 300 python3 -u tools/e2e_pair.py --world 1 --port 29681 --tag one --passes 5 --legs $L2 > $O/pair.jsonl 2> $O/one.err
timeout -k 10 300 python3 -u tools/e2e_pair.py --rank 0 --world 2 --port 29682 --tag two --passes 5 --legs $L2 >> $O/pair.jsonl \
    2> $O/two_0.err & a=$!
timeout -k 10 300 python3 -u tools/e2e_pair.py --rank 1 --world 2 --port 29682 --tag two --passes 5 --legs $L2 > /dev/null \
    2> $O/two_1.err & b=$!
ra=0; rb=0
wait $a || ra=$?
wait $b || rb=$?
[ $ra -eq 0 ] && [ $rb -eq 0 ]
echo pairs_ok
ECGPU_PIPE_ZC=2 timeout -k 10 400 python3 -u bench.py --cpu-seconds 0 > $O/bench_zc2.json 2> $O/bench_zc2.err
env ECGPU_BENCH_ONE_DEVICE=1 ECGPU_PIPE_ZC=2 timeout -k 10 300 python3 -u bench.py --gpus 2 --steps 5 --warmup 2 \
    --cpu-seconds 0 > $O/n2_full_zc2.json 2> $O/n2_full_zc2.err
echo session_ok
