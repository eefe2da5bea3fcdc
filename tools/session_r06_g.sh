#!/bin/bash
# Round 6: host pipelines with contiguous ring slots (ECGPU_PIPE_CONTIG=1: a
# contiguous host stripe moves as one 1-D copy each way) against the skewed
# slots' 2-D copies, one and two processes on the GPU; the N = 2 rehearsal in
# the state that collapsed the 2-D copies (after sharded_c5); the GPU suite;
# the default bench line.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06g
mkdir -p $O
rc=0
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.txt 2>&1 || rc=$?
tail -3 $O/gputest.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ]
L=duplex,pipe_encode,pipe_decode,pipe_encode_skew,pipe_decode_skew,pipe_encode_zc2,pipe_decode_zc2
timeout -k 10 240 python3 -u tools/e2e_pair.py --world 1 --port 29671 --tag one --legs $L > $O/pair.jsonl 2> $O/one.err
timeout -k 10 240 python3 -u tools/e2e_pair.py --rank 0 --world 2 --port 29672 --tag two --legs $L >> $O/pair.jsonl \
    2> $O/two_0.err & a=$!
timeout -k 10 240 python3 -u tools/e2e_pair.py --rank 1 --world 2 --port 29672 --tag two --legs $L > /dev/null \
    2> $O/two_1.err & b=$!
ra=0; rb=0
wait $a || ra=$?
wait $b || rb=$?
[ $ra -eq 0 ] && [ $rb -eq 0 ]
echo pairs_ok
env ECGPU_BENCH_ONE_DEVICE=1 timeout -k 10 300 python3 -u bench.py --gpus 2 --steps 5 --warmup 2 --cpu-seconds 0 \
    > $O/n2_full.json 2> $O/n2_full.err
env ECGPU_BENCH_ONE_DEVICE=1 ECGPU_PIPE_CONTIG=0 timeout -k 10 300 python3 -u bench.py --gpus 2 --steps 5 --warmup 2 \
    --cpu-seconds 0 > $O/n2_full_skew.json 2> $O/n2_full_skew.err
echo rehearsals_ok
timeout -k 10 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err
echo session_ok
