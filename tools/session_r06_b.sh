#!/bin/bash
# Round 6, VERDICT r5 next #3: the two-process e2e encode collapse.  The raw
# copies and the pipelines (DMA, and the ECGPU_PIPE_ZC kernel-in-place forms)
# with one process, then two processes on cuda:0
# (each timed pass barrier-started), then the same two-process encode and
# duplex legs under rocprofv3 --kernel-trace --memory-copy-trace (one process
# each, no counters), summarised by tools/copy_overlap.py;
# then the default bench line.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06b
mkdir -p $O
pair() {  # pair <tag> <port> <legs> [extra args]: two ranks, wait for both
  local tag=$1 port=$2 legs=$3; shift 3
  timeout -k 10 240 python3 -u tools/e2e_pair.py --rank 0 --world 2 --port $port --legs $legs --tag $tag "$@" \
      >> $O/pair.jsonl 2> $O/pair_${tag}_0.err & local a=$!
  timeout -k 10 240 python3 -u tools/e2e_pair.py --rank 1 --world 2 --port $port --legs $legs --tag $tag "$@" \
      > /dev/null 2> $O/pair_${tag}_1.err & local b=$!
  local ra=0 rb=0
  wait $a || ra=$?
  wait $b || rb=$?
  [ $ra -eq 0 ] && [ $rb -eq 0 ]
}
timeout -k 10 240 python3 -u tools/e2e_pair.py --world 1 --port 29611 --tag one --legs h2d,d2h,duplex,pipe_encode,pipe_decode,pipe_encode_zc1,pipe_encode_zc2,pipe_decode_zc1,pipe_decode_zc2 \
    > $O/pair.jsonl 2> $O/one.err
pair two 29612 h2d,d2h,duplex,pipe_encode,pipe_decode,pipe_encode_zc1,pipe_encode_zc2,pipe_decode_zc1,pipe_decode_zc2
pair two_depth2 29613 pipe_encode,pipe_encode_zc1 --depth 2
pair two_depth6 29614 pipe_encode,pipe_encode_zc1 --depth 6
echo rates_ok
port=29620
for leg in pipe_encode duplex pipe_encode_zc1 pipe_encode_zc2; do
  port=$((port + 1))
  P=$O/prof_$leg
  timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $P/r0 -o r0 -- \
      python3 -u tools/e2e_pair.py --rank 0 --world 2 --port $port --legs $leg --passes 2 --tag prof \
      > $O/prof_${leg}.jsonl 2> $O/prof_${leg}_0.err & a=$!
  timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $P/r1 -o r1 -- \
      python3 -u tools/e2e_pair.py --rank 1 --world 2 --port $port --legs $leg --passes 2 --tag prof \
      > /dev/null 2> $O/prof_${leg}_1.err & b=$!
  ra=0; rb=0
  wait $a || ra=$?
  wait $b || rb=$?
  [ $ra -eq 0 ] && [ $rb -eq 0 ]
  python3 tools/copy_overlap.py $P/r0 $P/r1 > $O/overlap_${leg}.json
done
# one process, the same traces, for the alone rates
P=$O/prof_one
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $P/r0 -o r0 -- \
    python3 -u tools/e2e_pair.py --world 1 --port 29631 --legs duplex,pipe_encode --passes 2 --tag prof_one \
    > $O/prof_one.jsonl 2> $O/prof_one.err
python3 tools/copy_overlap.py $P/r0 > $O/overlap_one.json
# the default bench line on this tree (w = 8 kernel build unchanged: no new profile pass)
timeout -k 10 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err
echo session_ok
