#!/bin/bash
# Round 6, third call: the GPU suite after the HIP last-error fix; then a
# bisection of the N = 2 rehearsal's e2e encode collapse (26.7-27.3 GiB/s in
# bench.py, 43.5 in tools/e2e_pair.py, with or without the NUMA affinity):
# the bench without its configs block / CPU legs, with a small slab, with the
# zero-copy pipeline; e2e_pair after bench-like kernel work and with the
# bench's host data; then the default N = 1 bench line.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06d
mkdir -p $O
rc=0
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.txt 2>&1 || rc=$?
tail -3 $O/gputest.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ]
r() {  # r <tag> [env...] -- the N = 2 rehearsal with the given environment
  local tag=$1; shift
  env ECGPU_BENCH_ONE_DEVICE=1 "$@" timeout -k 10 300 python3 -u bench.py --gpus 2 --steps 5 --warmup 2 \
      --no-configs --cpu-seconds 0 > $O/n2_$tag.json 2> $O/n2_$tag.err
}
r lean
r lean_zc2 ECGPU_PIPE_ZC=2
r lean_zc1 ECGPU_PIPE_ZC=1
env ECGPU_BENCH_ONE_DEVICE=1 timeout -k 10 300 python3 -u bench.py --gpus 2 --steps 5 --warmup 2 --no-configs \
    --cpu-seconds 0 --stripes 8 > $O/n2_small_slab.json 2> $O/n2_small_slab.err
echo rehearsals_ok
pair() {
  local tag=$1 port=$2; shift 2
  timeout -k 10 240 python3 -u tools/e2e_pair.py --rank 0 --world 2 --port $port --tag $tag "$@" \
      >> $O/pair.jsonl 2> $O/pair_${tag}_0.err & local a=$!
  timeout -k 10 240 python3 -u tools/e2e_pair.py --rank 1 --world 2 --port $port --tag $tag "$@" \
      > /dev/null 2> $O/pair_${tag}_1.err & local b=$!
  local ra=0 rb=0
  wait $a || ra=$?
  wait $b || rb=$?
  [ $ra -eq 0 ] && [ $rb -eq 0 ]
}
pair pre 29641 --legs pipe_encode,pipe_decode,pipe_encode_zc2 --pre 100
pair benchdata 29642 --legs pipe_encode,pipe_decode --bench-data
pair pre_benchdata 29643 --legs pipe_encode,pipe_decode --pre 100 --bench-data --passes 1
echo pairs_ok
timeout -k 10 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err
echo session_ok
