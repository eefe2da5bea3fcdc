#!/bin/bash
# Round 6: A/B of ECGPU_PIPE_D2H_COMP (a stripe's D2H queued on the compute
# stream behind its launch) against the default and against 2-D copies
# (ECGPU_PIPE_FLAT=0), one process, interleaved three times.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06ad
mkdir -p $O
: > $O/ab.jsonl
for rep in 1 2 3; do
  for v in default comp flat0; do
    case $v in
      default) K="";;
      comp) K="--knob ECGPU_PIPE_D2H_COMP=1";;
      flat0) K="--knob ECGPU_PIPE_FLAT=0";;
    esac
    timeout -k 10 120 python3 -u tools/e2e_pair.py --legs pipe_encode,pipe_decode --passes 5 --port 2961$rep \
      --tag "$v rep$rep" $K >> $O/ab.jsonl 2>> $O/ab.err
  done
done
echo session_ok
