#!/bin/bash
# Round-5 scheduling A/B (tools/encode_lab.hip --sched 1): the production
# gf_apply against lab::enc_sb (every source load issued before the
# arithmetic) on the C3 encode, the lost-parity re-encode, C2 and a dense
# C4-like map, each at the library's cap, one more, and uncapped.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05e
mkdir -p $O
L=./tools/encode_lab.bin
timeout -k 10 150 $L --sched 1 --k 10 --m 4 --rounds 7 --reps 10 > $O/c3_encode.txt 2>&1
timeout -k 10 150 $L --sched 1 --k 10 --m 1 --lost 1 --rounds 7 --reps 10 > $O/lost_parity.txt 2>&1
timeout -k 10 150 $L --sched 1 --k 6 --m 3 --mib 1 --stripes 512 --rounds 7 --reps 10 > $O/c2_encode.txt 2>&1
timeout -k 10 150 $L --sched 1 --dense 1 --k 10 --m 4 --rounds 7 --reps 10 > $O/dense.txt 2>&1
echo session_ok
