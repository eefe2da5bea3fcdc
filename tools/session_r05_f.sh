#!/bin/bash
# Round-5 R = 1 levers (tools/encode_lab.hip --sched 2) on the lost-parity
# re-encode (row 2 of RS(10,4), 4 MiB x 96) and on RS(10,1) all-ones-column
# encode: two columns per lane, the persistent double-buffered form, the LDS
# engine, residency 2 -- against production at the library's cap.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05f
mkdir -p $O
L=./tools/encode_lab.bin
timeout -k 10 200 $L --sched 2 --k 10 --m 1 --lost 1 --rounds 7 --reps 10 > $O/lost_parity.txt 2>&1
timeout -k 10 200 $L --sched 2 --k 6 --m 1 --lost 1 --mib 1 --stripes 512 --rounds 7 --reps 10 > $O/lost_parity_6.txt 2>&1
echo session_ok
