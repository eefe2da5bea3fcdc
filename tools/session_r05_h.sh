#!/bin/bash
# Round-5 small-shard skew sweep, part 2 (after r05g found no skew best at
# 64 / 128 KiB): 16, 32, 96, 192, 256 KiB and the ECX block size (~341 KiB)
# at RS(4,2) / RS(6,3) / RS(10,4), ~5 GiB per launch, every skew's slab
# interleaved in one process.  Output: gpurun_out/r05h/skew_small2.jsonl
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05h
mkdir -p $O
out=$O/skew_small2.jsonl
: > $out
L=./tools/encode_lab.bin
SK=0,2,4,6,8,10,12,14,18
for kib in 16 32 96 192 256 341; do
  for km in "4 2" "6 3" "10 4"; do
    set -- $km
    echo "RS($1,$2) $kib KiB" >&2
    timeout -k 10 170 $L --k $1 --m $2 --kib $kib --stripes 0 --skews $SK --rounds 5 --reps 6 >> $out
  done
done
echo session_ok
