#!/bin/bash
# Round-5 small-shard skew sweep, part 3: the tiniest shards (4 and 8 KiB),
# 65,535 stripes per launch (the grid's y limit), every skew's slab
# interleaved in one process.  Output: gpurun_out/r05j/skew_tiny.jsonl
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05j
mkdir -p $O
out=$O/skew_tiny.jsonl
: > $out
L=./tools/encode_lab.bin
SK=0,2,4,6,8,10,12
for kib in 4 8; do
  for km in "4 2" "6 3" "10 4"; do
    set -- $km
    echo "RS($1,$2) $kib KiB" >&2
    timeout -k 10 170 $L --k $1 --m $2 --kib $kib --stripes 65535 --skews $SK --rounds 5 --reps 6 >> $out
  done
done
echo session_ok
