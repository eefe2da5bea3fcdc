#!/bin/bash
# Round-5 small-shard skew sweep (tools/encode_lab.hip --skews): the shard
# sizes below the round-3 sweep's 256 KiB -- C1's RS(4,2) 64 KiB and the
# same sizes at RS(6,3) / RS(10,4) -- ~5 GiB per launch, every skew's slab
# interleaved in one process.  Output: gpurun_out/r05g/skew_small.jsonl
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05g
mkdir -p $O
out=$O/skew_small.jsonl
: > $out
L=./tools/encode_lab.bin
SK=0,2,4,6,8,10,12,14,18
for km in "4 2" "6 3" "10 4"; do
  set -- $km
  for kib in 64 128; do
    echo "RS($1,$2) $kib KiB" >&2
    timeout -k 10 240 $L --k $1 --m $2 --kib $kib --stripes 0 --skews $SK --rounds 5 --reps 6 >> $out
  done
done
echo session_ok
