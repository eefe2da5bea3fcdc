#!/bin/bash
# Round-5 skew sweep of the other schemes at the mid sizes: the round-3 table
# (512 KiB - 4 MiB) was chosen on RS(10,4) (plus RS(6,3) at 1 MiB); the small-
# shard sweep showed the best skew can depend on k + m.  RS(4,2) / RS(6,3) /
# RS(12,4), ~5 GiB per launch, every skew's slab interleaved in one process.
# Output: gpurun_out/r05l/skew_mid.jsonl
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05l
mkdir -p $O
out=$O/skew_mid.jsonl
: > $out
L=./tools/encode_lab.bin
SK=0,2,4,6,8,10,12,14,18
for kib in 512 1024 2048 4096; do
  for km in "4 2" "6 3" "12 4"; do
    set -- $km
    echo "RS($1,$2) $kib KiB" >&2
    timeout -k 10 170 $L --k $1 --m $2 --kib $kib --stripes 0 --skews $SK --rounds 5 --reps 6 >> $out
  done
done
echo session_ok
