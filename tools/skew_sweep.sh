#!/bin/bash
# Shard-stride skew sweep, RS(10,4), ~5 GiB per launch, one process per shard
# size with every skew's slab interleaved in it (tools/encode_lab.hip --skews).
# Output: gpurun_out/skew_sweep_<tag>.jsonl
set -e
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:-a}
mkdir -p gpurun_out
out=gpurun_out/skew_sweep_$TAG.jsonl
: > $out
for kib in 256 512 1024 2048 3072 4096 6144 8192 12288 16384 32768 65536; do
  timeout -k 10 120 ./tools/encode_lab.bin --k 10 --m 4 --kib $kib --stripes 0 --skews 0,2,6,8,10,12,14,18 --rounds 5 --reps 6 >> $out
done
