#!/bin/bash
# Round-5 fine / large skew sweep at the headline sizes: the round-3 sweep
# tried even KiB skews 0-18 only.  256-B to 64-KiB skews for RS(10,4) 4 MiB
# (the timed step) and RS(12,4) 16 MiB (C5), ~5 GiB per launch, every skew's
# slab interleaved in one process.  Output: gpurun_out/r05n/skew_fine.jsonl
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05n
mkdir -p $O
out=$O/skew_fine.jsonl
: > $out
L=./tools/encode_lab.bin
SK=0,1,2,4,6,8,12,16,20,24,28,36,64,96,128,256
echo "RS(10,4) 4 MiB" >&2
timeout -k 10 200 $L --k 10 --m 4 --kib 4096 --stripes 0 --skew-unit 256 --skews $SK --rounds 5 --reps 6 >> $out
echo "RS(12,4) 16 MiB" >&2
timeout -k 10 200 $L --k 12 --m 4 --kib 16384 --stripes 0 --skew-unit 256 --skews $SK --rounds 5 --reps 6 >> $out
echo session_ok
