#!/bin/bash
# Round-5 step-level stride A/B at the headline sizes (after the fine sweep
# found 3-9 KiB flat within ~1 % at 4 MiB): encode + decode{0} plans through
# the library on slabs at the library's skew (+6 KiB at 4 MiB, +8 KiB at 16 MiB)
# and at its neighbours, interleaved rounds.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05o
mkdir -p $O
timeout -k 10 300 python3 -u tools/probe_small_stride.py --sizes 4096 --shapes '10,4' --skews 3,4,5,7,9 --gib 5.25 --rounds 7 > $O/step_4m.jsonl 2> $O/step_4m.err
timeout -k 10 300 python3 -u tools/probe_small_stride.py --sizes 16384 --shapes '12,4' --skews 7,9,24 --gib 6 --rounds 7 > $O/step_16m.jsonl 2> $O/step_16m.err
echo session_ok
