#!/bin/bash
# Round 6: device -> pinned D2H on an SDMA engine (below HIP) against HIP's
# blit-kernel D2H, alone and beside the encode pipeline's H2D.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06aa
mkdir -p $O
timeout -k 10 120 ./tools/sdma_d2h_probe.bin > $O/sdma_d2h.jsonl 2> $O/sdma_d2h.err
echo session_ok
