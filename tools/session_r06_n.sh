#!/bin/bash
# Round 6: every host-memory path on the final runtime (tools/bench_e2e.py, as
# r05_e2e.json), with the contiguous pipeline slots and, for the pipelines,
# with ECGPU_PIPE_CONTIG=0 beside it; the GPU suite on this tree first.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06n
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.txt 2>&1
tail -1 $O/gputest.txt
timeout -k 10 500 python3 -u tools/bench_e2e.py --parts pcie,pcie_duplex,e2e_pipeline_pinned,e2e_pipeline_pageable,e2e_read_pipeline_1,e2e_read_pipeline_4,dropin_pageable,dropin_pinned,ecx_accum,call_latency,pipeline_depth \
    > $O/e2e.json 2> $O/e2e.err
ECGPU_PIPE_CONTIG=0 timeout -k 10 300 python3 -u tools/bench_e2e.py --parts e2e_pipeline_pinned,e2e_pipeline_pageable,e2e_read_pipeline_1,e2e_read_pipeline_4 \
    > $O/e2e_skew.json 2> $O/e2e_skew.err
echo session_ok
