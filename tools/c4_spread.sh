#!/bin/bash
# C4 launch-to-launch spread: one kernel trace of the
# bench's own command (its configs block holds C4's 25 launches), then two PMC
# passes of the same command, each with --kernel-trace so every counter row
# has its dispatch's duration, then an in-process residency A/B of C4 beside
# the C3 encode.  One counter group per rocprofv3 run (MI355X_MICROARCH.md).
#   python tools/c4_spread.py gpurun_out/c4 > profiles/r05_c4_spread.json
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c4
BCMD="python3 bench.py --cpu-seconds 0 --e2e-stripes 0"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c4/trace -o run -- $BCMD > gpurun_out/c4/trace.log 2>&1
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/c4/pmc_sq -o run -- $BCMD > gpurun_out/c4/pmc_sq.log 2>&1
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/c4/pmc_tcc -o run -- $BCMD > gpurun_out/c4/pmc_tcc.log 2>&1
timeout -k 10 300 python3 tools/probe_dense.py --shapes C4_decode_0123,C3_encode --variants default,bpcu6_always,bpcu5_always,bpcu4_always,cap_never --rounds 6 --reps 10 --tag r05_c4_cap > gpurun_out/c4/ab.jsonl 2> gpurun_out/c4/ab.err
