#!/bin/bash
# PMC passes over tools/probe_dense.py --pmc (C3 encode, decode{0}, the
# lost-parity decode, C4 decode{0,1,2,3}, C2 encode at the bench's sizes), one
# counter group per rocprofv3 run (MI355X_MICROARCH.md: counters are not split
# over passes; at most 8 SQ, 4 TCC, 2 GRBM per pass).  Then a kernel trace of
# the same command.  Output under gpurun_out/pmc_dense_<n>/; summarise with
#   python tools/pmc_summary.py gpurun_out/pmc_dense_* > profiles/r04_pmc_dense.json
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
CMD="python3 tools/probe_dense.py --pmc --rounds 1 --reps 5"
FIRST=${1:-1}  # first pass to run (re-runs of later passes)
timeout -s KILL 60 rocprofv3 -L > gpurun_out/rocprofv3_counters.txt 2>&1 || true
n=0
for c in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_COUNT" \
         "FETCH_SIZE" "WRITE_SIZE" \
         "SQ_INSTS_SMEM SQ_INST_CYCLES_SMEM SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_INST_LEVEL_VMEM GRBM_GUI_ACTIVE"; do
  n=$((n + 1))
  [ $n -lt $FIRST ] && continue
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_dense_$n -o run -- $CMD > gpurun_out/pmc_dense_$n.log 2>&1
done
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc_dense_trace -o run -- $CMD > gpurun_out/pmc_dense_trace.log 2>&1
