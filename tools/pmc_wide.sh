#!/bin/bash
# PMC passes over the w = 32 lab (tools/wide_lab.bin), one counter group per
# rocprofv3 run (MI355X_MICROARCH.md: rocprofv3 does not split counters over
# passes).  Output under gpurun_out/pmc_wide<K>_<n>/.
#   bash tools/pmc_wide.sh [K]        (RS(K,4) w = 32 64 MiB; default K = 10)
set -e
K=${1:-10}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
n=0
for c in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  n=$((n + 1))
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_wide${K}_$n -o run -- ./tools/wide_lab.bin --w 32 --k $K --rounds 1 --reps 5 > gpurun_out/pmc_wide${K}_$n.log 2>&1
done
