#!/bin/bash
# PMC passes over the bit-matrix packet lab (tools/packet_lab.bin): the
# production gf_xor_packets16p<32> and the half-VALU timing probe, one counter
# group per rocprofv3 run (rocprofv3 does not split counters over passes).
# Output under gpurun_out/pmc_packets_<n>/.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
n=0
for c in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE GRBM_COUNT" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_WAIT_INST_ANY" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  n=$((n + 1))
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_packets_$n -o run -- ./tools/packet_lab.bin --only probe_halfvalu --rounds 1 --reps 5 > gpurun_out/pmc_packets_$n.log 2>&1
done
