#!/bin/bash
# Round-4 lab session on the GPU box (one gpurun call): the w = 32 K = 11 / 12
# chunkings and the w = 16 unit kernel in the lab, the w = 16 unit knob through
# the API call under a kernel trace, a PMC record of the K = 12 w = 32 kernels,
# and the dense-shape scalar / VMEM-FIFO counter pass.  Every step has its own
# time limit; the chain stops at the first failure.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 240 ./tools/wide_lab.bin --w 32 --k 12 --rounds 9 --only prod_u1,prod_pipe,pipe_nch > $O/r04_wide_lab_k12.jsonl 2> $O/r04_wide_lab_k12.err
timeout -k 10 240 ./tools/wide_lab.bin --w 32 --k 11 --rounds 9 --only prod_u1,prod_pipe,pipe_nch > $O/r04_wide_lab_k11.jsonl 2> $O/r04_wide_lab_k11.err
timeout -k 10 240 ./tools/wide_lab.bin --w 16 --k 10 --rounds 9 --only prod_nib16_4,prod_nib16u > $O/r04_wide_lab_w16.jsonl 2> $O/r04_wide_lab_w16.err
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/ab16u -o run -- python3 tools/ab_wide16.py --knob ECGPU_WIDE16_UNITS --values 0,1 > $O/ab16u.log 2>&1
python3 tools/ab_wide16.py --summarize $O/ab16u --knob ECGPU_WIDE16_UNITS --values 0,1 > $O/r04_ab_wide16_units.json
rm -rf $O/ab16u
bash tools/pmc_wide.sh 12
python3 tools/pmc_summary.py $O/pmc_wide12_* > $O/r04_pmc_wide12.json
rm -rf $O/pmc_wide12_*/
bash tools/pmc_dense.sh 5
python3 tools/pmc_summary.py $O/pmc_dense_5 $O/pmc_dense_trace > $O/r04_pmc_dense_5.json
rm -rf $O/pmc_dense_5 $O/pmc_dense_trace
echo session_ok
