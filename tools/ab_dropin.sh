#!/bin/bash
# A/B of the synchronous drop-in path's staging knobs on the GPU box:
#   bash tools/ab_dropin.sh "ECGPU_ZC_KIB=1024" "ECGPU_ZC_KIB=0" ...
# Each argument is an environment setting for one quick run of
# tools/dropin_latency.bin; results are appended to gpurun_out/ab.txt.
mkdir -p gpurun_out
for cfg in "$@"; do
  echo "== $cfg" >> gpurun_out/ab.txt
  env $cfg timeout -k 10 120 ./tools/dropin_latency.bin --quick >> gpurun_out/ab.txt 2>&1 || exit 1
done
