#!/bin/bash
# Round 6: the zero-copy pipeline's grid.  ECGPU_ZC_GRID (64 workgroups) was
# tuned on PCIe *reads* of synchronous calls; the pipeline's kernel also
# writes the parity over PCIe.  One process, the skewed DMA pipeline as the
# reference, ZC_GRID 64 / 128 / 256 / 512 / uncapped; then two processes at
# the two best grids.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06i
mkdir -p $O
L=pipe_encode_skew,pipe_encode_zc2,pipe_decode_zc2,pipe_encode_zc1,pipe_encode
port=29690
for g in 64 128 256 512 0; do
  port=$((port + 1))
  timeout -k 10 200 python3 -u tools/e2e_pair.py --world 1 --port $port --tag one_g$g --passes 5 --legs $L \
      --knob ECGPU_ZC_GRID=$g >> $O/pair.jsonl 2> $O/one_g$g.err
done
echo one_ok
for g in 128 256; do
  port=$((port + 1))
  timeout -k 10 240 python3 -u tools/e2e_pair.py --rank 0 --world 2 --port $port --tag two_g$g --passes 5 --legs $L \
      --knob ECGPU_ZC_GRID=$g >> $O/pair.jsonl 2> $O/two_g${g}_0.err & a=$!
  timeout -k 10 240 python3 -u tools/e2e_pair.py --rank 1 --world 2 --port $port --tag two_g$g --passes 5 --legs $L \
      --knob ECGPU_ZC_GRID=$g > /dev/null 2> $O/two_g${g}_1.err & b=$!
  ra=0; rb=0
  wait $a || ra=$?
  wait $b || rb=$?
  [ $ra -eq 0 ] && [ $rb -eq 0 ]
done
echo session_ok
