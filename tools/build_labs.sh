#!/bin/bash
# Builds the kernel A/B labs in-tree (here, on the CPU; tools/*.bin travel to
# the GPU box with the tree).  Each lab lays its slab out at the library's
# shard stride (shard_stride.hpp) unless --skew-kib says otherwise.
set -e
cd "$(dirname "$0")/.."
H="erasure_coding_test_amd/csrc/gf_host.cpp erasure_coding_test_amd/csrc/matrix_host.cpp"
for lab in wide_lab packet_lab encode_lab; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include -I erasure_coding_test_amd/csrc \
    tools/$lab.hip $H -o tools/$lab.bin &
done
wait
