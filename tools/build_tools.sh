#!/bin/bash
# Builds the C++ measurement tools in-tree (here, on the CPU; the binaries
# travel to the GPU box with the tree): tools/*.bin (git-ignored).
set -e
cd "$(dirname "$0")/.."
g++ -O2 -Wall -std=c++17 tools/dropin_latency.cpp -Iinclude/dropin -Lerasure_coding_test_amd/lib -ljerasure_amd -lecgpu \
    -Wl,-rpath,'$ORIGIN/../erasure_coding_test_amd/lib' -o tools/dropin_latency.bin
g++ -O2 -Wall -std=c++17 tools/crossover.cpp -Iinclude/dropin -Lerasure_coding_test_amd/lib -ljerasure_amd -lecgpu \
    -Wl,-rpath,'$ORIGIN/../erasure_coding_test_amd/lib' -o tools/crossover.bin
/opt/rocm/bin/hipcc -O2 --offload-arch=gfx950 tools/host_overhead.cpp -Iinclude/dropin -Lerasure_coding_test_amd/lib -ljerasure_amd -lecgpu \
    -Wl,-rpath,'$ORIGIN/../erasure_coding_test_amd/lib' -o tools/host_overhead.bin
/opt/rocm/bin/hipcc -O2 --offload-arch=gfx950 tools/hip_overheads.cpp -o tools/hip_overheads.bin -lpthread
/opt/rocm/bin/hipcc -O2 --offload-arch=gfx950 tools/zero_copy_probe.cpp -o tools/zero_copy_probe.bin
/opt/rocm/bin/hipcc -O2 --offload-arch=gfx950 tools/pageable_duplex_probe.cpp -o tools/pageable_duplex_probe.bin -lpthread
/opt/rocm/bin/hipcc -O2 --offload-arch=gfx950 tools/sdma_d2h_probe.cpp -lhsa-runtime64 -o tools/sdma_d2h_probe.bin
