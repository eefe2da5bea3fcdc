#!/bin/bash
# Round 6: concurrent unchanged callers (the client's ENC_THREAD_NUM encode
# threads, client_main.cpp:1074-1164): 1 / 2 / 4 / 8 threads each encoding
# its own pageable stripe through the mangled names, every call on the GPU,
# the library defaults, every call on the CPU executor.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06s
mkdir -p $O
ECGPU_MIN_OFFLOAD_KIB=0 timeout -k 10 200 ./tools/dropin_latency.bin --threads > $O/threads_gpu.jsonl 2> $O/threads_gpu.err
timeout -k 10 200 ./tools/dropin_latency.bin --threads > $O/threads_lib.jsonl 2> $O/threads_lib.err
ECGPU_GPU=0 timeout -k 10 200 ./tools/dropin_latency.bin --threads > $O/threads_cpu.jsonl 2> $O/threads_cpu.err
echo session_ok
