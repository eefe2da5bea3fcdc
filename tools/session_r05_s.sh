#!/bin/bash
# Round-5: the device-validation and slab round-trip tests, then the whole -m gpu
# suite (one process, as the driver runs it).
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05s
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v -m gpu --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_devices.py -k "devices or scheme_aware" > $O/gputest_layouts.log 2>&1
timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > $O/gputest.log 2>&1
echo session_ok
