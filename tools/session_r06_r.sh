#!/bin/bash
# Round 6: the synchronous-call fuzz at 40,000 cases and 5,000 aliased calls
# against the compiled reference, on the GPU path (the package keeps every
# call on the MI355X), after the planner changes of this round.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06r
mkdir -p $O
ECGPU_FUZZ_CASES=40000 ECGPU_FUZZ_ALIAS_CASES=5000 timeout -k 10 900 python3 -u -m pytest -s tests/test_fuzz_gpu.py -m gpu \
    -q --timeout 800 --timeout-method thread > $O/fuzz.txt 2>&1
tail -2 $O/fuzz.txt
echo session_ok
