#!/bin/bash
# Round-5 closing pass on the final w = 8 kernel build: the fallback tests
# (cpu_fallback.cpp changed after the first pass), per-dispatch PMC of C2 /
# the lost-parity decode / the C3 encode next to their XOR stream probes
# (effective clock, issue and memory waits), the profile pass
# (tools/profile_round.sh) and the bench with the LDS engine timed.  Each
# step has its own time limit; the chain stops at the first failure.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_cpu_fallback.py tests/test_devices.py > $O/gputest_fallback.log 2>&1
PCMD="python3 tools/probe_dense.py --pmc --probes --rounds 2 --reps 8 --shapes C2_encode,C3_decode_parity,C3_encode,C4_decode_0123"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/probe_trace -o run -- $PCMD > $O/probe_trace.log 2>&1
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $O/probe_sq -o run -- $PCMD > $O/probe_sq.log 2>&1
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/probe_tcc -o run -- $PCMD > $O/probe_tcc.log 2>&1
bash tools/profile_round.sh r05 > $O/profile_r05.log 2>&1
timeout -k 10 300 python3 bench.py --kernel lds > $O/bench_lds.json 2> $O/bench_lds.err
echo session_ok
