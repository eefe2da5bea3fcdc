#!/bin/bash
# Round 6, second call: the GPU suite on the tree with the 16 MiB small-call
# threshold and the HBM-full test warmed and with headroom;
# the crossover grid's quick sizes and the drop-in latencies again (the lib
# arm is now the new default); then the N = 2 rehearsal of bench.py (both
# ranks on cuda:0) with and without its e2e NUMA affinity, the record that
# showed the two-process encode at 27.21 GiB/s in round 5; the host's CPU
# topology as the lease sees it.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06c
mkdir -p $O
python3 - > $O/host_cpus.json <<'PY'
import json, os, glob
aff = sorted(os.sched_getaffinity(0))
nodes = {os.path.basename(n): open(n + "/cpulist").read().strip() for n in sorted(glob.glob("/sys/devices/system/node/node*"))}
def rd(p):
    try:
        return open(p).read().strip()
    except OSError:
        return None
print(json.dumps({"affinity_count": len(aff), "affinity_head": aff[:8], "affinity_tail": aff[-8:], "nodes": nodes,
                  "cpu_max": rd("/sys/fs/cgroup/cpu.max"), "cpuset": rd("/sys/fs/cgroup/cpuset.cpus.effective"),
                  "os_cpu_count": os.cpu_count()}))
PY
rc=0
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.txt 2>&1 || rc=$?
tail -3 $O/gputest.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ]
timeout -k 10 300 ./tools/crossover.bin --quick > $O/crossover_quick.jsonl 2> $O/crossover_quick.err
timeout -k 10 200 ./tools/dropin_latency.bin > $O/dropin_latency.jsonl 2> $O/dropin_latency.err
echo latency_ok
ECGPU_BENCH_ONE_DEVICE=1 timeout -k 10 400 python3 -u bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench_n2.json 2> $O/bench_n2.err
ECGPU_BENCH_ONE_DEVICE=1 ECGPU_BENCH_E2E_NUMA=0 timeout -k 10 400 python3 -u bench.py --gpus 2 --steps 5 --warmup 2 \
    > $O/bench_n2_nonuma.json 2> $O/bench_n2_nonuma.err
echo session_ok
