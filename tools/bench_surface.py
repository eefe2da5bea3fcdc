"""Throughput of the non-north-star surface on device-resident shards:
w = 8 / 16 / 32 matrix encode and GF(2) bit-matrix / schedule encode, RS(10,4)
over 64 MiB shards (one stripe, 896 MiB of algorithmic traffic per call).

Times each synchronous API call (host planning + launch + sync, median of
reps) -- run under `rocprofv3 --kernel-trace --stats` for kernel-only times.

    python tools/bench_surface.py [--shard-mib 64] [--reps 10]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import erasure_coding_test_amd as E  # noqa: E402
from erasure_coding_test_amd import _native as N  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shard-mib", type=int, default=64)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    k, m, S = 10, 4, a.shard_mib << 20
    J = E.jerasure
    data = [torch.randint(0, 256, (S,), dtype=torch.uint8, device="cuda") for _ in range(k)]
    coding = [torch.empty(S, dtype=torch.uint8, device="cuda") for _ in range(m)]
    nbytes = (k + m) * S
    out = []

    def rec(name, fn):
        t = timed(fn, a.reps)
        out.append({"case": name, "ms": round(t * 1e3, 3), "GBps": round(nbytes / t / 1e9, 1)})

    for w in (8, 16, 32):
        M = E.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, w)
        rec(f"jerasure_matrix_encode w={w}", lambda M=M, w=w: J.jerasure_matrix_encode(k, m, w, M, data, coding, S))
        if w != 8:  # A/B: the v_perm column engine (a knob, switched in process)
            N.set_knob("ECGPU_WIDE", 1)
            rec(f"jerasure_matrix_encode w={w} (v_perm engine, ECGPU_WIDE=1)",
                lambda M=M, w=w: J.jerasure_matrix_encode(k, m, w, M, data, coding, S))
            N.reset_knob("ECGPU_WIDE")
    M8 = E.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    # the same shards through the batched plan API (gf_apply, pointer and
    # coefficient tables in HBM) against the synchronous call's inline launch
    plan = E.encode_plan(k, m, M8).bind([data], [coding], S)
    rec("encode_plan w=8 (plan launch, same shards)", lambda: plan.launch())
    # and on a skewed slab (the library's recommended shard stride)
    slab, shards = E.alloc_stripes(1, k, m, S)
    shards[0][0].copy_(data[0])
    rec("jerasure_matrix_encode w=8, skewed slab",
        lambda: J.jerasure_matrix_encode(k, m, 8, M8, shards[0][:k], shards[0][k:], S))
    bm = J.jerasure_matrix_to_bitmatrix(k, m, 8, M8)
    for ps in (1024, 4096, 65536):
        rec(f"jerasure_bitmatrix_encode w=8 packetsize={ps}",
            lambda ps=ps: J.jerasure_bitmatrix_encode(k, m, 8, bm, data, coding, S, ps))
    N.set_knob("ECGPU_PACKET", 3)  # the general pipelined 16-B kernel (no unit form)
    rec("jerasure_bitmatrix_encode w=8 packetsize=4096 (general kernel, ECGPU_PACKET=3)",
        lambda: J.jerasure_bitmatrix_encode(k, m, 8, bm, data, coding, S, 4096))
    N.reset_knob("ECGPU_PACKET")
    sched = J.jerasure_dumb_bitmatrix_to_schedule(k, m, 8, bm)
    rec("jerasure_schedule_encode (dumb) w=8 packetsize=4096",
        lambda: J.jerasure_schedule_encode(k, m, 8, sched, data, coding, S, 4096))
    print(json.dumps({"workload": f"RS(10,4), {a.shard_mib} MiB shards, device-resident, one stripe per call",
                      "results": out, "cpu_fallbacks": N.fallback_count()}, indent=1))


if __name__ == "__main__":
    main()
