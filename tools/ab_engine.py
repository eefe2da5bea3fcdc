"""Engine A/B in one process: the v_perm engine vs the LDS nibble-table engine
on the same launch, interleaved rounds, medians.

Prints JSON: per shape, multiply terms per shard touched and each engine's
median / min / max ms over the rounds.  (Round 2 ran it with ECGPU_DENSE=0,
a since-removed switch that had sent dense launches to the LDS engine.)

    python tools/ab_engine.py [--rounds 10]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import erasure_coding_test_amd as E  # noqa: E402
from erasure_coding_test_amd import _native as N  # noqa: E402

# name: (k, m, shard bytes, stripes, erasures or None for encode)
SHAPES = {
    "C4 RS(10,4) 4 MiB decode{0,1,2,3}": (10, 4, 4 << 20, 24, [0, 1, 2, 3]),
    "RS(10,4) 4 MiB decode{0,1}": (10, 4, 4 << 20, 24, [0, 1]),
    "RS(10,4) 4 MiB decode{0,1,2}": (10, 4, 4 << 20, 24, [0, 1, 2]),
    "RS(6,3) 1 MiB decode{0,1,2}": (6, 3, 1 << 20, 128, [0, 1, 2]),
    "RS(12,4) 16 MiB decode{0,1,2,3}": (12, 4, 16 << 20, 8, [0, 1, 2, 3]),
    "C3 RS(10,4) 4 MiB encode": (10, 4, 4 << 20, 24, None),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    out = {}
    for name, (k, m, S, B, er) in SHAPES.items():
        M = E.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
        slab, shards = E.alloc_stripes(B, k, m, S, dev)
        slab.random_(0, 256)
        if er is None:
            plans = {kind: E.encode_plan(k, m, M, 0).bind([st[:k] for st in shards], [st[k:] for st in shards], S)
                     for kind in (N.KERNEL_PERM, N.KERNEL_LDS)}
            nbytes = (k + m) * S * B
            coefs = M
            rows, nsrc = m, k
        else:
            plans = {kind: E.DecodePlan(k, m, M, er, 0, 0).bind_stripes(shards, S)
                     for kind in (N.KERNEL_PERM, N.KERNEL_LDS)}
            p0 = plans[N.KERNEL_PERM]
            nbytes = (len(p0.src_ids) + len(p0.out_ids)) * S * B
            coefs, rows, nsrc = p0.coefs, p0.rows, p0.nsrc
        for kind, p in plans.items():
            p.set_kernel(kind, True)
        mul = sum(1 for c in coefs if c > 1)
        ts = {N.KERNEL_PERM: [], N.KERNEL_LDS: []}
        for r in range(a.rounds):
            order = (N.KERNEL_PERM, N.KERNEL_LDS) if r % 2 == 0 else (N.KERNEL_LDS, N.KERNEL_PERM)
            for kind in order:
                ts[kind].append(bench.time_launches(lambda: plans[kind].launch(stream.cuda_stream), stream, 10, 2))
        res = {"multiply_terms_per_shard": round(mul / (rows + nsrc), 2), "bytes_per_launch": nbytes}
        for kind, label in ((N.KERNEL_PERM, "v_perm"), (N.KERNEL_LDS, "lds")):
            v = sorted(ts[kind])
            res[label] = {"median_ms": round(v[len(v) // 2], 4), "min_ms": round(v[0], 4), "max_ms": round(v[-1], 4),
                          "GBps": round(nbytes / (v[len(v) // 2] / 1e3) / 1e9, 1)}
        out[name] = res
        print(json.dumps({name: res}), file=sys.stderr, flush=True)
        for p in plans.values():
            p.close()
        del slab, shards
        torch.cuda.empty_cache()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
