"""Residency-cap sweep with repeats (DESIGN.md §5 "Residency cap").

The runtime caps the production kernel at 4 (K + R <= 9) or 3 workgroups
per CU (launches dense in GF multiplies excepted).  This sweep times every
BASELINE shape -- plus small and mid K + R encode and decode shapes -- under
each fixed block count (ECGPU_BLOCKS_PER_CU, 0 = never cap) and under the
default rule, in interleaved rounds, one process per setting per round (the
setting is read once per process).  Prints per shape and setting the median,
min and max GB/s of algorithmic bytes over the rounds as JSON.

    python tools/tune_residency.py [--rounds 3]
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# name: (k, m, shard bytes, stripes, erasures or None for encode)
SHAPES = {
    "C1 RS(4,2) 64 KiB encode": (4, 2, 64 << 10, 2048, None),
    "C1 RS(4,2) 64 KiB decode{0}": (4, 2, 64 << 10, 2048, [0]),
    "C2 RS(6,3) 1 MiB encode": (6, 3, 1 << 20, 128, None),
    "RS(6,3) 1 MiB decode{0,1}": (6, 3, 1 << 20, 128, [0, 1]),
    "RS(8,2) 1 MiB encode": (8, 2, 1 << 20, 128, None),
    "C3 RS(10,4) 4 MiB encode": (10, 4, 4 << 20, 24, None),
    "C3 RS(10,4) 4 MiB decode{0}": (10, 4, 4 << 20, 24, [0]),
    "C5 RS(12,4) 16 MiB encode": (12, 4, 16 << 20, 8, None),
}
SETTINGS = ["rule", "0", "2", "3", "4", "6", "8"]


def worker():
    import torch

    sys.path.insert(0, ROOT)
    import bench
    import erasure_coding_test_amd as E
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    out = {}
    for name, (k, m, S, B, er) in SHAPES.items():
        M = E.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
        slab, shards = E.alloc_stripes(B, k, m, S, dev)
        slab.random_(0, 256)
        if er is None:
            p = E.encode_plan(k, m, M, 0).bind([st[:k] for st in shards], [st[k:] for st in shards], S)
            nbytes = (k + m) * S * B
        else:
            p = E.DecodePlan(k, m, M, er, 0, 0).bind_stripes(shards, S)
            nbytes = (len(p.src_ids) + len(p.out_ids)) * S * B
        ms = bench.time_launches(lambda: p.launch(stream.cuda_stream), stream, 15, warmup=5)
        out[name] = nbytes / (ms / 1e3) / 1e9
        p.close()
        del slab, shards
        torch.cuda.empty_cache()
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--worker", action="store_true")
    a = ap.parse_args()
    if a.worker:
        return worker()
    res = {s: [] for s in SETTINGS}
    for r in range(a.rounds):
        order = SETTINGS if r % 2 == 0 else SETTINGS[::-1]
        for setting in order:
            env = dict(os.environ)
            env.pop("ECGPU_BLOCKS_PER_CU", None)
            if setting != "rule":
                env["ECGPU_BLOCKS_PER_CU"] = setting
            p = subprocess.run([sys.executable, os.path.abspath(__file__), "--worker"], env=env, capture_output=True,
                               text=True, timeout=300)
            if p.returncode != 0:
                print(p.stderr[-2000:], file=sys.stderr)
                return 1
            res[setting].append(json.loads(p.stdout.strip().splitlines()[-1]))
            print(f"round {r} setting {setting} done", file=sys.stderr, flush=True)
            time.sleep(0.5)
    summary = {}
    for name in SHAPES:
        summary[name] = {}
        for setting in SETTINGS:
            v = sorted(x[name] for x in res[setting])
            summary[name][setting] = {"median_GBps": round(v[len(v) // 2], 1), "min": round(v[0], 1),
                                      "max": round(v[-1], 1)}
    print(json.dumps({"rounds": a.rounds, "settings": "ECGPU_BLOCKS_PER_CU (0 = never cap; rule = 4 if K+R <= 9 else 3 "
                                                      "unless > 2.5 multiplies per shard)", "results": summary}, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
