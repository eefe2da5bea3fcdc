"""Shard-stride (skew) and batch sweep for one (k, m, shard size) encode or
decode through the production plan API, on the MI355X.

For every pad in --pads the slab is [stripes][k+m][S + pad]; every config
is timed in the same process with shuffled interleaved rounds (median).
GB/s = algorithmic bytes ((k+m)*S per stripe for encode) / launch time.

    python tools/tune_stride.py --k 6 --m 3 --shard-kib 1024 --stripes 96 \
        --pads 0,256,4096,8192,65536
"""
from __future__ import annotations

import argparse
import json
import os
import random
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import erasure_coding_test_amd as E  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=6)
    ap.add_argument("--m", type=int, default=3)
    ap.add_argument("--shard-kib", type=int, default=1024)
    ap.add_argument("--stripes", default="96", help="comma list of batch sizes")
    ap.add_argument("--pads", default="0,4096")
    ap.add_argument("--erasures", default="", help="comma list: decode these shards instead of encoding")
    ap.add_argument("--rounds", type=int, default=12)
    a = ap.parse_args()
    k, m, S = a.k, a.m, a.shard_kib << 10
    M = E.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    er = [int(x) for x in a.erasures.split(",")] if a.erasures else None
    cases = []
    for B in [int(x) for x in a.stripes.split(",")]:
        for pad in [int(x) for x in a.pads.split(",")]:
            slab = torch.empty((B, k + m, S + pad), dtype=torch.uint8, device="cuda")
            slab.random_(0, 256)
            shards = [[slab[s, i, :S] for i in range(k + m)] for s in range(B)]
            if er is None:
                p = E.encode_plan(k, m, M).bind([st[:k] for st in shards], [st[k:] for st in shards], S)
                nbytes = (k + m) * S * B
            else:
                p = E.DecodePlan(k, m, M, er).bind_stripes(shards, S)
                nbytes = (len(p.src_ids) + len(p.out_ids)) * S * B
            cases.append({"stripes": B, "pad": pad, "plan": p, "slab": slab, "bytes": nbytes, "t": []})
    for rnd in range(a.rounds + 2):
        random.Random(rnd).shuffle(cases)
        for c in cases:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            c["plan"].launch()
            e1.record()
            torch.cuda.synchronize()
            if rnd >= 2:
                c["t"].append(e0.elapsed_time(e1))
    cases.sort(key=lambda c: (c["stripes"], c["pad"]))
    for c in cases:
        med = statistics.median(c["t"])
        print(json.dumps({"k": k, "m": m, "shard_kib": a.shard_kib, "erasures": er, "stripes": c["stripes"],
                          "pad": c["pad"], "median_ms": round(med, 4),
                          "GBps": round(c["bytes"] / med / 1e6, 1)}))


if __name__ == "__main__":
    main()
