"""The BASELINE launch shapes furthest below their XOR stream probes, in one
process: C4's dense decode{0,1,2,3}, C3's lost-parity
decode {12} (one dense row), C2's RS(6,3) 1 MiB encode, with the C3 encode
and the XOR-only decode{0} beside them as references.  The bench's own slab
layout and batch sizes (bench.config_block), random data.

  python tools/probe_dense.py                 # interleaved A/B of knob variants, JSON lines
  python tools/probe_dense.py --pmc --reps 5  # every shape once per round, default knobs
                                              # (run under rocprofv3 --pmc, tools/pmc_dense.sh)

A variant is a set of knobs (ecgpu_set_knob) applied while its plans are
created and launched; plans are rebuilt per variant so engine / store
policy knobs take effect.  Medians of HIP-event launch times.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import erasure_coding_test_amd as E  # noqa: E402
from erasure_coding_test_amd import _native as N  # noqa: E402

# name: (k, m, shard bytes, stripes, erasures or None for encode, written shards)
SHAPES = {
    "C3_encode": (10, 4, 4 << 20, 96, None),
    "C3_decode_0": (10, 4, 4 << 20, 96, [0]),
    "C3_decode_parity": (10, 4, 4 << 20, 96, [12]),
    "C4_decode_0123": (10, 4, 4 << 20, 96, [0, 1, 2, 3]),
    "C2_encode": (6, 3, 1 << 20, 512, None),
}

VARIANTS = {
    "default": {},
    "cap_never": {"cap": 0},
    "cap_always": {"cap": 1},
    "bpcu6_always": {"cap": 1, "blocks_per_cu": 6},
    "bpcu5_always": {"cap": 1, "blocks_per_cu": 5},
    "bpcu4_always": {"cap": 1, "blocks_per_cu": 4},
    "bpcu3_always": {"cap": 1, "blocks_per_cu": 3},
    "lds_engine": {"kernel": 1},
    "lds_engine_uncapped": {"kernel": 1, "cap": 0},
}


def build(shape, slabs):
    k, m, S, B, er = SHAPES[shape]
    key = (k, m, S, B)
    if key not in slabs:
        slab, shards = E.alloc_stripes(B, k, m, S)
        bench.fill_random(slab, list(range(B)), 40 + k)
        M = E.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
        # consistent stripes: a decode rewrites its shards with the same bytes
        E.encode_plan(k, m, M).bind([st[:k] for st in shards], [st[k:] for st in shards], S).launch()
        torch.cuda.synchronize()
        slabs[key] = (slab, shards, M)
    slab, shards, M = slabs[key]
    if er is None:
        p = E.encode_plan(k, m, M).bind([st[:k] for st in shards], [st[k:] for st in shards], S)
        nbytes = (k + m) * S * B
    else:
        p = E.DecodePlan(k, m, M, er, 0).bind_stripes(shards, S)
        nbytes = (k + len(er)) * S * B
    return p, nbytes


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--pmc", action="store_true", help="default knobs only, every shape --reps times per round")
    ap.add_argument("--variants", default=",".join(VARIANTS))
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--tag", default="")
    ap.add_argument("--probes", action="store_true",
                    help="after each shape's launches, its XOR stream probe (bench.xor_stream_probe) on the same slab: "
                         "per-dispatch PMC of kernel and probe side by side (effective clock, round 5)")
    a = ap.parse_args()
    shapes = a.shapes.split(",")
    variants = ["default"] if a.pmc else a.variants.split(",")
    stream = torch.cuda.current_stream()
    slabs = {}
    times = {(s, v): [] for s in shapes for v in variants}
    sizes = {}
    for rnd in range(a.rounds):
        order = variants if rnd % 2 == 0 else variants[::-1]
        for v in order:
            N.reset_knob(None)
            for name, val in VARIANTS[v].items():
                N.set_knob(name, val)
            for s in shapes:
                p, nbytes = build(s, slabs)
                sizes[s] = nbytes
                ms = bench.time_launches(lambda: p.launch(stream.cuda_stream), stream, a.reps, warmup=2)
                times[(s, v)].append(ms)
                p.close()
                if a.probes:
                    k, m, S, B, er = SHAPES[s]
                    slab = slabs[(k, m, S, B)][0]
                    bench.xor_stream_probe(slab, S, k, m if er is None else len(er), reps=a.reps)
        N.reset_knob(None)
    for s in shapes:
        base = statistics.median(times[(s, "default")])
        for v in variants:
            ms = statistics.median(times[(s, v)])
            print(json.dumps({"run": a.tag or "probe_dense", "shape": s, "variant": v, "knobs": VARIANTS[v],
                              "median_ms": round(ms, 4), "ms_per_round": [round(x, 4) for x in times[(s, v)]],
                              "GBps": round(sizes[s] / (ms / 1e3) / 1e9, 1),
                              "frac": round(sizes[s] / (ms / 1e3) / 1e9 / bench.HBM_PEAK_GBS, 4),
                              "vs_default": round(base / ms, 4)}), flush=True)


if __name__ == "__main__":
    main()
