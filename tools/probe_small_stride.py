"""Small-shard stride A/B through the library (round 5): for each (k, m,
shard size) an encode plan and a decode{0} plan bound to two slabs of the same
stripes -- one at the library's stride for the scheme
(ecgpu_recommended_shard_stride_km, through alloc_stripes) and one at the
round-4 table's skew (+12 KiB at 256 KiB, +8 KiB at 512 KiB, +10 KiB at the
other sizes here; ECGPU_SHARD_SKEW_KIB while it is allocated) -- timed in interleaved rounds
(HIP events on the launch stream, median), ~2.5 GiB streamed per launch.
Parity of both slabs is compared with each other after the timing.

    python tools/probe_small_stride.py [--sizes 16,64] [--shapes '4,2;10,4'] [--rounds 5] [--reps 10] > out.jsonl
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from statistics import median

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = [(4, 2), (6, 3), (10, 4)]
SIZES_KIB = [16, 64, 128, 256]
PEAK_GBS = 8000.0
OLD_SKEW_KIB = {256: 12, 512: 8}  # the round-4 table (+10 KiB at the other sizes here)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--gib", type=float, default=2.5)
    ap.add_argument("--sizes", default=",".join(map(str, SIZES_KIB)), help="shard sizes, KiB")
    ap.add_argument("--shapes", default=";".join(f"{k},{m}" for k, m in SHAPES), help="k,m;k,m;...")
    ap.add_argument("--skews", default="", help="KiB skews to time beside the library's layout instead of "
                                                "the round-4 table's (e.g. 3,4,5,7 at 4 MiB)")
    args = ap.parse_args()
    shapes = [tuple(int(x) for x in sh.split(",")) for sh in args.shapes.split(";")]
    sizes = [int(x) for x in args.sizes.split(",")]
    import torch

    import erasure_coding_test_amd as E
    from erasure_coding_test_amd import _native as N
    from bench import time_launches
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    stream = torch.cuda.current_stream(dev)
    for k, m in shapes:
        M = E.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
        for kib in sizes:
            S = kib << 10
            B = max(1, int(args.gib * (1 << 30)) // ((k + m) * S))
            layouts = {}
            old = OLD_SKEW_KIB.get(kib, 10)
            others = [(f"skew{x}", int(x)) for x in args.skews.split(",") if x] or [(f"round4_skew{old}", old)]
            for name, skew in [("library", None)] + others:
                if skew is not None:
                    N.set_knob("ECGPU_SHARD_SKEW_KIB", skew)
                try:
                    slab, shards = E.alloc_stripes(B, k, m, S, dev)
                finally:
                    N.reset_knob("ECGPU_SHARD_SKEW_KIB")
                g = torch.Generator(device=dev).manual_seed(0x5A11 ^ kib)
                slab.random_(0, 256, generator=g)
                enc = E.encode_plan(k, m, M, dev.index).bind([st[:k] for st in shards], [st[k:] for st in shards], S)
                dec = E.DecodePlan(k, m, M, [0], 0, dev.index).bind_stripes(shards, S)
                layouts[name] = dict(slab=slab, shards=shards, enc=enc, dec=dec, stride=slab.shape[2], t_enc=[], t_dec=[])
            for _ in range(args.rounds):
                for L in layouts.values():
                    L["t_enc"].append(time_launches(lambda: L["enc"].launch(stream.cuda_stream), stream, args.reps, 2))
                    L["t_dec"].append(time_launches(lambda: L["dec"].launch(stream.cuda_stream), stream, args.reps, 2))
            # the same data in both layouts?  compare parity of stripe 0 / B-1 after re-encoding from equal data
            a = layouts["library"]
            same = True
            for name, _ in others:
                b = layouts[name]
                for s in (0, B - 1):
                    b["slab"][s, :k, :S].copy_(a["slab"][s, :k, :S])
                a["enc"].launch(stream.cuda_stream)
                b["enc"].launch(stream.cuda_stream)
                torch.cuda.synchronize(dev)
                same = same and all(torch.equal(a["slab"][s, k:, :S], b["slab"][s, k:, :S]) for s in (0, B - 1))
            for name, L in layouts.items():
                te, td = median(L["t_enc"]), median(L["t_dec"])
                print(json.dumps({
                    "k": k, "m": m, "shard_kib": kib, "stripes": B, "layout": name, "stride": int(L["stride"]),
                    "encode_ms": round(te, 4), "encode_frac": round((k + m) * S * B / (te / 1e3) / 1e9 / PEAK_GBS, 4),
                    "decode0_ms": round(td, 4), "decode0_frac": round((k + 1) * S * B / (td / 1e3) / 1e9 / PEAK_GBS, 4),
                    "step_ms": round(te + td, 4),
                    "parity_equal_across_layouts": bool(same)}), flush=True)
                L["enc"].close()
                L["dec"].close()
            del layouts, a
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
