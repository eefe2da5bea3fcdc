"""In-process A/B of a w = 16 knob through the API call
(jerasure_matrix_encode, RS(10,4) w = 16, 64 MiB shards) on two shard
layouts: separately allocated tensors (what a caller passing malloc'd shards
gets) and the library's skewed stripe slab.  Default: the packed nibble
kernel's grid cap (ECGPU_WIDE16_BPCU 0 / 3 / 4); --knob ECGPU_WIDE16_UNITS
--values 0,1 compares its unit-structure form.  The knob is switched with
ecgpu_set_knob between launches.  Run under rocprofv3 --kernel-trace;
launches are attributed by order (rounds x layouts x settings x reps).

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ab16 -o run -- python3 tools/ab_wide16.py [--knob K --values a,b]
    python3 tools/ab_wide16.py --summarize gpurun_out/ab16 [--knob K --values a,b]
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
KNOB = "ECGPU_WIDE16_BPCU"
SETTINGS = ["0", "3", "4"]
LAYOUTS = ["separate", "slab"]
ROUNDS, REPS = 6, 5


def run():
    import torch

    import erasure_coding_test_amd as E
    from erasure_coding_test_amd import _native as N
    k, m, w, S = 10, 4, 16, 64 << 20
    M = E.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, w)
    sep_d = [torch.randint(0, 256, (S,), dtype=torch.uint8, device="cuda") for _ in range(k)]
    sep_c = [torch.empty(S, dtype=torch.uint8, device="cuda") for _ in range(m)]
    slab, shards = E.alloc_stripes(1, k, m, S)
    slab.random_(0, 256)
    lay = {"separate": (sep_d, sep_c), "slab": (shards[0][:k], shards[0][k:])}
    for _ in range(ROUNDS):
        for L in LAYOUTS:
            d, c = lay[L]
            for st in SETTINGS:
                N.set_knob(KNOB, int(st))
                for _ in range(REPS):
                    E.jerasure.jerasure_matrix_encode(k, m, w, M, d, c, S)
    torch.cuda.synchronize()


def summarize(d):
    f = glob.glob(os.path.join(d, "**", "run_kernel_trace.csv"), recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if "gf_apply_wide_nib16" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    out, i = {}, 0
    for _ in range(ROUNDS):
        for L in LAYOUTS:
            for st in SETTINGS:
                out.setdefault(f"{L} {KNOB}={st}", []).extend(durs[i:i + REPS])
                i += REPS
    res = {key: {"median_us": round(statistics.median(v), 1), "min_us": round(min(v), 1), "n": len(v)}
           for key, v in out.items()}
    names = sorted({r["Kernel_Name"].split("(")[0] for r in rows})
    print(json.dumps({"kernel": names, "call": "jerasure_matrix_encode RS(10,4) w=16 64 MiB", "knob": KNOB,
                      "launches": len(durs), "results": res}, indent=1))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--summarize")
    ap.add_argument("--knob", default=KNOB)
    ap.add_argument("--values", default=",".join(SETTINGS))
    a = ap.parse_args()
    KNOB, SETTINGS = a.knob, a.values.split(",")
    summarize(a.summarize) if a.summarize else run()
