"""Chooses the library's small-call routing rule (SURVEY §5 "min offload size",
DESIGN.md §8) from a tools/crossover.cpp record: for every measured call
(shape x shard size x pageable/pinned x warm/cold) the GPU and CPU-executor
arms' medians are known, so a candidate rule's cost is the time of the arm it
picks.  Two rule families:

  size    CPU iff bytes moved < T                        (T swept)
  model   CPU iff cpu_est < gpu_est, with
            cpu_est = moved / Bm + mul_bytes / Bx         (mul_bytes: size x the
                                                           map's coefficients > 1)
            gpu_est = G0 + moved / Bg                     (all four swept)

Reported per rule: the geometric-mean and worst slowdown against the better
arm of each call, overall and per memory / temperature class.

    python3 tools/crossover_fit.py gpurun_out/r06a/crossover.jsonl
"""
from __future__ import annotations

import itertools
import json
import math
import sys

# (nonunit, unit) coefficients of each shape's fused map (planner.hpp): the
# ECX multiply-add is acc = c*block + 1*acc; Vandermonde RS(k,m) has a unit
# first row and column; decode{0} with row_k_ones is an XOR of 10 survivors;
# C4's decode rows are the inverse's dense 4 x 10.
TERMS = {
    "ECX region multiply-add (r2 accumulator)": (1, 1),
    "ECX region xor (r3 == r2 accumulator)": (0, 2),
    "region xor r1 ^ r2 -> r3": (0, 2),
    "RS(4,2) encode (C1)": (3, 5),
    "RS(3,3) encode (client default)": (4, 5),
    "RS(6,3) encode (C2)": (10, 8),
    "RS(10,4) encode (C3)": (27, 13),
    "RS(10,4) decode{0}": (0, 10),
    "RS(10,4) decode{0,1,2,3} (C4)": (40, 0),
}


def load(path):
    rows = []
    for line in open(path):
        d = json.loads(line)
        if "shape" in d:
            nonunit, unit = TERMS[d["shape"]]
            d["mul_bytes"] = nonunit * d["shard_bytes"]
            d["cls"] = f"{d['memory']}/{d['buffers']}"
            rows.append(d)
    return rows


def score(rows, pick):
    """pick(row) -> 'cpu' | 'gpu'; geometric-mean and worst slowdown."""
    out = {}
    for cls in sorted({r["cls"] for r in rows}) + ["all"]:
        rs = [r for r in rows if cls in ("all", r["cls"])]
        sl = [(r["cpu_us"] if pick(r) == "cpu" else r["gpu_us"]) / min(r["cpu_us"], r["gpu_us"]) for r in rs]
        out[cls] = (round(math.exp(sum(map(math.log, sl)) / len(sl)), 4), round(max(sl), 3))
    return out


def main():
    rows = load(sys.argv[1])
    res = []
    for t_kib in [0, 256, 512, 1024, 2048, 3072, 4096, 6144, 8192, 12288, 16384, 24576, 32768, 1 << 20]:
        res.append(({"rule": "size", "T_KiB": t_kib},
                    score(rows, lambda r, t=t_kib: "cpu" if r["bytes_moved"] < (t << 10) else "gpu")))
    # model: bandwidths in GB/s (= bytes per ns, so bytes / (B * 1e3) is microseconds)
    grid = itertools.product([20, 30, 45, 60, 90], [100, 150, 200, 260, 350], [10, 20, 30, 40], [30, 40, 50, 60])
    for bm, bx, g0, bg in grid:
        def pick(r, bm=bm, bx=bx, g0=g0, bg=bg):
            cpu = r["bytes_moved"] / (bm * 1e3) + r["mul_bytes"] / (bx * 1e3)
            gpu = g0 + r["bytes_moved"] / (bg * 1e3)
            return "cpu" if cpu < gpu else "gpu"
        res.append(({"rule": "model", "Bm": bm, "Bx": bx, "G0": g0, "Bg": bg}, score(rows, pick)))
    res.sort(key=lambda x: (x[1]["all"][0], x[1]["all"][1]))
    for rule, s in res[:12]:
        print(json.dumps({**rule, **{k: list(v) for k, v in s.items()}}))
    print("--- size rules")
    for rule, s in res:
        if rule["rule"] == "size":
            print(json.dumps({**rule, **{k: list(v) for k, v in s.items()}}))


if __name__ == "__main__":
    main()
