"""Reads the rocprofv3 memory-copy (and kernel) traces of processes that shared
one GPU (tools/e2e_pair.py under `rocprofv3 --kernel-trace
--memory-copy-trace --output-format csv`) and reports, per direction, how the
processes' copies overlapped and what each copy ran at.

    python3 tools/copy_overlap.py DIR0 DIR1 [--h2d-bytes B] [--d2h-bytes B]

Timestamps are the host's monotonic clock in ns, common to the processes.
Per process and direction: copies, the union of their busy time, the median
copy duration and rate; for the pair: the time both processes had a copy of
the same direction in flight, the time any H2D and any D2H overlapped, and
each direction's bytes over the union of its busy time (the link's achieved
rate in that direction while busy).  Copies are split into those that ran
alone in their direction and those that shared it with the other process.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import statistics


def load(d, suffix):
    files = glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    return rows


def direction(r):
    text = " ".join(str(v) for v in r.values()).upper()
    if "HOST_TO_DEVICE" in text:
        return "h2d"
    if "DEVICE_TO_HOST" in text:
        return "d2h"
    return None


def union(iv):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def total(iv):
    return sum(e - s for s, e in iv)


def intersect(a, b):
    i = j = 0
    out = []
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if s < e:
            out.append([s, e])
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return out


def overlap_with(s, e, iv):
    return sum(max(0, min(e, b) - max(s, a)) for a, b in iv)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--h2d-bytes", type=int, default=10 * (4 << 20))
    ap.add_argument("--d2h-bytes", type=int, default=4 * (4 << 20))
    ap.add_argument("--skip-null-stream", action="store_true",
                    help="ignore copies on stream 0 (a script's own setup copies through torch's null stream)")
    a = ap.parse_args()
    size = {"h2d": a.h2d_bytes, "d2h": a.d2h_bytes}
    copies = []  # per process: {dir: [(s, e)]}
    kernels = []
    for d in a.dirs:
        per = {"h2d": [], "d2h": []}
        for r in load(d, "memory_copy_trace.csv"):
            k = direction(r)
            if a.skip_null_stream and str(r.get("Stream_Id", "")).strip() == "0":
                continue
            if k:
                per[k].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
        copies.append(per)
        kernels.append([(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in load(d, "kernel_trace.csv")])
    out = {"processes": len(a.dirs), "per_process": [], "pair": {}}
    busy = {k: [union(p[k]) for p in copies] for k in ("h2d", "d2h")}
    for i, p in enumerate(copies):
        rec = {"dir": a.dirs[i], "kernels": len(kernels[i])}
        for k in ("h2d", "d2h"):
            iv = p[k]
            if not iv:
                continue
            durs = [(e - s) / 1e3 for s, e in iv]
            others = union([x for j, b in enumerate(busy[k]) if j != i for x in b])
            alone, shared = [], []
            for s, e in iv:
                (shared if overlap_with(s, e, others) > 0.5 * (e - s) else alone).append((e - s) / 1e3)
            rec[k] = {"copies": len(iv), "busy_ms": round(total(busy[k][i]) / 1e6, 2),
                      "median_us": round(statistics.median(durs), 1),
                      "median_GBps": round(size[k] / statistics.median(durs) / 1e3, 1),
                      "alone": {"copies": len(alone),
                                "median_GBps": round(size[k] / statistics.median(alone) / 1e3, 1) if alone else None},
                      "shared_with_other_process": {
                          "copies": len(shared),
                          "median_GBps": round(size[k] / statistics.median(shared) / 1e3, 1) if shared else None}}
        out["per_process"].append(rec)
    allc = [x for p in copies for k in ("h2d", "d2h") for x in p[k]]
    if allc:
        t0, t1 = min(s for s, _ in allc), max(e for _, e in allc)
        pair = {"span_ms": round((t1 - t0) / 1e6, 2)}
        for k in ("h2d", "d2h"):
            u = union([x for b in busy[k] for x in b])
            n = sum(len(p[k]) for p in copies)
            pair[k] = {"busy_ms": round(total(u) / 1e6, 2), "busy_frac_of_span": round(total(u) / (t1 - t0), 3),
                       "GBps_while_busy": round(n * size[k] / total(u), 1) if u else None}
            if len(busy[k]) >= 2:
                both = intersect(busy[k][0], busy[k][1])
                pair[k]["both_processes_ms"] = round(total(both) / 1e6, 2)
        hu = union([x for b in busy["h2d"] for x in b])
        du = union([x for b in busy["d2h"] for x in b])
        pair["h2d_and_d2h_overlap_ms"] = round(total(intersect(hu, du)) / 1e6, 2)
        if len(copies) >= 2:
            # cross-process duplex: one process's H2D against the other's D2H
            pair["h2d0_d2h1_overlap_ms"] = round(total(intersect(busy["h2d"][0], busy["d2h"][1])) / 1e6, 2)
            pair["h2d1_d2h0_overlap_ms"] = round(total(intersect(busy["h2d"][1], busy["d2h"][0])) / 1e6, 2)
        out["pair"] = pair
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
