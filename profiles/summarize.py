"""Summarise rocprofv3 outputs of a bench.py run into profiles/<tag>_*.json.

Inputs (written on the GPU box under gpurun_out/):
  <trace>/run_kernel_stats.csv, <trace>/run_kernel_trace.csv
      from  rocprofv3 --kernel-trace --stats --output-format csv -- python bench.py ...
  <fetch>/run_counter_collection.csv   from  rocprofv3 --pmc FETCH_SIZE ...
  <write>/run_counter_collection.csv   from  rocprofv3 --pmc WRITE_SIZE ...

HBM-traffic correction (MI355X_MICROARCH.md §HBM): on gfx950 FETCH_SIZE
reports exactly half of the bytes of a wide coalesced streaming read, so the
read side is doubled; WRITE_SIZE is exact for 16-B/lane streaming stores.
Both counters are in KiB.  Only full-size launches (grid = the bench's batch)
are averaged; the bench's one-stripe self-check launch is excluded by grid size.

    python profiles/summarize.py --tag r01 --trace gpurun_out/prof_trace \
        --fetch gpurun_out/prof_fetch --write gpurun_out/prof_write
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import shutil
import statistics

HERE = os.path.dirname(os.path.abspath(__file__))
ENCODE = "gf_apply<10, 4, 3,"
DECODE = "gf_apply<10, 1, 4,"
WORKLOAD = "RS(10,4) encode + decode{0}, 4 MiB shards, 96 stripes/GPU"
S, K, M, B = 4 << 20, 10, 4, 96


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def grid(r):
    if "Grid_Size" in r:
        return int(r["Grid_Size"])
    return int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])


def full_grid(rs):
    g = max(grid(r) for r in rs)
    return [r for r in rs if grid(r) == g]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--trace", required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    a = ap.parse_args()

    out = {"workload": WORKLOAD, "source": "rocprofv3 (ROCm 7.2) on MI355X, bench.py defaults", "kernels": {}}
    trace = rows(os.path.join(a.trace, "run_kernel_trace.csv"))
    fetch = rows(os.path.join(a.fetch, "run_counter_collection.csv"))
    write = rows(os.path.join(a.write, "run_counter_collection.csv"))
    for label, name, alg_read, alg_write in (("encode", ENCODE, K * S * B, M * S * B),
                                             ("decode", DECODE, K * S * B, 1 * S * B)):
        tr = full_grid([r for r in trace if name in r["Kernel_Name"]])
        durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in tr]
        fe = full_grid([r for r in fetch if name in r["Kernel_Name"]])
        wr = full_grid([r for r in write if name in r["Kernel_Name"]])
        fetch_kib = statistics.mean(float(r["Counter_Value"]) for r in fe)
        write_kib = statistics.mean(float(r["Counter_Value"]) for r in wr)
        read_b = 2 * fetch_kib * 1024  # gfx950 FETCH_SIZE = 1/2 of streamed bytes
        write_b = write_kib * 1024
        avg_ns = statistics.mean(durs)
        alg = alg_read + alg_write
        out["kernels"][label] = {
            "kernel": name, "launches": len(durs), "avg_duration_ns": round(avg_ns, 1),
            "min_duration_ns": min(durs), "max_duration_ns": max(durs),
            "algorithmic_bytes_per_launch": alg, "achieved_GBps": round(alg / avg_ns, 1),
            "pmc_fetch_kib_raw": round(fetch_kib, 1), "pmc_write_kib_raw": round(write_kib, 1),
            "hbm_read_bytes_corrected": round(read_b), "hbm_write_bytes": round(write_b),
            "hbm_bytes_per_launch": round(read_b + write_b),
            "traffic_over_algorithmic": round((read_b + write_b) / alg, 4),
        }
    with open(os.path.join(HERE, f"{a.tag}_rocprof_summary.json"), "w") as f:
        json.dump(out, f, indent=1)
    enc = out["kernels"]["encode"]
    with open(os.path.join(HERE, "pmc_encode.json"), "w") as f:
        json.dump({"workload": WORKLOAD, "kernel": ENCODE, "hbm_bytes_per_launch": enc["hbm_bytes_per_launch"],
                   "from": f"profiles/{a.tag}_rocprof_summary.json"}, f, indent=1)
    shutil.copy(os.path.join(a.trace, "run_kernel_stats.csv"), os.path.join(HERE, f"{a.tag}_kernel_stats.csv"))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
