"""Summarise rocprofv3 outputs of a default bench.py run into profiles/<tag>_*.json.

Inputs (written on the GPU box under gpurun_out/):
  <trace>/run_kernel_stats.csv, <trace>/run_kernel_trace.csv
      from  rocprofv3 --kernel-trace --stats --output-format csv -- python3 bench.py
  <fetch>/run_counter_collection.csv   from  rocprofv3 --pmc FETCH_SIZE -- python3 bench.py
  <write>/run_counter_collection.csv   from  rocprofv3 --pmc WRITE_SIZE -- python3 bench.py

HBM-traffic correction (MI355X_MICROARCH.md §HBM): on gfx950 FETCH_SIZE
reports exactly half of the bytes of a wide coalesced streaming read, so the
read side is doubled; WRITE_SIZE is exact for 16-B/lane streaming stores.
Both counters are in KiB.  Per kernel only the full-size launches (the
largest grid of that kernel name) are averaged, so the bench's one-stripe
self-check launches are excluded.

Kernels: every launch shape of the default bench line -- the timed C3 encode
and decode{0} (96 stripes) and the configs block's C2 encode (512 stripes),
C4 decode{0,1,2,3} (96 stripes) and C5 encode (24 stripes).

    python profiles/summarize.py --tag r02 --trace gpurun_out/prof_trace \
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
MiB = 1 << 20
# label: (kernel-name prefix, algorithmic read bytes, algorithmic write bytes)
KERNELS = {
    "encode": ("gf_apply<10, 4, 3,", 10 * 4 * MiB * 96, 4 * 4 * MiB * 96),
    "decode": ("gf_apply<10, 1, 4,", 10 * 4 * MiB * 96, 1 * 4 * MiB * 96),
    "C2_encode": ("gf_apply<6, 3, 3,", 6 * MiB * 512, 3 * MiB * 512),
    "C4_decode_0123": ("gf_apply<10, 4, 0,", 10 * 4 * MiB * 96, 4 * 4 * MiB * 96),
    "C5_encode": ("gf_apply<12, 4, 3,", 12 * 16 * MiB * 24, 4 * 16 * MiB * 24),
}
WORKLOAD_KEY = "C3:96"  # bench.py load_traffic key: --config C3, 96 stripes/GPU


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def grid(r):
    if "Grid_Size" in r:
        return int(r["Grid_Size"])
    return int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])


def full_grid(rs):
    if not rs:
        return []
    g = max(grid(r) for r in rs)
    return [r for r in rs if grid(r) == g]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--trace", required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    a = ap.parse_args()

    out = {"workload_key": WORKLOAD_KEY, "source": "rocprofv3 (ROCm 7.2) on MI355X, `python3 bench.py` defaults",
           "kernels": {}}
    trace = rows(os.path.join(a.trace, "run_kernel_trace.csv"))
    fetch = rows(os.path.join(a.fetch, "run_counter_collection.csv"))
    write = rows(os.path.join(a.write, "run_counter_collection.csv"))
    for label, (name, alg_read, alg_write) in KERNELS.items():
        tr = full_grid([r for r in trace if name in r["Kernel_Name"]])
        if not tr:
            continue
        durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in tr]
        fe = full_grid([r for r in fetch if name in r["Kernel_Name"]])
        wr = full_grid([r for r in write if name in r["Kernel_Name"]])
        alg = alg_read + alg_write
        e = {"kernel": tr[0]["Kernel_Name"], "launches": len(durs), "avg_duration_ns": round(statistics.mean(durs), 1),
             "median_duration_ns": statistics.median(durs), "min_duration_ns": min(durs), "max_duration_ns": max(durs),
             "algorithmic_bytes_per_launch": alg,
             "achieved_GBps_median": round(alg / statistics.median(durs), 1)}
        if fe and wr:
            fetch_kib = statistics.mean(float(r["Counter_Value"]) for r in fe)
            write_kib = statistics.mean(float(r["Counter_Value"]) for r in wr)
            read_b = 2 * fetch_kib * 1024  # gfx950 FETCH_SIZE = 1/2 of streamed bytes
            write_b = write_kib * 1024
            e.update({"pmc_fetch_kib_raw": round(fetch_kib, 1), "pmc_write_kib_raw": round(write_kib, 1),
                      "hbm_read_bytes_corrected": round(read_b), "hbm_write_bytes": round(write_b),
                      "hbm_bytes_per_launch": round(read_b + write_b),
                      "traffic_over_algorithmic": round((read_b + write_b) / alg, 4)})
        out["kernels"][label] = e
    with open(os.path.join(HERE, f"{a.tag}_rocprof_summary.json"), "w") as f:
        json.dump(out, f, indent=1)
    for label in ("encode", "decode"):
        e = out["kernels"].get(label, {})
        with open(os.path.join(HERE, f"pmc_{label}.json"), "w") as f:
            json.dump({"workload_key": WORKLOAD_KEY, "kernel": KERNELS[label][0],
                       "hbm_bytes_per_launch": e.get("hbm_bytes_per_launch"),
                       "from": f"profiles/{a.tag}_rocprof_summary.json"}, f, indent=1)
    shutil.copy(os.path.join(a.trace, "run_kernel_stats.csv"), os.path.join(HERE, f"{a.tag}_kernel_stats.csv"))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
