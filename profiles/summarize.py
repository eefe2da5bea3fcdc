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
and decode{0} (96 stripes), the configs block's other C3 decode shapes (a
seeded single data erasure, XOR-only like decode{0} and so the same kernel:
told apart by launch order -- the timed steps' W + K launches come first,
then the configs entry's CFG_WARMUP + CFG_REPS; and erasure {12}, the dense
re-encode of one parity row), C2 encode (512 stripes), C4 decode{0,1,2,3}
(96 stripes) and C5 encode (24 stripes).

Every record carries the kernel build ID of the library that was profiled
(ecgpu_build_id(1), read from the in-tree libecgpu.so without touching the
GPU); bench.py reports pmc_*.json's traffic only when it matches the library
it runs.

    python profiles/summarize.py --tag r02 --trace gpurun_out/prof_trace \
        --fetch gpurun_out/prof_fetch --write gpurun_out/prof_write
"""
from __future__ import annotations

import argparse
import csv
import ctypes
import json
import os
import shutil
import statistics
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (launch counts of the default command; no GPU touched)

MiB = 1 << 20
_A = bench.parse([])
TIMED = _A.warmup + _A.steps  # timed-loop launches of each kernel (warm-up included)
CFG = bench.CFG_WARMUP + bench.CFG_REPS
# label: (kernel-name prefix, algorithmic read bytes, algorithmic write bytes,
#         (first, end) slice of that kernel's full-grid launches in launch order, or None for all)
KERNELS = {
    "encode": ("gf_apply<10, 4, 3,", 10 * 4 * MiB * 96, 4 * 4 * MiB * 96, None),
    "decode": ("gf_apply<10, 1, 4,", 10 * 4 * MiB * 96, 1 * 4 * MiB * 96, (0, TIMED)),
    "C3_decode_data_random": ("gf_apply<10, 1, 4,", 10 * 4 * MiB * 96, 1 * 4 * MiB * 96, (TIMED, TIMED + CFG)),
    "C3_decode_parity": ("gf_apply<10, 1, 1,", 10 * 4 * MiB * 96, 1 * 4 * MiB * 96, None),
    "C2_encode": ("gf_apply<6, 3, 3,", 6 * MiB * 512, 3 * MiB * 512, None),
    "C4_decode_0123": ("gf_apply<10, 4, 0,", 10 * 4 * MiB * 96, 4 * 4 * MiB * 96, None),
    "C5_encode": ("gf_apply<12, 4, 3,", 12 * 16 * MiB * 24, 4 * 16 * MiB * 24, None),
}
WORKLOAD_KEY = "C3:96"  # bench.py load_traffic key: --config C3, 96 stripes/GPU


def kernel_build_id() -> str:
    lib = ctypes.CDLL(os.path.join(ROOT, "erasure_coding_test_amd", "lib", "libecgpu.so"))
    lib.ecgpu_build_id.restype = ctypes.c_char_p
    lib.ecgpu_build_id.argtypes = [ctypes.c_int]
    return lib.ecgpu_build_id(1).decode()


def in_order(rs):
    """Launch order: dispatch id (counter collection) or start time (trace)."""
    for key in ("Dispatch_Id", "Correlation_Id", "Start_Timestamp"):
        if rs and key in rs[0]:
            return sorted(rs, key=lambda r: int(r[key]))
    return rs


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def grid(r):
    if "Grid_Size" in r:
        return int(r["Grid_Size"])
    return int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])


def full_grid(rs, occ=None):
    """The kernel's largest-grid launches, in launch order, sliced by occ."""
    if not rs:
        return []
    g = max(grid(r) for r in rs)
    out = in_order([r for r in rs if grid(r) == g])
    return out[occ[0]:occ[1]] if occ else out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--trace", required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    a = ap.parse_args()

    kid = kernel_build_id()
    out = {"workload_key": WORKLOAD_KEY, "source": "rocprofv3 (ROCm 7.2) on MI355X, `python3 bench.py` defaults",
           "kernel_build_id": kid, "kernels": {}}
    trace = rows(os.path.join(a.trace, "run_kernel_trace.csv"))
    fetch = rows(os.path.join(a.fetch, "run_counter_collection.csv"))
    write = rows(os.path.join(a.write, "run_counter_collection.csv"))
    for label, (name, alg_read, alg_write, occ) in KERNELS.items():
        tr = full_grid([r for r in trace if name in r["Kernel_Name"]], occ)
        if not tr:
            continue
        durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in tr]
        fe = full_grid([r for r in fetch if name in r["Kernel_Name"]], occ)
        wr = full_grid([r for r in write if name in r["Kernel_Name"]], occ)
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
            json.dump({"workload_key": WORKLOAD_KEY, "kernel": KERNELS[label][0], "kernel_build_id": kid,
                       "hbm_bytes_per_launch": e.get("hbm_bytes_per_launch"),
                       "from": f"profiles/{a.tag}_rocprof_summary.json"}, f, indent=1)
    shutil.copy(os.path.join(a.trace, "run_kernel_stats.csv"), os.path.join(HERE, f"{a.tag}_kernel_stats.csv"))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
