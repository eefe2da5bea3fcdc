"""Summarise rocprofv3 PMC / kernel-trace directories (tools/pmc_dense.sh,
tools/pmc_wide.sh) per kernel: every counter's mean over the kernel's
full-grid launches, the trace's durations, and derived fractions.

    python tools/pmc_summary.py gpurun_out/pmc_dense_* > profiles/r04_pmc_dense.json

Units (MI355X_MICROARCH.md): SQ_*_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* are
quad-cycles summed over waves; GRBM_GUI_ACTIVE is summed over the 8 XCDs;
FETCH_SIZE / WRITE_SIZE in KiB, FETCH doubled (gfx950 reports half of a wide
streaming read).
"""
from __future__ import annotations

import csv
import glob
import json
import os
import statistics
import sys


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def grid(r):
    if "Grid_Size" in r:
        return int(r["Grid_Size"])
    return int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])


def short(name):
    return name.split("(")[0].replace("void ecgpu::dev::", "")


def main(dirs):
    counters, durs = {}, {}
    for d in dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            by = {}
            for r in rows(path):
                by.setdefault(r["Kernel_Name"], []).append(r)
            for k, rs in by.items():
                g = max(grid(r) for r in rs)
                per = {}
                for r in rs:
                    if grid(r) == g:
                        per.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
                c = counters.setdefault(short(k), {})
                for name, vals in per.items():
                    c[name] = statistics.mean(vals)
        for path in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
            by = {}
            for r in rows(path):
                by.setdefault(r["Kernel_Name"], []).append(r)
            for k, rs in by.items():
                g = max(grid(r) for r in rs)
                durs[short(k)] = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rs if grid(r) == g]
    out = {}
    for k in sorted(set(counters) | set(durs)):
        c = counters.get(k, {})
        e = {"counters": {n: round(v, 1) for n, v in sorted(c.items())}}
        if k in durs:
            e["median_duration_ns"] = statistics.median(durs[k])
            e["launches"] = len(durs[k])
        dv = {}
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_VMEM"):
                if n in c:
                    dv[n.lower().replace("sq_", "") + "_frac_of_wave_cycles"] = round(c[n] / wc, 4)
        if "GRBM_GUI_ACTIVE" in c:
            dv["gpu_active_cycles_per_xcd"] = round(c["GRBM_GUI_ACTIVE"] / 8)
            if "median_duration_ns" in e:
                dv["effective_clock_GHz"] = round(c["GRBM_GUI_ACTIVE"] / 8 / e["median_duration_ns"], 3)
        if "SQ_BUSY_CYCLES" in c and "GRBM_GUI_ACTIVE" in c:
            dv["sq_busy_per_gui_active"] = round(c["SQ_BUSY_CYCLES"] / c["GRBM_GUI_ACTIVE"], 4)
        if "SQ_WAVES" in c and wc:
            dv["wave_cycles_per_wave"] = round(wc / c["SQ_WAVES"])
        if "SQ_INSTS_VALU" in c and "SQ_WAVES" in c:
            dv["valu_insts_per_wave"] = round(c["SQ_INSTS_VALU"] / c["SQ_WAVES"], 1) if c["SQ_WAVES"] else None
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            dv["hbm_bytes"] = round((2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024)
        e["derived"] = dv
        out[k] = e
    json.dump({"what": "rocprofv3 PMC passes, one counter group per run; means over each kernel's full-grid launches",
               "dirs": dirs, "kernels": out}, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1:])
