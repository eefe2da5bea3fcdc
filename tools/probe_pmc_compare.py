"""Kernel vs its XOR stream probe, per dispatch (round 5):
median duration from a plain kernel trace and, from PMC passes that also
carry --kernel-trace, the effective clock (GRBM_GUI_ACTIVE / 8 XCDs /
duration), the share of wave cycles issuing VALU, waiting to issue, waiting on
anything, and the mean number of DRAM read requests in flight
(TCC_EA0_RDREQ_LEVEL / GRBM_GUI_ACTIVE).  Full-grid dispatches only.

    python tools/probe_pmc_compare.py gpurun_out/r05b > profiles/r05_probe_pmc.json
"""
import csv
import glob
import json
import os
import statistics
import sys

PAIRS = [("C2 encode RS(6,3) 1 MiB x 512", "gf_apply<6, 3, 3,", "diag_xor_mix<6, 3>"),
         ("lost parity {12}, RS(10,4) 4 MiB x 96", "gf_apply<10, 1, 1,", "diag_xor_mix<10, 1>"),
         ("C3 encode RS(10,4) 4 MiB x 96", "gf_apply<10, 4, 3,", "diag_xor_mix<10, 4>"),
         ("C4 decode{0,1,2,3}", "gf_apply<10, 4, 0,", "diag_xor_mix<10, 4>")]


def rows(p):
    with open(p) as f:
        return list(csv.DictReader(f))


def grid(r):
    return int(r.get("Grid_Size") or 0) or int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])


def dispatches(d, match, residency=None):
    """The full-grid dispatches of `match` under directory d, in launch order,
    each {"us": .., counters...}.  residency (0 uncapped, 3, 4): only the
    probe's dispatches at that residency -- bench.xor_stream_probe runs each
    of uncapped / 3 / 4 per CU in turn, 2 warm-ups + REPS launches each."""
    out = {}
    for tp in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        tr = [r for r in rows(tp) if match in r["Kernel_Name"]]
        if not tr:
            continue
        g = max(grid(r) for r in tr)
        for r in tr:
            if grid(r) == g:
                out[(tp, int(r["Dispatch_Id"]))] = {"us": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3}
        for cp in glob.glob(os.path.join(os.path.dirname(tp), "*counter_collection.csv")):
            for r in rows(cp):
                key = (tp, int(r["Dispatch_Id"]))
                if key in out:
                    out[key][r["Counter_Name"]] = float(r["Counter_Value"])
    if residency is None:
        return list(out.values())
    keep = []
    for tp in sorted({k[0] for k in out}):
        seq = [out[k] for k in sorted(k for k in out if k[0] == tp)]
        per = 2 + REPS
        keep += [x for i, x in enumerate(seq) if (0, 3, 4)[(i // per) % 3] == residency]
    return keep


REPS = 8  # tools/c4_spread.sh / session_r05_b.sh: probe_dense --reps 8


def med(xs):
    xs = [x for x in xs if x is not None]
    return round(statistics.median(xs), 4) if xs else None


def summary(ds_trace, ds_pmc):
    def f(d, num, den):
        return d[num] / d[den] if num in d and den in d and d[den] else None
    return {
        "launches_timed": len(ds_trace), "median_us": med([d["us"] for d in ds_trace]),
        "eff_clock_MHz": med([f(d, "GRBM_GUI_ACTIVE", "us") and d["GRBM_GUI_ACTIVE"] / 8 / d["us"] for d in ds_pmc]),
        "valu_share": med([f(d, "SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES") for d in ds_pmc]),
        "wait_inst_share": med([f(d, "SQ_WAIT_INST_ANY", "SQ_WAVE_CYCLES") for d in ds_pmc]),
        "wait_any_share": med([f(d, "SQ_WAIT_ANY", "SQ_WAVE_CYCLES") for d in ds_pmc]),
        "dram_reads_in_flight": med([f(d, "TCC_EA0_RDREQ_LEVEL_sum", "GRBM_GUI_ACTIVE") for d in ds_pmc]),
        "dram_credit_stall_per_kcycle": med([f(d, "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum", "GRBM_GUI_ACTIVE") and
                                             1e3 * d["TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum"] / d["GRBM_GUI_ACTIVE"]
                                             for d in ds_pmc]),
    }


def main(d):
    out = {"source": f"rocprofv3 over tools/probe_dense.py --pmc --probes ({d})", "pairs": {}}
    trace = os.path.join(d, "probe_trace")
    pmc = [os.path.join(d, x) for x in ("probe_sq", "probe_tcc")]
    for name, kern, probe in PAIRS:
        e = {}
        tr = dispatches(trace, kern)
        e["kernel"] = summary(tr, [x for p in pmc for x in dispatches(p, kern)])
        e["kernel"]["name"] = kern
        for res in (0, 3, 4):
            tr = dispatches(trace, probe, res)
            e[f"probe_{res or 'uncapped'}"] = summary(tr, [x for p in pmc for x in dispatches(p, probe, res)])
        best = min((k for k in e if k.startswith("probe_")), key=lambda k: e[k]["median_us"] or 1e9)
        e["best_probe"] = best
        e["probe_time_over_kernel"] = round(e[best]["median_us"] / e["kernel"]["median_us"], 4)
        out["pairs"][name] = e
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
