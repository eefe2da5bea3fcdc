"""How a launch's time depends on its predecessor (write-back of the
predecessor's dirty lines): RS(10,4) 4 MiB x 24 stripes, encode and decode{0}
timed with HIP events in the sequences E,E,E... / D,D,D... / E,D,E,D... and
with an idle gap (synchronize + sleep) before each launch.

    python tools/probe_sequence.py
"""
from __future__ import annotations

import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import erasure_coding_test_amd as E  # noqa: E402


def main():
    k, m, S, B = 10, 4, 4 << 20, 24
    M = E.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    slab, shards = E.alloc_stripes(B, k, m, S)
    slab.random_(0, 256)
    enc = E.encode_plan(k, m, M).bind([st[:k] for st in shards], [st[k:] for st in shards], S)
    dec = E.DecodePlan(k, m, M, [0]).bind_stripes(shards, S)
    st = torch.cuda.current_stream()
    plans = {"E": enc, "D": dec}
    res = {}
    for name, seq, idle in (("E after E", "EE", False), ("D after D", "DD", False), ("E after D", "DE", False),
                            ("D after E", "ED", False), ("E after idle", "E", True), ("D after idle", "D", True)):
        ts = []
        for it in range(30):
            if idle:
                torch.cuda.synchronize()
                time.sleep(0.002)
            else:
                plans[seq[0]].launch(st.cuda_stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            plans[seq[-1]].launch(st.cuda_stream)
            e1.record(st)
            torch.cuda.synchronize()
            if it >= 5:
                ts.append(e0.elapsed_time(e1))
        nbytes = (k + m) * S * B if seq[-1] == "E" else (k + 1) * S * B
        med = statistics.median(ts)
        res[name] = {"median_ms": round(med, 4), "GBps": round(nbytes / med / 1e6, 1)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
