"""w = 16 / 32 column-engine probe for PMC passes: RS(10,4) encode of one
stripe of 64 MiB device-resident shards, `--reps` calls per width.

    rocprofv3 --pmc <counters> -- python3 tools/probe_wide.py [--w 32] [--reps 5]
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import erasure_coding_test_amd as E  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--w", type=int, nargs="+", default=[16, 32])
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--shard-mib", type=int, default=64)
    a = ap.parse_args()
    k, m, S = 10, 4, a.shard_mib << 20
    data = [torch.randint(0, 256, (S,), dtype=torch.uint8, device="cuda") for _ in range(k)]
    coding = [torch.empty(S, dtype=torch.uint8, device="cuda") for _ in range(m)]
    for w in a.w:
        M = E.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, w)
        for _ in range(a.reps):
            E.jerasure.jerasure_matrix_encode(k, m, w, M, data, coding, S)
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
