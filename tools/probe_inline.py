"""Inline (gf_apply_inl, tables in the kernel arguments) vs plan launch
(gf_apply, tables in HBM) for one-stripe device-resident calls whose launch
is dense in multiplies: RS(k,4) random-matrix encode, 64 MiB shards.
Run under rocprofv3 --kernel-trace --stats.  The knob ECGPU_INLINE is read
once per process (knobs.hpp), so the two arms are switched in-process with
ecgpu_set_knob between calls and restored at the end.

    rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/inl -o run -- python3 tools/probe_inline.py
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import erasure_coding_test_amd as E  # noqa: E402
from erasure_coding_test_amd import _native as N  # noqa: E402


def main():
    S = 64 << 20
    rng = np.random.default_rng(5)
    for k in (10, 14, 16):
        m = 4
        M = [int(x) for x in rng.integers(2, 256, k * m)]  # every coefficient a multiply
        data = [torch.randint(0, 256, (S,), dtype=torch.uint8, device="cuda") for _ in range(k)]
        coding = [torch.empty(S, dtype=torch.uint8, device="cuda") for _ in range(m)]
        ref = None
        for rnd in range(3):
            for inl in ("1", "0"):
                N.set_knob("ECGPU_INLINE", int(inl))
                for _ in range(5):
                    E.jerasure.jerasure_matrix_encode(k, m, 8, M, data, coding, S)
                torch.cuda.synchronize()
                out = torch.stack(coding).cpu()
                if ref is None:
                    ref = out
                assert torch.equal(out, ref), (k, inl)
        print(f"k={k}: inline and plan outputs equal")
    N.reset_knob("ECGPU_INLINE")


if __name__ == "__main__":
    main()
