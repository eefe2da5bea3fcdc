"""Throughput of the library's CPU executor (csrc/cpu_exec.cpp) through the
drop-in's mangled names, at each SIMD level the host has, beside the
reference compiled here (oracle/_ref, as the yardstick): RS(10,4) 4 MiB
encode and decode{0,1,2,3}, one thread, pageable buffers.  The executor runs
small host-memory calls (below ECGPU_MIN_OFFLOAD_KIB), every host-memory call
with ECGPU_GPU=0, and the §8b fallback after a HIP error; this says how fast.

    python tools/cpu_exec_rate.py          -> one JSON line
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from fallback_driver import LIB, REF, bind, ints, matrix, ptrs  # noqa: E402


def rate(f, k, m, size, reps):
    M = matrix(f, k, m)
    rng = np.random.default_rng(1)
    data = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(k)]
    coding = [np.zeros(size, np.uint8) for _ in range(m)]
    f["encode"](k, m, 8, ints(M), ptrs(data), ptrs(coding), size)
    t0 = time.perf_counter()
    for _ in range(reps):
        f["encode"](k, m, 8, ints(M), ptrs(data), ptrs(coding), size)
    enc = reps * k * size / (time.perf_counter() - t0) / 2**30
    keep = [d.copy() for d in data[:4]]
    t0 = time.perf_counter()
    for _ in range(reps):
        assert f["decode"](k, m, 8, ints(M), 0, ints([0, 1, 2, 3, -1]), ptrs(data), ptrs(coding), size) == 0
    dec = reps * k * size / (time.perf_counter() - t0) / 2**30
    assert all(np.array_equal(a, b) for a, b in zip(keep, data[:4]))
    return round(enc, 2), round(dec, 2)


def main():
    k, m, size = 10, 4, 4 << 20
    d = bind(os.path.join(LIB, "libjerasure_amd.so"))
    core = ctypes.CDLL(os.path.join(LIB, "libecgpu.so"))
    core.ecgpu_set_knob.argtypes = [ctypes.c_char_p, ctypes.c_int]
    core.ecgpu_get_knob.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]
    core.ecgpu_cpu_call_count.restype = ctypes.c_int64
    core.ecgpu_fallback_count.restype = ctypes.c_int64
    assert core.ecgpu_set_knob(b"ECGPU_GPU", 0) == 0
    out = {"workload": "RS(10,4) 4 MiB, one thread, pageable buffers", "unit": "GiB/s of data"}
    for level, name in ((2, "avx512_gfni"), (1, "avx2_nibble"), (0, "scalar")):
        core.ecgpu_set_knob(b"ECGPU_CPU_SIMD", level)
        e, dd = rate(d, k, m, size, 20 if level else 3)
        out[f"executor_{name}_encode"], out[f"executor_{name}_decode_0123"] = e, dd
    for lib, name in (("libjerasure_ref.so", "reference_O2"), ("libjerasure_ref_o3.so", "reference_O3")):
        path = os.path.join(REF, lib)
        if os.path.exists(path):
            e, dd = rate(bind(path), k, m, size, 3)
            out[f"{name}_encode"], out[f"{name}_decode_0123"] = e, dd
    out["cpu_calls"] = int(core.ecgpu_cpu_call_count())
    out["fallbacks"] = int(core.ecgpu_fallback_count())
    print(json.dumps(out))


if __name__ == "__main__":
    main()
