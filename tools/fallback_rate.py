"""Throughput of the CPU fallback (csrc/cpu_fallback.cpp) through the drop-in,
beside the reference compiled here (oracle/_ref, as the yardstick): RS(10,4)
4 MiB encode and decode{0,1,2,3}, one thread.  The fallback only runs after a
HIP error; this says how fast a datanode keeps going then.

    ECGPU_CPU_FALLBACK=1 ECGPU_TEST_INJECT_HIP=2 python tools/fallback_rate.py
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


def rate(f, k, m, size, reps=5):
    M = matrix(f, k, m)
    rng = np.random.default_rng(1)
    data = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(k)]
    coding = [np.zeros(size, np.uint8) for _ in range(m)]
    f["encode"](k, m, 8, ints(M), ptrs(data), ptrs(coding), size)
    t0 = time.perf_counter()
    for _ in range(reps):
        f["encode"](k, m, 8, ints(M), ptrs(data), ptrs(coding), size)
    enc = reps * k * size / (time.perf_counter() - t0) / 2**30
    t0 = time.perf_counter()
    for _ in range(reps):
        assert f["decode"](k, m, 8, ints(M), 0, ints([0, 1, 2, 3, -1]), ptrs(data), ptrs(coding), size) == 0
    dec = reps * k * size / (time.perf_counter() - t0) / 2**30
    return round(enc, 2), round(dec, 2)


def main():
    k, m, size = 10, 4, 4 << 20
    fb = bind(os.path.join(LIB, "libjerasure_amd.so"))
    ref = bind(os.path.join(REF, "libjerasure_ref.so"))
    e1, d1 = rate(fb, k, m, size)
    e2, d2 = rate(ref, k, m, size)
    core = ctypes.CDLL(os.path.join(LIB, "libecgpu.so"))
    core.ecgpu_fallback_count.restype = ctypes.c_int64
    print(json.dumps({"workload": "RS(10,4) 4 MiB, one thread, pageable buffers", "unit": "GiB/s of data",
                      "fallback_encode": e1, "fallback_decode_0123": d1,
                      "reference_O2_encode": e2, "reference_O2_decode_0123": d2,
                      "fallbacks": int(core.ecgpu_fallback_count())}))


if __name__ == "__main__":
    main()
