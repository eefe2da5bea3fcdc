"""Seeded fuzz of the CPU fallback (csrc/cpu_fallback.cpp) against the
reference compiled here (oracle/_ref, the checker): random synchronous calls
through libjerasure_amd.so's mangled names -- matrix encode (k 1..20, m 1..8,
coefficients with zeros and ones), decode of up to m + 1 erasures (return codes
too), dot products with and without src_ids, region multiply / XOR -- at
sizes in whole 8-byte words up to 256 KiB, a quarter of them with buffers
repeated inside the call (identical pointers: the reference's sequential
semantics).  Run by tests/test_cpu_fallback.py with ECGPU_CPU_FALLBACK=1 and
ECGPU_TEST_INJECT_HIP set, so every call completes on the CPU, and by
tests/test_cpu_exec.py with ECGPU_GPU=0 (every call on the CPU executor by
choice) at each ECGPU_CPU_SIMD level.

    python tests/fallback_fuzz.py [cases] [seed]     -> one JSON line, exit 0 if all matched
"""
from __future__ import annotations

import ctypes
import json
import os
import sys

import numpy as np

TESTS = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(TESTS)
sys.path.insert(0, TESTS)
sys.path.insert(0, ROOT)
from fallback_driver import LIB, REF, bind, ints, matrix, ptrs, set_injection  # noqa: E402

SIZES = [8, 24, 4096, 4104, 65536, 100000, 262144]


def main():
    cases = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 20261017
    d = bind(os.path.join(LIB, "libjerasure_amd.so"))
    r = bind(os.path.join(REF, "libjerasure_ref.so"))
    core = ctypes.CDLL(os.path.join(LIB, "libecgpu.so"))
    set_injection(core)
    rng = np.random.default_rng(seed)
    bad, kinds = [], {"encode": 0, "decode": 0, "dotprod": 0, "region": 0, "aliased": 0}
    for case in range(cases):
        kind = ("encode", "decode", "dotprod", "region")[int(rng.integers(0, 4))]
        size = int(rng.choice(SIZES))
        if size == 100000:
            size = 8 * int(rng.integers(1, 100000 // 8))
        kinds[kind] += 1
        if kind in ("encode", "dotprod"):
            k, m = int(rng.integers(1, 21 if kind == "encode" else 17)), int(rng.integers(1, 9))
            M = [int(x) for x in rng.choice([0, 1, 2, 3, 0x8E, int(rng.integers(0, 256))], size=k * m)]
            pool = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(k + m)]
            owner = list(range(k + m))
            if rng.random() < 0.25:  # identical pointers: a buffer passed twice
                kinds["aliased"] += 1
                for i in range(1, k + m):
                    if rng.random() < 0.25:
                        owner[i] = int(rng.integers(0, i))
            row = M[:k]
            src_ids = [int(x) for x in rng.permutation(k + m)[:k]] if kind == "dotprod" and rng.random() < 0.5 else None
            dest = int(rng.integers(0, k + m))
            if src_ids is not None and dest in src_ids:
                dest = next(i for i in range(k + m) if i not in src_ids)
            outs = []
            for lib in (d, r):
                bufs = {u: pool[u].copy() for u in set(owner)}
                arr = [bufs[o] for o in owner]
                if kind == "encode":
                    lib["encode"](k, m, 8, ints(M), ptrs(arr[:k]), ptrs(arr[k:]), size)
                else:
                    lib["dotprod"](k, 8, ints(row), None if src_ids is None else ints(src_ids), dest,
                                   ptrs(arr[:k]), ptrs(arr[k:]), size)
                outs.append([bufs[u] for u in sorted(bufs)])
            if not all(np.array_equal(a, b) for a, b in zip(*outs)):
                bad.append((case, kind, k, m, size, owner))
        elif kind == "decode":
            k, m = int(rng.integers(2, 17)), int(rng.integers(1, 9))
            M = matrix(r, k, m)
            ne = int(rng.integers(1, m + 2))
            er = sorted(int(x) for x in rng.choice(k + m, size=min(ne, k + m), replace=False))
            rko = int(rng.integers(0, 2))
            stripe = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(k + m)]
            r["encode"](k, m, 8, ints(M), ptrs(stripe[:k]), ptrs(stripe[k:]), size)
            for e in er:
                stripe[e][:] = rng.integers(0, 256, size, dtype=np.uint8)
            outs, rcs = [], []
            for lib in (d, r):
                b = [s.copy() for s in stripe]
                rcs.append(lib["decode"](k, m, 8, ints(M), rko, ints(er + [-1]), ptrs(b[:k]), ptrs(b[k:]), size))
                outs.append(b)
            if rcs[0] != rcs[1] or not all(np.array_equal(a, b) for a, b in zip(*outs)):
                bad.append((case, kind, k, m, size, er, rko, rcs))
        else:
            a = rng.integers(0, 256, size, dtype=np.uint8)
            b = rng.integers(0, 256, size, dtype=np.uint8)
            c, op = int(rng.integers(0, 256)), int(rng.integers(0, 4))
            outs = []
            for lib in (d, r):
                x, y, z = a.copy(), b.copy(), np.zeros(size, np.uint8)
                if op == 0:
                    lib["rmul8"](x.ctypes.data, c, size, y.ctypes.data, 0)
                elif op == 1:
                    lib["rmul8"](x.ctypes.data, c, size, y.ctypes.data, 1)
                elif op == 2:
                    lib["rmul8"](x.ctypes.data, c, size, None, 0)  # in place
                else:
                    lib["rxor"](x.ctypes.data, y.ctypes.data, x.ctypes.data, size)  # r3 == r1
                    lib["rxor"](x.ctypes.data, y.ctypes.data, z.ctypes.data, size)
                outs.append((x, y, z))
            if not all(np.array_equal(p, q) for p, q in zip(*outs)):
                bad.append((case, kind, op, c, size))
    core.ecgpu_fallback_count.restype = ctypes.c_int64
    core.ecgpu_cpu_call_count.restype = ctypes.c_int64
    print(json.dumps({"cases": cases, "kinds": kinds, "mismatches": [str(b) for b in bad[:10]],
                      "fallbacks": int(core.ecgpu_fallback_count()), "cpu_calls": int(core.ecgpu_cpu_call_count())}),
          flush=True)
    return 0 if not bad else 3


if __name__ == "__main__":
    sys.exit(main())
