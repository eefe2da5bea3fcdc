"""CPU reference rates for the synchronous drop-in comparison.

The reference's own src/erasure_coding (oracle/_ref, compiled -O2 here and
shipped with the tree -- test infrastructure, timed like bench.py's
cpu_baseline leg) encoding one stripe, at 1 thread and at 16 threads each
pinned to its own CPU, splitting byte ranges like the reference client's
encode_mul_thread (client_main.cpp:1074-1164).  Prints one JSON line per
config: GiB/s of data shards.

    python tools/cpu_reference_rates.py
"""
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle.oracle import Reference, alloc_shards  # noqa: E402


def rate(o, k, m, S, threads, seconds=2.0, erasures=None):
    M = o.vandermonde_coding_matrix(k, m)
    rng = np.random.default_rng(0)
    data = alloc_shards(k, S)
    for d in data:
        d[:S] = rng.integers(0, 256, S, dtype=np.uint8)
    coding = alloc_shards(m, S)
    cpus = sorted(os.sched_getaffinity(0))[:16]
    threads = min(threads, len(cpus))
    ranges, off = [], 0
    for t in range(threads):
        n = S // threads + (S % threads if t == 0 else 0)
        ranges.append((off, n))
        off += n

    def views(bufs, a, n):
        return [np.frombuffer((ctypes.c_uint8 * (n + 16)).from_address(b.ctypes.data + a), dtype=np.uint8) for b in bufs]

    parts = [(views(data, a, n), views(coding, a, n), n) for a, n in ranges]

    def run(t):
        os.sched_setaffinity(0, {cpus[t]})
        d, c, n = parts[t]
        if erasures:
            o.matrix_decode(k, m, M, 0, erasures, d, c, n)
        else:
            o.matrix_encode(k, m, M, d, c, n)

    if erasures:
        o.matrix_encode(k, m, M, data, coding, S)
    iters, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        ts = [threading.Thread(target=run, args=(t,)) for t in range(threads)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        iters += 1
    el = time.perf_counter() - t0
    return iters * k * S / el / 2**30, el / iters * 1e6


def main():
    o = Reference()
    for name, k, m, S, er in (("C1 RS(4,2) 64 KiB encode", 4, 2, 64 << 10, None),
                              ("default RS(3,3) 1 MiB encode", 3, 3, 1 << 20, None),
                              ("C2 RS(6,3) 1 MiB encode", 6, 3, 1 << 20, None),
                              ("C3 RS(10,4) 4 MiB encode", 10, 4, 4 << 20, None),
                              ("C3 RS(10,4) 4 MiB decode{0}", 10, 4, 4 << 20, [0]),
                              ("C4 RS(10,4) 4 MiB decode{0,1,2,3}", 10, 4, 4 << 20, [0, 1, 2, 3]),
                              ("C5 RS(12,4) 16 MiB encode", 12, 4, 16 << 20, None)):
        out = {"case": name}
        for th in (1, 16):
            g, us = rate(o, k, m, S, th, erasures=er)
            out[f"t{th}_GiBps"] = round(g, 3)
            out[f"t{th}_us_per_call"] = round(us, 1)
        out["source"] = "reference src/erasure_coding g++ -O2 (oracle/_ref), threads pinned, byte ranges split like " \
                        "client_main.cpp:1074-1164"
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
