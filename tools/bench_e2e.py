"""Host-memory (PCIe-inclusive) and per-config measurements for DESIGN.md.

Not the headline (bench.py is); these are the rates a caller whose shards
originate and terminate in host memory sees, and the other BASELINE configs.

  e2e_pinned   RS(10,4) 4 MiB stripes in pinned host memory: H2D of the 10
               data shards on a copy stream, encode on the compute stream,
               D2H of the 4 parity shards on a second copy stream; 3-deep
               ring of device stripe buffers so copies overlap compute.
  e2e_pipeline same stripes through the C-level HostPipeline
               (ecgpu_pipeline_*): per-shard H2D/D2H on its own streams,
               pinned and pageable source buffers.
  e2e_read_pipeline  the read path: ecgpu_pipeline_create_decode over the
               same pinned stripes (10 survivors in, erased shards out).
  dropin_pageable  jerasure_matrix_encode / _decode straight on malloc'd
               (pageable) numpy buffers through the C ABI -- the reference
               client's call shape (client_main.cpp:1060, :2118).
  configs      device-resident C2 RS(6,3) 1 MiB, C3 decode{0}, C4 decode
               {0,1,2,3}, C5 RS(12,4) 16 MiB encode (kernel time, HBM GB/s).
  pcie         raw pinned H2D / D2H copy rates (the ceiling for e2e).
  pcie_duplex  H2D and D2H at once in the 10:4 proportion (the e2e write path's PCIe ceiling).

    python tools/bench_e2e.py [--stripes 48]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import erasure_coding_test_amd as E  # noqa: E402

GiB = 2**30


def timed_events(fn, reps=10, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / 1e3)
    return statistics.median(ts)


def pcie_rates(nbytes=1 << 30):
    h = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    d = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    h2d = timed_events(lambda: d.copy_(h, non_blocking=True), reps=5)
    d2h = timed_events(lambda: h.copy_(d, non_blocking=True), reps=5)
    return {"h2d_GBps": round(nbytes / h2d / 1e9, 1), "d2h_GBps": round(nbytes / d2h / 1e9, 1)}


def pcie_duplex(k=10, m=4, S=4 << 20, stripes=48):
    """Both directions at once in the write path's 10:4 proportion: k*S*stripes
    H2D on one stream while m*S*stripes go D2H on another (pinned, one copy
    each).  The data rate (k*S per stripe / wall time) is the PCIe-only
    ceiling of the e2e write path."""
    hi = torch.empty(k * S * stripes, dtype=torch.uint8).pin_memory()
    ho = torch.empty(m * S * stripes, dtype=torch.uint8).pin_memory()
    di = torch.empty(k * S * stripes, dtype=torch.uint8, device="cuda")
    do = torch.empty(m * S * stripes, dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def both():
        with torch.cuda.stream(s1):
            di.copy_(hi, non_blocking=True)
        with torch.cuda.stream(s2):
            ho.copy_(do, non_blocking=True)
        s1.synchronize()
        s2.synchronize()
    both()
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        both()
        ts.append(time.perf_counter() - t0)
    t = statistics.median(ts)
    return {"data_GiBps": round(k * S * stripes / t / GiB, 1), "h2d_GBps": round(k * S * stripes / t / 1e9, 1),
            "d2h_GBps_while": round(m * S * stripes / t / 1e9, 1)}


def e2e_pinned(stripes=48, k=10, m=4, S=4 << 20, ring=3):
    """Pinned host stripes [s][k+m][S]; device ring of `ring` contiguous
    stripe buffers so each stripe moves as ONE k*S H2D copy and ONE m*S D2H
    copy (PCIe-bound: layout skew is irrelevant here)."""
    M = E.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    host = torch.empty((stripes, k + m, S), dtype=torch.uint8).pin_memory()
    host[:, :k].random_(0, 256)
    slots = []
    for _ in range(ring):
        buf = torch.empty((k + m, S), dtype=torch.uint8, device="cuda")
        plan = E.encode_plan(k, m, M).bind([[buf[j] for j in range(k)]], [[buf[k + i] for i in range(m)]], S)
        slots.append((buf, plan))
    comp = torch.cuda.current_stream()
    h2d, d2h = torch.cuda.Stream(), torch.cuda.Stream()
    loaded = [torch.cuda.Event() for _ in range(ring)]
    computed = [torch.cuda.Event() for _ in range(ring)]
    drained = [torch.cuda.Event() for _ in range(ring)]

    def run():
        for s in range(stripes):
            r = s % ring
            buf, plan = slots[r]
            with torch.cuda.stream(h2d):
                h2d.wait_event(drained[r])
                buf[:k].copy_(host[s, :k], non_blocking=True)
                loaded[r].record(h2d)
            comp.wait_event(loaded[r])
            plan.launch(comp.cuda_stream)
            computed[r].record(comp)
            with torch.cuda.stream(d2h):
                d2h.wait_event(computed[r])
                host[s, k:].copy_(buf[k:], non_blocking=True)
                drained[r].record(d2h)
        torch.cuda.synchronize()

    run()
    t0 = time.perf_counter()
    run()
    t = time.perf_counter() - t0
    ref = torch.empty((m, S), dtype=torch.uint8, device="cuda")
    d = host[stripes - 1, :k].cuda()
    E.encode_plan(k, m, M).bind([[d[j] for j in range(k)]], [[ref[i] for i in range(m)]], S).launch()
    torch.cuda.synchronize()
    ok = bool(torch.equal(ref.cpu(), host[stripes - 1, k:]))
    return {"workload": f"RS(10,4) 4 MiB encode, {stripes} stripes pinned host -> HBM -> pinned host",
            "data_GiBps": round(stripes * k * S / t / GiB, 2),
            "h2d_GBps": round(stripes * k * S / t / 1e9, 1), "parity_ok": ok}


def e2e_pipeline(stripes=48, k=10, m=4, S=4 << 20, depth=3, pinned=True, devices=None):
    """devices: None = HostPipeline on the current device; a list = the
    multi-device HostPipelineGroup over those ordinals (round-robin stripes)."""
    M = E.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    host = torch.empty((stripes, k + m, S), dtype=torch.uint8)
    if pinned:
        host = host.pin_memory()
    host[:, :k].random_(0, 256)
    p = E.HostPipeline(k, m, M, S, depth=depth) if devices is None else E.HostPipelineGroup(
        k, m, M, S, devices=devices, depth=depth)

    def run():
        for s in range(stripes):
            p.submit([host[s, j] for j in range(k)], [host[s, k + i] for i in range(m)])
        p.drain()

    run()
    t0 = time.perf_counter()
    run()
    t = time.perf_counter() - t0
    p.close()
    ref = torch.empty((m, S), dtype=torch.uint8, device="cuda")
    d = host[stripes - 1, :k].cuda()
    E.encode_plan(k, m, M).bind([[d[j] for j in range(k)]], [[ref[i] for i in range(m)]], S).launch()
    torch.cuda.synchronize()
    ok = bool(torch.equal(ref.cpu(), host[stripes - 1, k:]))
    via = "ecgpu_pipeline" if devices is None else f"ecgpu_pipeline_group over devices {devices}"
    return {"workload": f"RS(10,4) 4 MiB encode via {via}, {stripes} stripes "
                        f"{'pinned' if pinned else 'pageable'} host, depth {depth}",
            "data_GiBps": round(stripes * k * S / t / GiB, 2), "parity_ok": ok}


def e2e_read_pipeline(erasures, stripes=48, k=10, m=4, S=4 << 20, depth=3):
    """Read path: survivors pinned host -> HBM -> decode -> erased shards back."""
    M = E.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    host = torch.empty((stripes, k + m, S), dtype=torch.uint8).pin_memory()
    host[:, :k].random_(0, 256)
    enc = E.HostPipeline(k, m, M, S, depth=depth)
    for s in range(stripes):
        enc.submit([host[s, j] for j in range(k)], [host[s, k + i] for i in range(m)])
    enc.drain()
    enc.close()
    want = host[stripes - 1].clone()
    p = E.HostPipeline.decoder(k, m, M, erasures, S, depth=depth)

    def run():
        for s in range(stripes):
            p.submit([host[s, j] for j in range(k)], [host[s, k + i] for i in range(m)])
        p.drain()

    run()
    host[stripes - 1, erasures] = 0
    t0 = time.perf_counter()
    run()
    t = time.perf_counter() - t0
    p.close()
    return {"workload": f"RS(10,4) 4 MiB decode {erasures} via ecgpu_pipeline_create_decode, {stripes} stripes "
                        f"pinned host, depth {depth}",
            "data_GiBps": round(stripes * k * S / t / GiB, 2), "parity_ok": bool(torch.equal(host[stripes - 1], want))}


def dropin_pageable(k=10, m=4, S=4 << 20, reps=5):
    M = E.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    rng = np.random.default_rng(0)
    data = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
    coding = [np.zeros(S, np.uint8) for _ in range(m)]
    E.jerasure.jerasure_matrix_encode(k, m, 8, M, data, coding, S)
    t0 = time.perf_counter()
    for _ in range(reps):
        E.jerasure.jerasure_matrix_encode(k, m, 8, M, data, coding, S)
    te = (time.perf_counter() - t0) / reps
    bufs = data + coding
    saved = bufs[0].copy()
    t0 = time.perf_counter()
    for _ in range(reps):
        bufs[0][:] = 0
        E.jerasure.jerasure_matrix_decode(k, m, 8, M, 0, [0], bufs[:k], bufs[k:], S)
    td = (time.perf_counter() - t0) / reps
    return {"workload": "jerasure_matrix_encode/decode{0} on pageable malloc buffers, RS(10,4) 4 MiB, synchronous",
            "encode_ms": round(te * 1e3, 2), "encode_data_GiBps": round(k * S / te / GiB, 2),
            "decode_ms": round(td * 1e3, 2), "decode_ok": bool(np.array_equal(bufs[0], saved))}


def dropin_pinned(k=10, m=4, S=4 << 20, reps=10):
    """Synchronous jerasure_matrix_encode / decode{0} on pinned host buffers
    (torch pin_memory = hipHostMalloc): the kernel reads and writes them in
    place (ECGPU_ZC_PINNED, default on) -- no staging DMA."""
    M = E.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    data = [torch.randint(0, 256, (S,), dtype=torch.uint8).pin_memory() for _ in range(k)]
    coding = [torch.zeros(S, dtype=torch.uint8).pin_memory() for _ in range(m)]
    E.jerasure.jerasure_matrix_encode(k, m, 8, M, data, coding, S)
    t0 = time.perf_counter()
    for _ in range(reps):
        E.jerasure.jerasure_matrix_encode(k, m, 8, M, data, coding, S)
    te = (time.perf_counter() - t0) / reps
    bufs = data + coding
    saved = bufs[0].clone()
    td = 0.0
    for _ in range(reps):
        bufs[0].zero_()  # the erasure, outside the timed call
        t0 = time.perf_counter()
        E.jerasure.jerasure_matrix_decode(k, m, 8, M, 0, [0], bufs[:k], bufs[k:], S)
        td += time.perf_counter() - t0
    td /= reps
    return {"workload": f"jerasure_matrix_encode/decode{{0}} on pinned host buffers, RS({k},{m}) {S >> 20} MiB, "
                        f"synchronous", "encode_ms": round(te * 1e3, 3), "encode_data_GiBps": round(k * S / te / GiB, 2),
            "decode_ms": round(td * 1e3, 3), "decode_ok": bool(torch.equal(bufs[0], saved))}


def dropin_split(reps=5, rounds=3):
    """Synchronous jerasure_matrix_encode on host buffers with the call split
    into byte ranges run concurrently (ECGPU_SPLIT = 0 / 2 / 4 / 8; on one GPU
    every range shares its link), pageable and pinned, C3 RS(10,4) 4 MiB and
    C5 RS(12,4) 16 MiB; interleaved rounds, medians."""
    from erasure_coding_test_amd import _native as N
    out = {}
    for k, m, S in ((10, 4, 4 << 20), (12, 4, 16 << 20)):
        M = E.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
        for pinned in (False, True):
            if pinned:
                data = [torch.randint(0, 256, (S,), dtype=torch.uint8).pin_memory() for _ in range(k)]
                coding = [torch.zeros(S, dtype=torch.uint8).pin_memory() for _ in range(m)]
            else:
                rng = np.random.default_rng(k)
                data = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
                coding = [np.zeros(S, np.uint8) for _ in range(m)]
            times = {w: [] for w in (0, 2, 4, 8)}
            ref = None
            for _ in range(rounds):
                for ways in times:
                    N.set_knob("split", ways)
                    N.set_knob("split_min_kib", 256)
                    E.jerasure.jerasure_matrix_encode(k, m, 8, M, data, coding, S)
                    t0 = time.perf_counter()
                    for _ in range(reps):
                        E.jerasure.jerasure_matrix_encode(k, m, 8, M, data, coding, S)
                    times[ways].append((time.perf_counter() - t0) / reps)
                    got = [bytes(np.asarray(c)[:4096]) + bytes(np.asarray(c)[-4096:]) for c in coding]
                    ref = ref or got
                    assert got == ref, ("split result differs", ways)
            N.reset_knob("split")
            N.reset_knob("split_min_kib")
            key = f"RS({k},{m}) {S >> 20} MiB {'pinned' if pinned else 'pageable'}"
            out[key] = {f"split{w}_ms": round(sorted(t)[len(t) // 2] * 1e3, 3) for w, t in times.items()}
            out[key].update({f"split{w}_data_GiBps": round(k * S / sorted(t)[len(t) // 2] / GiB, 2)
                             for w, t in times.items()})
    return out


def ecx_accum(k=10, m=4, S=4 << 20, stripes=12):
    """ECX incremental accumulation (ecx_datanode_main.cpp:680-735) through
    ParityAccumulator: per stripe, k synchronous adds (one arriving source
    block each, coefficient column j of the coding matrix) into m HBM-resident
    accumulators, then m reads of the finished parity.  Blocks device-resident,
    in pinned host memory, or in pageable host memory; the parity read goes to
    the same kind of memory.  HBM bytes per stripe: k blocks read, m
    accumulators written once and read+written k-1 times.  *_async: the adds
    are queued (ecgpu_accum_add_async: block j+1's H2D overlaps block j's
    update) and sync() waits for them.  per_add_us = (k adds + sync) / k;
    per_read_us = one parity read-out; stripe_ms = both."""
    M = E.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    cols = [[M[i * k + j] for i in range(m)] for j in range(k)]
    out = {}
    for where in ("device", "pinned", "pageable", "device_async", "pinned_async", "pageable_async"):
        wait = not where.endswith("_async")
        if where.startswith("device"):
            blocks = torch.randint(0, 256, (k, S), dtype=torch.uint8, device="cuda")
            parity = torch.empty((m, S), dtype=torch.uint8, device="cuda")
        else:
            blocks = torch.randint(0, 256, (k, S), dtype=torch.uint8)
            parity = torch.empty((m, S), dtype=torch.uint8)
            if where.startswith("pinned"):
                blocks, parity = blocks.pin_memory(), parity.pin_memory()
        acc = E.ParityAccumulator(m, S)

        def adds():
            acc.reset()
            for j in range(k):
                acc.add(blocks[j], cols[j], wait=wait)
            acc.sync()

        def reads():
            for i in range(m):
                acc.read(i, parity[i])

        adds()
        reads()
        torch.cuda.synchronize()
        ta = tr = 0.0
        for _ in range(stripes):
            t0 = time.perf_counter()
            adds()
            t1 = time.perf_counter()
            reads()
            ta += t1 - t0
            tr += time.perf_counter() - t1
        torch.cuda.synchronize()
        t = (ta + tr) / stripes
        hbm = (k + m + 2 * m * (k - 1)) * S
        out[where] = {"stripe_ms": round(t * 1e3, 3), "per_add_us": round(ta / stripes / k * 1e6, 1),
                      "per_read_us": round(tr / stripes / m * 1e6, 1),
                      "add_GiBps": round(k * S * stripes / ta / GiB, 2),
                      "data_GiBps": round(k * S / t / GiB, 2), "hbm_GBps_if_device": round(hbm / t / 1e9, 1)}
        acc.close()
    return {"workload": f"ParityAccumulator RS({k},{m}), {S >> 20} MiB blocks, {k} adds + {m} reads per stripe, "
                        f"{stripes} stripes, synchronous or queued adds", "results": out}


def call_latency(reps=200):
    """Fixed cost of one synchronous drop-in call (host planning, pointer
    classification, pointer-table upload, launch, stream sync): RS(10,4)
    jerasure_matrix_encode / decode{0} on 4 KiB device-resident shards, and
    a ParityAccumulator add, median over `reps` calls."""
    k, m, S = 10, 4, 4096
    M = E.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    data = [torch.randint(0, 256, (S,), dtype=torch.uint8, device="cuda") for _ in range(k)]
    coding = [torch.empty(S, dtype=torch.uint8, device="cuda") for _ in range(m)]
    acc = E.ParityAccumulator(m, S)
    col = [M[i * k] for i in range(m)]
    cases = {"jerasure_matrix_encode": lambda: E.jerasure.jerasure_matrix_encode(k, m, 8, M, data, coding, S),
             "jerasure_matrix_decode{0}": lambda: E.jerasure.jerasure_matrix_decode(k, m, 8, M, 0, [0], data, coding,
                                                                                    S),
             "ParityAccumulator.add": lambda: acc.add(data[0], col)}
    out = {}
    for name, fn in cases.items():
        for _ in range(10):
            fn()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        out[name] = {"median_us": round(statistics.median(ts) * 1e6, 1), "p10_us": round(sorted(ts)[reps // 10] * 1e6, 1)}
    acc.close()
    return {"workload": "RS(10,4), 4 KiB device-resident shards, synchronous calls", "results": out}


def device_configs():
    out = []
    cases = [("C2 RS(6,3) 1 MiB encode", 6, 3, 1 << 20, 96, None),
             ("C3 RS(10,4) 4 MiB decode{0}", 10, 4, 4 << 20, 24, [0]),
             ("C4 RS(10,4) 4 MiB decode{0,1,2,3}", 10, 4, 4 << 20, 24, [0, 1, 2, 3]),
             ("C5 RS(12,4) 16 MiB encode", 12, 4, 16 << 20, 8, None)]
    for name, k, m, S, B, er in cases:
        M = E.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
        slab, shards = E.alloc_stripes(B, k, m, S)
        slab.random_(0, 256)
        E.encode_plan(k, m, M).bind([st[:k] for st in shards], [st[k:] for st in shards], S).launch()
        if er is None:
            p = E.encode_plan(k, m, M).bind([st[:k] for st in shards], [st[k:] for st in shards], S)
            nbytes, data = (k + m) * S * B, k * S * B
        else:
            t0 = time.perf_counter()
            p = E.DecodePlan(k, m, M, er)
            plan_us = (time.perf_counter() - t0) * 1e6
            p.bind_stripes(shards, S)
            nbytes, data = (len(p.src_ids) + len(p.out_ids)) * S * B, k * S * B
        t = timed_events(p.launch)
        rec = {"config": name, "stripes": B, "launch_ms": round(t * 1e3, 4), "hbm_GBps": round(nbytes / t / 1e9, 1),
               "frac_of_8TBps": round(nbytes / t / 8e12, 4), "data_GiBps": round(data / t / GiB, 1)}
        if er is not None:
            rec["host_plan_us"] = round(plan_us, 1)
        out.append(rec)
        del slab, shards, p
        torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stripes", type=int, default=48)
    ap.add_argument("--parts", default="", help="comma list of result keys to run (default: all)")
    a = ap.parse_args()
    parts = {"pcie": pcie_rates, "pcie_duplex": lambda: pcie_duplex(stripes=a.stripes),
             "e2e_pinned": lambda: e2e_pinned(a.stripes),
             "e2e_pipeline_pinned": lambda: e2e_pipeline(a.stripes),
             "e2e_pipeline_pageable": lambda: e2e_pipeline(a.stripes, pinned=False),
             "e2e_group_all_devices": lambda: e2e_pipeline(
                 a.stripes, devices=list(range(torch.cuda.device_count()))),
             "e2e_group_dev0_twice": lambda: e2e_pipeline(a.stripes, devices=[0, 0]),
             "e2e_read_pipeline_1": lambda: e2e_read_pipeline([0], a.stripes),
             "e2e_read_pipeline_4": lambda: e2e_read_pipeline([0, 1, 2, 3], a.stripes),
             "dropin_pageable": dropin_pageable,
             "dropin_pinned": dropin_pinned,
             "dropin_pinned_c2": lambda: dropin_pinned(6, 3, 1 << 20, 50),
             "dropin_split": dropin_split,
             "pipeline_depth": lambda: {f"depth{d}_round{r}": e2e_pipeline(a.stripes, depth=d)["data_GiBps"]
                                        for r in range(2) for d in (2, 3, 4, 6)},
             "ecx_accum": ecx_accum,
             "call_latency": call_latency,
             "device_configs": device_configs}
    want = a.parts.split(",") if a.parts else list(parts)
    res = {name: parts[name]() for name in want}
    from erasure_coding_test_amd import _native as N
    res["cpu_fallbacks"] = N.fallback_count()  # the package keeps the fallback off: must be 0
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
