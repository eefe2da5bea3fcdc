"""Two processes on one GPU and one PCIe link: where the e2e write path's
aggregate goes.

The N = 2 rehearsal of bench.py (both ranks on cuda:0) measured the
pipelined RS(10,4) 4 MiB encode at 27.21 GiB/s of data for the pair against
50.49 for one process, while the 10:1 decode held 44.76.  This script runs
the same passes -- and the raw copies under them -- once per process with a
gloo barrier starting every timed pass together, so the same legs can be
read with 1 and 2 processes and, under `rocprofv3 --kernel-trace
--memory-copy-trace`, per copy.

Legs (per rank, `stripes` stripes of pinned host memory [stripes][k+m][S]):
  h2d          the k data shards of every stripe to HBM (one copy per stripe)
  d2h          the m parity shards of every stripe back (one copy per stripe)
  duplex       both at once on two streams (the write path's PCIe traffic,
               no compute)
  pipe_encode  ecgpu_pipeline (H2D, encode, D2H overlapped, depth 3)
  pipe_decode  ecgpu_pipeline_create_decode, erasure {0} (10 in, 1 out)
  pipe_*_zc1   the same with ECGPU_PIPE_ZC=1: the kernel writes the outputs
               into the pinned host stripes in place (no D2H DMA)
  pipe_*_zc2   ECGPU_PIPE_ZC=2: the kernel also reads the sources in place
               (no DMA at all)
  pipe_*_skew  ECGPU_PIPE_CONTIG=0: ring slots at the skewed shard stride, so
               each stripe moves as 2-D copies (the round-5 layout)
Pipeline legs check the last stripe after the last pass (its outputs zeroed
before it): encode parity against a device-resident encode, decode against
the original shard.

    python3 tools/e2e_pair.py --rank R --world W --port P [--legs a,b] [--depth 3]

Rank 0 prints one JSON line per leg: the aggregate data rate (every rank's
k*S*stripes over the slowest rank's pass) and each rank's own pass.
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

GiB = 2**30


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--world", type=int, default=1)
    ap.add_argument("--port", type=int, default=29611)
    ap.add_argument("--stripes", type=int, default=24)
    ap.add_argument("--depth", type=int, default=3)
    ap.add_argument("--passes", type=int, default=3)
    ap.add_argument("--legs", default="h2d,d2h,duplex,pipe_encode,pipe_decode")
    ap.add_argument("--tag", default="")
    ap.add_argument("--pre", type=int, default=0,
                    help="before the legs: this many bench-step encode launches over a 96-stripe 4 MiB slab "
                         "(5.3 GiB resident, as bench.py's ranks hold when their e2e leg starts)")
    ap.add_argument("--c5", action="store_true",
                    help="before the legs: bench.py's sharded_c5 on this rank (24 RS(12,4) 16 MiB stripes = 6 GiB, "
                         "13 encode launches, the slab freed and torch.cuda.empty_cache())")
    ap.add_argument("--churn-gib", type=int, default=0,
                    help="before the legs: allocate this many GiB of HBM, fill it, free it and empty torch's cache")
    ap.add_argument("--knob", action="append", default=[],
                    help="name=value: a library knob for the whole run (ecgpu_set_knob), e.g. ECGPU_ZC_GRID=256")
    ap.add_argument("--bench-data", action="store_true",
                    help="fill the host stripes like bench.py's e2e leg (one random stripe, copied from HBM)")
    a = ap.parse_args()

    import torch
    import torch.distributed as dist
    import erasure_coding_test_amd as E

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{a.port}", rank=a.rank, world_size=a.world,
                            timeout=datetime.timedelta(seconds=120))
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    k, m, S, n = 10, 4, 4 << 20, a.stripes
    M = E.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    keep = None
    if a.pre:
        slab, shards = E.alloc_stripes(96, k, m, S)
        slab.random_(0, 256)
        plan = E.encode_plan(k, m, M).bind([st[:k] for st in shards], [st[k:] for st in shards], S)
        for _ in range(a.pre):
            plan.launch()
        torch.cuda.synchronize(dev)
        keep = (slab, shards, plan)  # held, like the bench's slab
    if a.c5:
        M5 = E.reed_sol.reed_sol_vandermonde_coding_matrix(12, 4, 8)
        slab5, sh5 = E.alloc_stripes(24, 12, 4, 16 << 20)
        slab5.random_(0, 256)
        p5 = E.encode_plan(12, 4, M5).bind([st[:12] for st in sh5], [st[12:] for st in sh5], 16 << 20)
        for _ in range(13):
            p5.launch()
        torch.cuda.synchronize(dev)
        p5.close()
        del slab5, sh5
        torch.cuda.empty_cache()
    if a.churn_gib:
        junk = torch.empty(a.churn_gib << 30, dtype=torch.uint8, device=dev)
        junk.fill_(1)
        torch.cuda.synchronize(dev)
        del junk
        torch.cuda.empty_cache()
    host = torch.empty((n, k + m, S), dtype=torch.uint8).pin_memory()
    if a.bench_data:
        src = torch.randint(0, 256, (k, S), dtype=torch.uint8, device=dev)
        for s in range(n):
            host[s, :k].copy_(src)
            host[s, 0, :8].fill_(s)
        torch.cuda.synchronize(dev)
    else:
        host[:, :k].random_(0, 256)
    for s in range(n):  # valid codewords, so the decode legs have consistent survivors
        d = host[s, :k].to(dev)
        par = torch.empty((m, S), dtype=torch.uint8, device=dev)
        E.encode_plan(k, m, M, 0).bind([[d[j] for j in range(k)]], [[par[i] for i in range(m)]], S).launch()
        torch.cuda.synchronize(dev)
        host[s, k:].copy_(par.cpu())
    dk = torch.empty((3, k, S), dtype=torch.uint8, device=dev)
    dm = torch.empty((3, m, S), dtype=torch.uint8, device=dev)
    dm.random_(0, 256)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def h2d():
        with torch.cuda.stream(s1):
            for s in range(n):
                dk[s % 3].copy_(host[s, :k], non_blocking=True)
        s1.synchronize()

    def d2h():
        with torch.cuda.stream(s2):
            for s in range(n):
                host[s, k:].copy_(dm[s % 3], non_blocking=True)
        s2.synchronize()

    def duplex():
        for s in range(n):
            with torch.cuda.stream(s1):
                dk[s % 3].copy_(host[s, :k], non_blocking=True)
            with torch.cuda.stream(s2):
                host[s, k:].copy_(dm[s % 3], non_blocking=True)
        s1.synchronize()
        s2.synchronize()

    def pipe(p):
        def run():
            for s in range(n):
                p.submit([host[s, j] for j in range(k)], [host[s, k + i] for i in range(m)])
            p.drain()
        return run

    from erasure_coding_test_amd import _native as N
    for kv in a.knob:
        name, value = kv.split("=")
        N.set_knob(name, int(value))

    def pipeline(decode, zc, contig=1):
        def make():
            N.set_knob("pipe_zc", zc)  # read at creation
            N.set_knob("pipe_contig", contig)
            p = (E.HostPipeline.decoder(k, m, M, [0], S, depth=a.depth, device=0) if decode
                 else E.HostPipeline(k, m, M, S, depth=a.depth, device=0))
            N.reset_knob("pipe_zc")
            N.reset_knob("pipe_contig")
            return p
        return None, make

    legs = {"h2d": (h2d, None), "d2h": (d2h, None), "duplex": (duplex, None),
            "pipe_encode": pipeline(False, 0), "pipe_decode": pipeline(True, 0),
            "pipe_encode_zc1": pipeline(False, 1), "pipe_encode_zc2": pipeline(False, 2),
            "pipe_decode_zc1": pipeline(True, 1), "pipe_decode_zc2": pipeline(True, 2),
            "pipe_encode_skew": pipeline(False, 0, 0), "pipe_decode_skew": pipeline(True, 0, 0)}
    for name in a.legs.split(","):
        fn, make = legs[name]
        p = make() if make else None
        run = fn or pipe(p)
        run()  # warm
        torch.cuda.synchronize(dev)
        ts = []
        ok = None
        for it in range(a.passes):
            if p is not None and it == a.passes - 1:
                # the last pass must rewrite what it outputs: scribble over it first
                want = host[n - 1].clone()
                host[:, [0] if name.startswith("pipe_decode") else slice(k, k + m)] = 0
            dist.barrier()
            t0 = time.perf_counter()
            run()
            ts.append(time.perf_counter() - t0)
        if p is not None:
            p.close()
            if name.startswith("pipe_encode"):
                d = host[n - 1, :k].to(dev)
                ref = torch.empty((m, S), dtype=torch.uint8, device=dev)
                E.encode_plan(k, m, M, 0).bind([[d[j] for j in range(k)]], [[ref[i] for i in range(m)]], S).launch()
                torch.cuda.synchronize(dev)
                ok = bool(torch.equal(ref.cpu(), host[n - 1, k:])) and bool(torch.equal(want, host[n - 1]))
            else:
                ok = bool(torch.equal(want, host[n - 1]))
        mine = {"rank": a.rank, "pass_ms": [round(t * 1e3, 2) for t in ts], "ok": ok}
        allr = [None] * a.world
        dist.all_gather_object(allr, mine)
        if a.rank == 0:
            moved = {"h2d": k, "d2h": m}.get(name, k) * S * n  # data bytes: k per stripe (d2h: the m parity)
            agg = [a.world * moved / max(r["pass_ms"][i] for r in allr) * 1e3 / GiB for i in range(a.passes)]
            print(json.dumps({"tag": a.tag, "leg": name, "world": a.world, "stripes": n, "depth": a.depth,
                              "unit": "GiB/s (h2d/duplex/pipe: data shards; d2h: parity shards), all ranks",
                              "aggregate_GiBps": [round(x, 2) for x in agg],
                              "aggregate_median_GiBps": round(sorted(agg)[len(agg) // 2], 2),
                              "per_rank_pass_ms": [r["pass_ms"] for r in allr],
                              "ok": [r["ok"] for r in allr]}), flush=True)
    assert N.fallback_count() == 0 and N.cpu_call_count() == 0
    del keep
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
