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
    host = torch.empty((n, k + m, S), dtype=torch.uint8).pin_memory()
    host[:, :k].random_(0, 256)
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

    legs = {"h2d": (h2d, None), "d2h": (d2h, None), "duplex": (duplex, None),
            "pipe_encode": (None, lambda: E.HostPipeline(k, m, M, S, depth=a.depth, device=0)),
            "pipe_decode": (None, lambda: E.HostPipeline.decoder(k, m, M, [0], S, depth=a.depth, device=0))}
    for name in a.legs.split(","):
        fn, make = legs[name]
        p = make() if make else None
        run = fn or pipe(p)
        run()  # warm
        torch.cuda.synchronize(dev)
        ts = []
        for _ in range(a.passes):
            dist.barrier()
            t0 = time.perf_counter()
            run()
            ts.append(time.perf_counter() - t0)
        if p is not None:
            p.close()
        mine = {"rank": a.rank, "pass_ms": [round(t * 1e3, 2) for t in ts]}
        allr = [None] * a.world
        dist.all_gather_object(allr, mine)
        if a.rank == 0:
            moved = {"h2d": k, "d2h": m}.get(name, k) * S * n  # data bytes: k per stripe (d2h: the m parity)
            agg = [a.world * moved / max(r["pass_ms"][i] for r in allr) * 1e3 / GiB for i in range(a.passes)]
            print(json.dumps({"tag": a.tag, "leg": name, "world": a.world, "stripes": n, "depth": a.depth,
                              "unit": "GiB/s (h2d/duplex/pipe: data shards; d2h: parity shards), all ranks",
                              "aggregate_GiBps": [round(x, 2) for x in agg],
                              "aggregate_median_GiBps": round(sorted(agg)[len(agg) // 2], 2),
                              "per_rank_pass_ms": [r["pass_ms"] for r in allr]}), flush=True)
    from erasure_coding_test_amd import _native as N
    assert N.fallback_count() == 0
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
