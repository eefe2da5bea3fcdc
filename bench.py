"""Headline benchmark: device-resident RS(10,4) encode + decode, 4 MiB shards.

BASELINE.json metric: "GiB/s device-resident RS encode+decode, RS(10,4) 4 MiB
shards, 1/2/4/8 GPU".  One step = one pass of the hot path over one batch of
synthetic stripes resident in HBM:

  encode  : B stripes x (10 data -> 4 parity)          (jerasure_matrix_encode)
  decode  : B stripes, data shard 0 erased, rebuilt from the first 10
            survivors (jerasure_matrix_decode, row_k_ones=0 -- the client's
            call, client_main.cpp:2118)

value = user-data bytes processed by all ranks / wall time of the K timed
steps (max over ranks) = N * K * B * 2 * k * S / t, in GiB/s.  Stripes are
independent, so each rank codes its own B stripes (weak scaling, no data-path
collective); the only cross-rank traffic is the timing barrier and one
max-reduce on the host (gloo).

    python bench.py [--gpus N --steps K --warmup W --stripes B]
    torchrun --nproc-per-node N bench.py --gpus N ...        (N > 1)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

K_DATA, M_PARITY, SHARD = 10, 4, 4 << 20
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--stripes", type=int, default=96,
                    help="stripes per GPU per step (96 x 56 MiB = 5.3 GiB resident; throughput plateaus from 96, "
                         "DESIGN.md §6)")
    ap.add_argument("--kernel", choices=["perm", "lds"], default="perm")
    ap.add_argument("--nt", type=int, default=1, help="non-temporal loads/stores")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget (0 = skip)")
    return ap.parse_args()


def dist_setup(n_gpus):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    return rank, local, world


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(x: float, world: int) -> float:
    if world == 1:
        return x
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def stripes_for_rank(total: int, rank: int, world: int) -> list:
    """Round-robin stripe ids over ranks; used by the
    multi-rank tests to check every stripe is coded exactly once."""
    return list(range(rank, total, world))


def load_traffic(workload: str):
    """HBM bytes per encode launch from the committed rocprofv3 PMC summary
    (profiles/pmc_encode.json, written by profiles/summarize.py), or None."""
    p = os.path.join(ROOT, "profiles", "pmc_encode.json")
    try:
        with open(p) as f:
            d = json.load(f)
        if d.get("workload") == workload:
            return d.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    return None


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_has_avx2() -> bool:
    try:
        with open("/proc/cpuinfo") as f:
            return any(line.startswith("flags") and " avx2" in line for line in f)
    except OSError:
        return False


def cpu_baseline(seconds: float, threads: int = 1, o3: bool = False):
    """Reference CPU path on the host: oracle/_ref (the reference's own
    src/erasure_coding compiled -O2) if shipped, else our C restatement.
    Bounded sample of the same workload: one RS(10,4) 4 MiB stripe, encode +
    decode{0}, repeated until `seconds` of wall time.  With threads > 1 each
    call is split by byte range over threads exactly like the reference
    client's encode_mul_thread (client_main.cpp:1074-1164; thread 0 takes the
    remainder) -- ctypes releases the GIL, so the threads run in parallel."""
    import ctypes
    import threading

    import numpy as np

    from oracle.oracle import REFERENCE_O3_SO, Reference, Restatement, alloc_shards
    if o3:
        o = Reference(REFERENCE_O3_SO)  # caller checked avx2 and the file
    else:
        try:
            o = Reference()
        except (FileNotFoundError, OSError):
            o = Restatement()
    k, m, S = K_DATA, M_PARITY, SHARD
    M = o.vandermonde_coding_matrix(k, m)
    rng = np.random.default_rng(0)
    data = alloc_shards(k, S)
    for d in data:
        d[:S] = rng.integers(0, 256, S, dtype=np.uint8)
    coding = alloc_shards(m, S)
    ranges, off = [], 0
    for t in range(threads):
        n = S // threads + (S % threads if t == 0 else 0)
        ranges.append((off, n))
        off += n

    def views(bufs, off, n):
        return [np.frombuffer((ctypes.c_uint8 * (n + 16)).from_address(b.ctypes.data + off), dtype=np.uint8)
                for b in bufs]

    parts = [(views(data, a, n), views(coding, a, n), n) for a, n in ranges]

    def one(p):
        d, c, n = p
        o.matrix_encode(k, m, M, d, c, n)
        o.matrix_decode(k, m, M, 0, [0], d, c, n)

    iters, t0 = 0, time.perf_counter()
    while True:
        if threads == 1:
            one(parts[0])
        else:
            ts = [threading.Thread(target=one, args=(p,)) for p in parts]
            for t in ts:
                t.start()
            for t in ts:
                t.join()
        iters += 1
        el = time.perf_counter() - t0
        if el >= seconds or iters >= 2000:
            break
    gib = iters * 2 * k * S / 2**30
    flags = "-O3 -march=x86-64-v3" if o3 else "-O2"
    src = f"reference src/erasure_coding compiled g++ {flags}" if o.kind == "reference" else "oracle/ec_oracle.c -O2"
    return {"value": round(gib / el, 4), "unit": "GiB/s", "cores": threads, "kind": o.kind,
            "sample": f"{iters} x (RS(10,4) 4 MiB stripe encode + decode of erasure {{0}}), {threads} thread(s) "
                      f"splitting byte ranges like client_main.cpp:1074-1164, {el:.1f} s, {src}, "
                      f"host CPU {cpu_model()}"}


def copy_ceiling(slab, reps: int = 10):
    """Measured stream-copy ceiling on this GPU: the
    diagnostic 16-B non-temporal copy kernel (libecgpu_diag.so, diag_copy)
    moving shards 0..6 -> 7..13 of every stripe of the bench slab, i.e. the
    same bytes, shard stride and skew as the coding launches.  Returns GB/s of
    (read + written) bytes, or None when the diagnostic library is absent."""
    import ctypes

    from erasure_coding_test_amd import _native as N
    path = os.path.join(N.LIB_DIR, "libecgpu_diag.so")
    if not os.path.exists(path):
        return None
    L = ctypes.CDLL(path)
    L.ecgpu_diag_launch.restype = ctypes.c_int
    L.ecgpu_diag_launch.argtypes = [ctypes.c_int] * 5 + [ctypes.c_void_p] * 4 + [
        ctypes.c_int, ctypes.c_longlong, ctypes.c_ulonglong, ctypes.c_ulonglong, ctypes.c_int, ctypes.c_void_p,
        ctypes.c_void_p]
    B, n_sh, S = slab.shape[0], slab.shape[1], SHARD
    half = n_sh // 2
    dev = slab.device
    src = torch.tensor([slab[b, i].data_ptr() for b in range(B) for i in range(half)], dtype=torch.int64, device=dev)
    dst = torch.tensor([slab[b, half + i].data_ptr() for b in range(B) for i in range(half)], dtype=torch.int64,
                       device=dev)
    stream = torch.cuda.current_stream(dev)
    best = None
    for policy in range(4):  # bit 0: non-temporal loads, bit 1: non-temporal stores
        ts = []
        for i in range(reps + 2):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            rc = L.ecgpu_diag_launch(1, 1, 1, 1, policy, None, None, src.data_ptr(), dst.data_ptr(), B * half, S, 0,
                                     0, 1, stream.cuda_stream, None)
            e1.record(stream)
            torch.cuda.synchronize(dev)
            if rc != 0:
                return None
            if i >= 2:
                ts.append(e0.elapsed_time(e1))
        ts.sort()
        ms = ts[len(ts) // 2]
        if best is None or ms < best[0]:
            best = (ms, policy)
    ms, policy = best
    return {"GBps": round(2 * S * B * half / (ms / 1e3) / 1e9, 1), "avg_launch_ms": round(ms, 4),
            "kernel": f"diag_copy 16 B/lane, shards 0..{half - 1} -> {half}..{n_sh - 1} of every stripe; best of the "
                      f"4 cache policies (here loads {'nt' if policy & 1 else 'plain'}, stores "
                      f"{'nt' if policy & 2 else 'plain'}), median of {reps}"}


def host_threads() -> int:
    """The CPU share this process may use (affinity), capped at 16 (the GPU box's per-GPU share)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def main():
    args = parse()
    rank, local, world = dist_setup(args.gpus)
    import erasure_coding_test_amd as E
    from erasure_coding_test_amd import _native as N

    # ECGPU_BENCH_ONE_DEVICE=1: every rank on cuda:0 -- a multi-rank rehearsal
    # on a one-GPU box (the numbers are then not a scaling measurement).
    if os.environ.get("ECGPU_BENCH_ONE_DEVICE") == "1":
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    k, m, S, B = K_DATA, M_PARITY, SHARD, args.stripes
    M = E.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)

    # B stripes x (k+m) shards in one HBM slab at the library's recommended
    # shard stride (S + 4 KiB skew); random data (zeros would flatter DVFS).
    slab, shards = E.alloc_stripes(B, k, m, S, dev)
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    slab.random_(0, 256, generator=g)

    kind = N.KERNEL_LDS if args.kernel == "lds" else N.KERNEL_PERM
    enc = E.encode_plan(k, m, M, local).bind([st[:k] for st in shards], [st[k:] for st in shards], S)
    enc.set_kernel(kind, bool(args.nt))
    dec = E.DecodePlan(k, m, M, [0], 0, local).bind_stripes(shards, S)
    dec.set_kernel(kind, bool(args.nt))
    stream = torch.cuda.current_stream(dev)

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        enc.launch(stream.cuda_stream)
        if ev is not None:
            ev[1].record(stream)
        dec.launch(stream.cuda_stream)
        if ev is not None:
            ev[2].record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]

    barrier(world)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(evs[i])
    torch.cuda.synchronize(dev)
    # each rank's clock stops when its own GPU work has drained; the closing
    # barrier still brackets the region and the max over ranks below makes
    # the slowest rank the job's time (the barrier's own latency is not work)
    elapsed = time.perf_counter() - t0
    barrier(world)
    t = max_over_ranks(elapsed, world)

    enc_ms = sum(e[0].elapsed_time(e[1]) for e in evs) / args.steps
    dec_ms = sum(e[1].elapsed_time(e[2]) for e in evs) / args.steps
    enc_bytes = (k + m) * S * B           # algorithmic HBM bytes per encode launch
    dec_bytes = (k + 1) * S * B           # 10 survivors read + 1 shard written
    user_bytes = world * args.steps * B * 2 * k * S
    value = user_bytes / t / 2**30

    # sanity: the decode must have rebuilt shard 0 bit-exactly (it is rewritten
    # every step from the survivors; compare with an independent encode check)
    ok = True
    if rank == 0:
        # re-encode stripe 0 with the OTHER multiply engine (LDS nibble tables,
        # gf_apply_lds) so the check is independent of the timed kernel and its
        # launch does not mix into the timed kernel's rocprof statistics
        chk = torch.empty((m, S), dtype=torch.uint8, device=dev)
        ref = E.encode_plan(k, m, M, local).bind([shards[0][:k]], [[chk[i] for i in range(m)]], S)
        ref.set_kernel(N.KERNEL_LDS, True)
        ref.launch(stream.cuda_stream)
        torch.cuda.synchronize(dev)
        ok = all(bool(torch.equal(chk[i], shards[0][k + i])) for i in range(m))
        # after the parity check: the copy overwrites the slab
        copy = copy_ceiling(slab)

    workload = f"RS(10,4) encode + decode{{0}}, 4 MiB shards, {B} stripes/GPU"
    if rank == 0:
        cpu = cpu_all = cpu_o3 = None
        if world == 1 and args.cpu_seconds > 0:
            cpu = cpu_baseline(args.cpu_seconds)
            cpu_all = cpu_baseline(max(2.0, args.cpu_seconds / 2), host_threads())
            from oracle.oracle import REFERENCE_O3_SO
            if host_has_avx2() and os.path.exists(REFERENCE_O3_SO):
                cpu_o3 = cpu_baseline(max(2.0, args.cpu_seconds / 2), 1, o3=True)
        achieved = enc_bytes / (enc_ms / 1e3) / 1e9
        traffic = load_traffic(workload)
        out = {
            "metric": "GiB/s device-resident RS encode+decode, RS(10,4) 4 MiB shards, 1/2/4/8 GPU",
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (uniform random bytes, device-generated)",
            "config": {"workload": workload, "k": k, "m": m, "shard_bytes": S, "stripes_per_gpu": B,
                       "shard_stride_bytes": int(slab.stride(1)),
                       "erasures": [0], "kernel": args.kernel, "nontemporal": bool(args.nt),
                       "parallelism": f"stripes sharded over {world} GPU(s), no collective"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "kernel": "gf_apply (encode launch)", "algorithmic_bytes_per_launch": enc_bytes,
                         "avg_launch_ms": round(enc_ms, 4),
                         # the north star's read-only accounting: data-shard bytes only, which
                         # caps at k/(k+m) = 0.714 of peak for any encode
                         "read_only_frac": round(k * S * B / (enc_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4)},
            "copy_ceiling": copy,
            "encode_frac_of_copy": round(achieved / copy["GBps"], 4) if copy else None,
            "decode_kernel": {"avg_launch_ms": round(dec_ms, 4), "algorithmic_bytes_per_launch": dec_bytes,
                              "achieved_GBps": round(dec_bytes / (dec_ms / 1e3) / 1e9, 1)},
            "cpu_baseline": cpu,
            "cpu_baseline_all_cores": cpu_all,
            "cpu_baseline_o3": cpu_o3,
            "selfcheck_parity_ok": ok,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
