"""Headline benchmark: device-resident RS encode (+ decode), one rank per GPU.

BASELINE.json metric: "GiB/s device-resident RS encode+decode, RS(10,4) 4 MiB
shards, 1/2/4/8 GPU".  One step = one pass of the hot path over one batch of
synthetic stripes resident in HBM:

  --config C3 (default; the metric's workload)
     encode  : B stripes x (10 data -> 4 parity)          (jerasure_matrix_encode)
     decode  : B stripes, data shard 0 erased, rebuilt from the first 10
               survivors (jerasure_matrix_decode, row_k_ones=0 -- the client's
               call, client_main.cpp:2118)
  --config C5 (BASELINE.json configs[4])
     encode  : 8 stripes/GPU x RS(12,4), 16 MiB shards

value = user-data bytes processed by all ranks / wall time of the K timed
steps (max over ranks), in GiB/s.  Stripes are independent, so each rank codes
its own stripes -- global stripe ids round-robin over ranks (rank r owns ids
r, r+N, ...), the reference's byte-range / stripe splitting
(client_main.cpp:1074-1164, ecx_datanode_main.cpp:1113-1117) mapped onto GPUs
-- with no data-path collective (weak scaling); the only cross-rank traffic is
the timing barrier, one max-reduce and the per-rank report, on gloo (host).

Launch:
    python bench.py                                  N = 1, in process
    python bench.py --gpus N                         spawns N rank processes
                                                     (one per visible GPU) itself
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N
                                                     the driver's form; ranks
                                                     come from the environment
--gpus N with fewer than N visible GPUs exits non-zero, as does a WORLD_SIZE
that disagrees with --gpus.  ECGPU_BENCH_ONE_DEVICE=1 puts every rank on
cuda:0 -- a multi-process rehearsal on a one-GPU box, labelled
"rehearsal": true (not a scaling measurement).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
HEADLINE_METRIC = "GiB/s device-resident RS encode+decode, RS(10,4) 4 MiB shards, 1/2/4/8 GPU"

# BASELINE.json configs: (k, m, shard bytes, default stripes per GPU, erasures decoded per step)
CONFIGS = {
    "C3": dict(k=10, m=4, shard=4 << 20, stripes=96, erasures=[0], cfg_id=3,
               metric=HEADLINE_METRIC,
               workload="RS(10,4) encode + decode{{0}}, 4 MiB shards, {B} stripes/GPU"),
    "C5": dict(k=12, m=4, shard=16 << 20, stripes=8, erasures=None, cfg_id=5,
               metric="GiB/s device-resident RS(12,4) encode, 16 MiB shards, stripes sharded across GPUs",
               workload="C5: RS(12,4) encode, 16 MiB shards, {B} stripes/GPU, global stripe ids round-robin "
                        "over ranks"),
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="C3")
    ap.add_argument("--stripes", type=int, default=0,
                    help="stripes per GPU per step (default: C3 96 x 56 MiB = 5.3 GiB resident -- throughput "
                         "plateaus from 96, DESIGN.md §6; C5 8 x 256 MiB)")
    ap.add_argument("--kernel", choices=["perm", "lds"], default="perm")
    ap.add_argument("--nt", type=int, default=1, help="non-temporal loads/stores")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget (0 = skip)")
    ap.add_argument("--no-configs", action="store_true",
                    help="skip the per-config block (C2 / C3 / C4 / C5 launches; run by every rank on its own GPU "
                         "at any N)")
    ap.add_argument("--e2e-stripes", type=int, default=24,
                    help="pinned host stripes for the PCIe-inclusive e2e rate on rank 0 (0 = skip)")
    ap.add_argument("--spawn-selftest", action="store_true",
                    help="launch / rendezvous / report path only, no GPU work (CPU test of --gpus N)")
    return ap.parse_args(argv)


# ------------------------------------------------------------------ launch ----
def launch_mode(gpus: int, env, device_count: int, selftest: bool = False):
    """('run' | 'spawn' | 'error', message).  Pure: tested on CPU."""
    rehearsal = env.get("ECGPU_BENCH_ONE_DEVICE") == "1"
    if gpus < 1:
        return "error", f"--gpus must be >= 1 (got {gpus})"
    world_env = env.get("WORLD_SIZE")
    if world_env is not None and world_env != "":
        if int(world_env) != gpus:
            return "error", f"WORLD_SIZE={world_env} but --gpus {gpus}: launch one rank per GPU"
        mode = "run"
    else:
        mode = "run" if gpus == 1 else "spawn"
    need = 1 if rehearsal else gpus
    if not selftest and gpus > 1 and device_count < need:
        return "error", (f"--gpus {gpus} needs {gpus} visible GPUs, found {device_count} (ECGPU_BENCH_ONE_DEVICE=1 "
                         f"runs every rank on cuda:0 as a labelled rehearsal)")
    return mode, ""


def rank_envs(n: int, port: int, base) -> list:
    """Environment of each spawned rank (torch.distributed.run's variables)."""
    out = []
    for r in range(n):
        e = dict(base)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        out.append(e)
    return out


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, argv) -> int:
    """Start n rank processes of this script (no GPU touched here) and return
    the worst exit code; if one rank fails the others are stopped rather than
    left waiting at a barrier."""
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=e)
             for e in rank_envs(n, free_port(), os.environ)]
    rc = 0
    while procs:
        for p in list(procs):
            r = p.poll()
            if r is None:
                continue
            procs.remove(p)
            if r != 0:
                rc = rc or (r if r > 0 else 1)
                for q in procs:  # the exact PIDs started above
                    q.terminate()
                for q in procs:
                    try:
                        q.wait(timeout=30)
                    except subprocess.TimeoutExpired:
                        q.kill()
                        q.wait()
                procs = []
                break
        time.sleep(0.05)
    return rc


def dist_setup():
    world = int(os.environ.get("WORLD_SIZE", "1") or "1")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # gloo prints its connection report ("[Gloo] Rank r is connected to
        # ...") on stdout, where the launcher reads this bench's one JSON
        # line; the ranks' reports interleave.  Send it to stderr: fd 1 points
        # at fd 2 until every rank has connected (the barrier).
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo", rank=rank, world_size=world)
            dist.barrier()
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
    return rank, local, world


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(x: float, world: int) -> float:
    if world == 1:
        return x
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather(obj, world: int) -> list:
    if world == 1:
        return [obj]
    import torch.distributed as dist
    out = [None] * world
    dist.all_gather_object(out, obj)
    return out


def device_identity(N, local: int) -> dict:
    """The physical GPU a rank runs on: its PCI bus id (hipDeviceGetPCIBusId,
    through the library) and UUID, so an N > 1 line proves its ranks used N
    distinct devices."""
    import ctypes

    import torch
    buf = ctypes.create_string_buffer(64)
    bus = buf.value.decode() if N.lib.ecgpu_device_pci_bus_id(local, buf, len(buf)) == 0 else None
    try:
        uuid = str(torch.cuda.get_device_properties(local).uuid)
    except Exception:  # noqa: BLE001 -- informative only
        uuid = None
    return {"pci_bus_id": bus, "uuid": uuid}


def distinct_devices(per_rank: list, rehearsal: bool):
    """(ok, note): every rank of a real N > 1 run must sit on its own GPU
    (PCI bus id, else UUID).  A rehearsal puts every rank on cuda:0 on
    purpose and is exempt.  Pure: tested on CPU."""
    if len(per_rank) <= 1:
        return True, "one rank"
    if rehearsal:
        return True, "rehearsal: every rank on cuda:0 by design (ECGPU_BENCH_ONE_DEVICE=1), not checked"
    seen = {}
    for p in per_rank:
        key = p.get("pci_bus_id") or p.get("uuid")
        if key is None:
            return False, f"rank {p.get('rank')} reported no PCI bus id or UUID: distinct devices unproven"
        seen.setdefault(key, []).append(p.get("rank"))
    dups = {k: v for k, v in seen.items() if len(v) > 1}
    if dups:
        return False, "ranks share a GPU: " + "; ".join(f"ranks {v} on {k}" for k, v in sorted(dups.items()))
    return True, f"{len(seen)} ranks on {len(seen)} distinct GPUs (PCI bus ids)"


def stripes_for_rank(total: int, rank: int, world: int) -> list:
    """Global stripe ids owned by a rank: round-robin."""
    return list(range(rank, total, world))


def global_stripe_ids(per_rank: int, rank: int, world: int) -> list:
    """The per_rank global ids of `rank` when every rank codes per_rank stripes."""
    return stripes_for_rank(per_rank * world, rank, world)


# ------------------------------------------------------------- host info ----
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


HOST_THREAD_CAP = 16  # the GPU box's CPU share per GPU (16 per one-GPU lease)


def cgroup_cpu_quota(root: str = "/sys/fs/cgroup"):
    """CPUs' worth of run time the cgroup grants this process (cgroup v2
    cpu.max, else v1 cfs quota / period), or None when unlimited / unknown.
    A one-GPU lease shows the whole machine in its affinity mask but is
    throttled to its share; threads beyond the quota would only queue."""
    try:
        with open(os.path.join(root, "cpu.max")) as f:
            quota, period = f.read().split()[:2]
        return None if quota == "max" else max(1, int(quota) // max(1, int(period)))
    except (OSError, ValueError):
        pass
    try:
        with open(os.path.join(root, "cpu", "cpu.cfs_quota_us")) as f:
            quota = int(f.read())
        with open(os.path.join(root, "cpu", "cpu.cfs_period_us")) as f:
            period = int(f.read())
        return None if quota <= 0 else max(1, quota // max(1, period))
    except (OSError, ValueError):
        return None


def affinity_cpus() -> list:
    try:
        return sorted(os.sched_getaffinity(0))
    except AttributeError:
        return list(range(os.cpu_count() or 1))


def host_cpus(cap=HOST_THREAD_CAP) -> list:
    """CPUs this process may run on (affinity), at most `cap` of them (the
    per-GPU share by default) and at most the cgroup's CPU quota."""
    cpus = affinity_cpus()
    quota = cgroup_cpu_quota()
    n = len(cpus) if cap is None else min(cap, len(cpus))
    if quota is not None:
        n = min(n, quota)
    return cpus[:max(1, n)] or [0]


def all_host_cpus() -> list:
    """Every CPU this process may run on (SURVEY.md §8d "all host cores"):
    the affinity mask, bounded by the cgroup quota."""
    return host_cpus(cap=None)


# ------------------------------------------------------------ CPU baseline ----
def cpu_baseline(seconds: float, host_stripe, k, m, erasures, threads: int = 1, o3: bool = False, cpus=None):
    """Reference CPU path on the host cores: oracle/_ref (the reference's own
    src/erasure_coding compiled -O2, or -O3 -march=x86-64-v3) if shipped, else
    our C restatement (oracle/ec_oracle.c).  Bounded sample of the same
    workload: ONE stripe of the GPU slab (copied to the host), encode (+ the
    step's decode), repeated until `seconds` of wall time.  With threads > 1
    each call is split by byte range over threads like the reference client's
    encode_mul_thread (client_main.cpp:1074-1164), in whole 8-B words with the
    remainder in the last range (the client gives it to thread 0); each thread is pinned to its own CPU (sched_setaffinity) and
    ctypes releases the GIL, so the threads run in parallel.

    Also the checker: the CPU's parity (and rebuilt shard) on that stripe must
    equal what the GPU left in HBM.  Returns (baseline dict, parity_ok)."""
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
    S = host_stripe.shape[1]
    M = o.vandermonde_coding_matrix(k, m)
    data = alloc_shards(k, S)
    for j in range(k):
        data[j][:S] = host_stripe[j]
    coding = alloc_shards(m, S)
    cpus = host_cpus() if cpus is None else cpus
    threads = max(1, min(threads, len(cpus)))
    # Every range but the last is a whole number of 8-B words, the last taking
    # the remainder: the reference's add / XOR loops run in 8-B words and write
    # up to 7 B past a range that is not (galois.cpp:452-465, :731-754), which
    # with the client's split (thread 0 takes the remainder; e.g. 4 MiB over 96
    # threads) lands in the next thread's range while that thread XORs into it.
    per = (S // threads) // 8 * 8
    ranges = [(t * per, per if t < threads - 1 else S - per * (threads - 1)) for t in range(threads)]

    def views(bufs, off, n):
        return [np.frombuffer((ctypes.c_uint8 * (n + 16)).from_address(b.ctypes.data + off), dtype=np.uint8)
                for b in bufs]

    parts = [(views(data, a, n), views(coding, a, n), n) for a, n in ranges]

    def one(p):
        d, c, n = p
        o.matrix_encode(k, m, M, d, c, n)
        if erasures:
            o.matrix_decode(k, m, M, 0, erasures, d, c, n)

    def run(t):
        os.sched_setaffinity(0, {cpus[t]})  # this thread only (Linux)
        one(parts[t])

    # one thread per byte range per call, joined per call, like the reference
    # client (pthread_create / pthread_join around each encode)
    iters, t0 = 0, time.perf_counter()
    while True:
        ts = [threading.Thread(target=run, args=(t,)) for t in range(threads)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        iters += 1
        el = time.perf_counter() - t0
        if el >= seconds or iters >= 2000:
            break
    ok = all(np.array_equal(coding[i][:S], host_stripe[k + i]) for i in range(m))
    if erasures:
        ok = ok and all(np.array_equal(data[j][:S], host_stripe[j]) for j in erasures if j < k)
    gib = iters * (2 if erasures else 1) * k * S / 2**30
    flags = "-O3 -march=x86-64-v3" if o3 else "-O2"
    src = f"reference src/erasure_coding compiled g++ {flags}" if o.kind == "reference" else "oracle/ec_oracle.c -O2"
    step = f"RS({k},{m}) {S >> 20} MiB stripe encode" + (f" + decode of erasures {set(erasures)}" if erasures else "")
    cap = ""
    if threads > 1:
        cap = (f" (of {len(affinity_cpus())} in the affinity mask, cgroup quota "
               f"{cgroup_cpu_quota() or 'none'}; the per-GPU share is {HOST_THREAD_CAP})")
    return ({"value": round(gib / el, 4), "unit": "GiB/s", "cores": threads, "kind": o.kind,
             "sample": f"{iters} x ({step}) on stripe 0 of the GPU slab, {threads} thread(s) pinned one per CPU{cap}, "
                       f"splitting byte ranges like client_main.cpp:1074-1164, {el:.1f} s, {src}, "
                       f"host CPU {cpu_model()}"}, ok)


# ----------------------------------------------------------- GPU helpers ----
def median(xs):
    s = sorted(xs)
    n = len(s)
    return s[n // 2] if n % 2 else 0.5 * (s[n // 2 - 1] + s[n // 2])


def time_launches(launch, stream, reps: int, warmup: int = 3) -> float:
    """Median device time (ms) of `launch` over `reps` runs, HIP events on
    the launch stream."""
    import torch
    for _ in range(warmup):
        launch()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for e0, e1 in evs:
        e0.record(stream)
        launch()
        e1.record(stream)
    torch.cuda.synchronize(stream.device)
    return median([e0.elapsed_time(e1) for e0, e1 in evs])


def fill_random(slab, ids, cfg_id):
    """Uniform random bytes per GLOBAL stripe id (zeros would flatter DVFS);
    the same global stripe gets the same bytes whichever rank owns it."""
    import torch
    for b, gid in enumerate(ids):
        g = torch.Generator(device=slab.device).manual_seed((cfg_id << 40) ^ (gid << 8) ^ 0xEC)
        slab[b].random_(0, 256, generator=g)


def roofline_entry(bytes_per_launch, ms):
    gbs = bytes_per_launch / (ms / 1e3) / 1e9
    return {"algorithmic_bytes_per_launch": int(bytes_per_launch), "median_launch_ms": round(ms, 4),
            "achieved_GBps": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4)}


def copy_ceiling(slab, shard, reps: int = 10):
    """Measured stream-copy ceiling on this GPU: the
    diagnostic 16-B copy kernel (libecgpu_diag.so, diag_copy) moving the first
    half of every stripe's shards onto the second half, i.e. the same bytes,
    shard stride and skew as the coding launches.  GB/s of (read + written)
    bytes, best of the 4 cache policies, or None without the library."""
    import ctypes

    import torch

    from erasure_coding_test_amd import _native as N
    path = os.path.join(N.LIB_DIR, "libecgpu_diag.so")
    if not os.path.exists(path):
        return None
    L = ctypes.CDLL(path)
    L.ecgpu_diag_launch.restype = ctypes.c_int
    L.ecgpu_diag_launch.argtypes = [ctypes.c_int] * 5 + [ctypes.c_void_p] * 4 + [
        ctypes.c_int, ctypes.c_longlong, ctypes.c_ulonglong, ctypes.c_ulonglong, ctypes.c_int, ctypes.c_void_p,
        ctypes.c_void_p]
    B, n_sh = slab.shape[0], slab.shape[1]
    half = n_sh // 2
    dev = slab.device
    src = torch.tensor([slab[b, i].data_ptr() for b in range(B) for i in range(half)], dtype=torch.int64, device=dev)
    dst = torch.tensor([slab[b, half + i].data_ptr() for b in range(B) for i in range(half)], dtype=torch.int64,
                       device=dev)
    stream = torch.cuda.current_stream(dev)
    best = None
    for policy in range(4):  # bit 0: non-temporal loads, bit 1: non-temporal stores
        rc = [0]

        def go():
            rc[0] = rc[0] or L.ecgpu_diag_launch(1, 1, 1, 1, policy, None, None, src.data_ptr(), dst.data_ptr(),
                                                 B * half, shard, 0, 0, 1, stream.cuda_stream, None)
        ms = time_launches(go, stream, reps, warmup=2)
        if rc[0] != 0:
            return None
        if best is None or ms < best[0]:
            best = (ms, policy)
    ms, policy = best
    return {"GBps": round(2 * shard * B * half / (ms / 1e3) / 1e9, 1), "median_launch_ms": round(ms, 4),
            "kernel": f"diag_copy 16 B/lane, shards 0..{half - 1} -> {half}..{n_sh - 1} of every stripe; best of the "
                      f"4 cache policies (here loads {'nt' if policy & 1 else 'plain'}, stores "
                      f"{'nt' if policy & 2 else 'plain'}), median of {reps}"}


def xor_stream_probe(slab, shard, k, m, reps: int = 10):
    """The coding launch's own streams without its arithmetic: the
    diagnostic kernel diag_xor_mix<k, m> (libecgpu_diag.so variant 16) issues
    k non-temporal 16-B loads and m non-temporal 16-B stores per lane over
    the same slab, shard stride and grid, with one XOR instead of the GF(2^8)
    multiplies.  A reference point for "is the arithmetic in the way?", NOT an
    upper bound: the arithmetic also spaces the stores out, and the real
    encode beats the probe on some shapes.  GB/s of (k + m) * S
    per stripe, best of uncapped and 3 / 4 resident workgroups per CU (the
    production residency caps, an unused dynamic LDS allocation); None
    without the library or for a (k, m) it does not instantiate."""
    import ctypes

    import torch

    from erasure_coding_test_amd import _native as N
    path = os.path.join(N.LIB_DIR, "libecgpu_diag.so")
    if not os.path.exists(path):
        return None
    L = ctypes.CDLL(path)
    L.ecgpu_diag_launch.restype = ctypes.c_int
    L.ecgpu_diag_launch.argtypes = [ctypes.c_int] * 5 + [ctypes.c_void_p] * 4 + [
        ctypes.c_int, ctypes.c_longlong, ctypes.c_ulonglong, ctypes.c_ulonglong, ctypes.c_int, ctypes.c_void_p,
        ctypes.c_void_p]
    B = slab.shape[0]
    dev = slab.device
    src = torch.tensor([slab[b, j].data_ptr() for b in range(B) for j in range(k)], dtype=torch.int64, device=dev)
    dst = torch.tensor([slab[b, k + i].data_ptr() for b in range(B) for i in range(m)], dtype=torch.int64,
                       device=dev)
    stream = torch.cuda.current_stream(dev)
    lds_per_cu = 160 << 10  # MI355X (gfx950) LDS per CU
    best = None
    saved = os.environ.get("ECGPU_DIAG_LDS")
    try:
        for blocks in (0, 3, 4):
            os.environ["ECGPU_DIAG_LDS"] = str((lds_per_cu // blocks) & ~511 if blocks else 0)
            rc = [0]

            def go():
                rc[0] = rc[0] or L.ecgpu_diag_launch(16, k, m, 1, 0, None, None, src.data_ptr(), dst.data_ptr(),
                                                     B, shard, 0, 0, 1, stream.cuda_stream, None)
            ms = time_launches(go, stream, reps, warmup=2)
            if rc[0] != 0:
                return None
            if best is None or ms < best[0]:
                best = (ms, blocks)
    finally:
        if saved is None:
            os.environ.pop("ECGPU_DIAG_LDS", None)
        else:
            os.environ["ECGPU_DIAG_LDS"] = saved
    ms, blocks = best
    return {"GBps": round((k + m) * shard * B / (ms / 1e3) / 1e9, 1), "median_launch_ms": round(ms, 4),
            "kernel": f"diag_xor_mix<{k},{m}>: the encode's {k} nt loads + {m} nt stores of 16 B per lane, one "
                      f"XOR, no multiplies; {'uncapped' if not blocks else f'{blocks} workgroups per CU'} "
                      f"(best of uncapped / 3 / 4), median of {reps}"}


def with_mix(entry, mix):
    """A configs entry against the XOR probe of its own streams (xor_stream_probe)."""
    if entry is not None and mix:
        entry["xor_probe_GBps"] = mix["GBps"]
        entry["vs_xor_probe"] = round(entry["achieved_GBps"] / mix["GBps"], 4)
    return entry


def e2e_host_pipelines(E, M, k, m, S, erasures, dev, stripes: int = 24, depth: int = 3, sync=None):
    """The north star's PCIe-inclusive rate (never `value`): `stripes` stripes
    of pinned host shards through the host pipelines, i.e. H2D, code and D2H
    of consecutive stripes overlapped on three HIP streams (client write path
    client_main.cpp:1714-1815: data in, parity out; read path :2055-2182:
    survivors in, the erased shards out).  After every rank's timed work: the
    link and the host memory are not shared with the timed region.  At N = 1
    rank 0 runs it after the CPU baselines; at N > 1 every rank runs it on its
    own GPU at once (e2e_all_ranks), `sync` -- a barrier -- starting each
    timed pass together.  Data GiB/s = k * S per stripe over the wall time of
    one pass (the first pass warms the pipelines); the last stripe's parity is
    checked against a device-resident encode of the same data, the decode
    against the shards it rebuilt."""
    import torch
    host = torch.empty((stripes, k + m, S), dtype=torch.uint8).pin_memory()
    g = torch.Generator(device=dev).manual_seed(0xE2E)
    src = torch.randint(0, 256, (k, S), dtype=torch.uint8, device=dev, generator=g)
    for s in range(stripes):
        host[s, :k].copy_(src)
        host[s, 0, :8].fill_(s)  # stripes differ
    torch.cuda.synchronize(dev)

    def timed_pass(p):
        def run():
            for s in range(stripes):
                p.submit([host[s, j] for j in range(k)], [host[s, k + i] for i in range(m)])
            p.drain()
        run()
        if sync is not None:
            sync()
        t0 = time.perf_counter()
        run()
        return time.perf_counter() - t0

    out = {"workload": f"RS({k},{m}) {S >> 20} MiB shards, {stripes} stripes of pinned host memory, "
                       f"pipeline depth {depth}, one GPU's PCIe link",
           "unit": "GiB/s of data shards", "note": "PCIe-inclusive; not the bench value (inputs resident in HBM)",
           "stripes": stripes, "data_bytes_per_pass": stripes * k * S, "host_numa_node": page_numa_node(host.data_ptr())}
    enc = E.HostPipeline(k, m, M, S, depth=depth, device=dev.index)
    t = timed_pass(enc)
    enc.close()
    last = host[stripes - 1]
    d = last[:k].to(dev)
    ref = torch.empty((m, S), dtype=torch.uint8, device=dev)
    E.encode_plan(k, m, M, dev.index).bind([[d[j] for j in range(k)]], [[ref[i] for i in range(m)]], S).launch()
    torch.cuda.synchronize(dev)
    out["encode"] = {"data_GiBps": round(stripes * k * S / t / 2**30, 2), "pass_ms": round(t * 1e3, 2),
                     "parity_ok": bool(torch.equal(ref.cpu(), last[k:]))}
    if erasures:
        want = last.clone()
        dec = E.HostPipeline.decoder(k, m, M, erasures, S, depth=depth, device=dev.index)
        host[:, erasures] = 0  # every stripe's erased shards are rebuilt by the timed passes
        t = timed_pass(dec)
        dec.close()
        out["decode"] = {"erasures": erasures, "data_GiBps": round(stripes * k * S / t / 2**30, 2),
                         "pass_ms": round(t * 1e3, 2), "rebuilt_ok": bool(torch.equal(host[stripes - 1], want))}
    del host
    return out


# ------------------------------------------------------- NUMA placement ----
def pci_numa_node(bus_id, sysfs="/sys/bus/pci/devices"):
    """The NUMA node a PCI device (a GPU, by its bus id) hangs off, or None."""
    if not bus_id:
        return None
    try:
        with open(os.path.join(sysfs, bus_id.lower(), "numa_node")) as f:
            n = int(f.read().strip())
        return n if n >= 0 else None
    except (OSError, ValueError):
        return None


def parse_cpulist(text: str) -> set:
    """'0-3,8,10-11' -> {0, 1, 2, 3, 8, 10, 11}"""
    out = set()
    for part in text.strip().split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        out.update(range(int(a), int(b or a) + 1))
    return out


def node_cpus(node, sysfs="/sys/devices/system/node"):
    try:
        with open(os.path.join(sysfs, f"node{node}", "cpulist")) as f:
            return parse_cpulist(f.read())
    except (OSError, ValueError):
        return set()


def page_numa_node(addr: int):
    """The NUMA node holding the page at `addr` (move_pages(2) query), or None."""
    import ctypes
    try:
        libc = ctypes.CDLL(None, use_errno=True)
        page = ctypes.c_void_p(addr & ~(os.sysconf("SC_PAGE_SIZE") - 1))
        status = ctypes.c_int(-1)
        sys_move_pages = 279  # x86-64
        rc = libc.syscall(ctypes.c_long(sys_move_pages), 0, ctypes.c_ulong(1), ctypes.byref(page), None,
                          ctypes.byref(status), 0)
        return int(status.value) if rc == 0 and status.value >= 0 else None
    except (OSError, AttributeError, ValueError):
        return None


def e2e_aggregate(per_rank: list) -> dict:
    """Whole-job PCIe-inclusive rate at N > 1: every rank's pass bytes over the
    slowest rank's pass time (the ranks start each pass together)."""
    out = {"unit": "GiB/s of data shards, all ranks", "ranks": len(per_rank),
           "note": "sum of the ranks' data bytes / the slowest rank's pass time; each timed pass starts on a barrier"}
    for leg in ("encode", "decode"):
        legs = [r.get(leg) for r in per_rank]
        if not legs or any(x is None for x in legs):
            continue
        total = sum(r["data_bytes_per_pass"] for r in per_rank)
        slowest = max(x["pass_ms"] for x in legs) / 1e3
        ok = all(x.get("parity_ok", x.get("rebuilt_ok", True)) for x in legs)
        out[leg] = {"data_GiBps": round(total / slowest / 2**30, 2), "slowest_pass_ms": round(slowest * 1e3, 2),
                    "per_rank_GiBps": [x["data_GiBps"] for x in legs], "ok": bool(ok)}
    return out


def e2e_all_ranks(E, M, k, m, S, erasures, dev, local, world, stripes):
    """N > 1: every rank's e2e pass on its own GPU and PCIe link at once, with
    the rank's threads (and so the first touch of its pinned buffers) on the
    NUMA node its GPU hangs off, when the host tells which that is."""
    import ctypes
    from erasure_coding_test_amd import _native as N
    buf = ctypes.create_string_buffer(64)
    bus = buf.value.decode() if N.lib.ecgpu_device_pci_bus_id(local, buf, len(buf)) == 0 else None
    gpu_node = pci_numa_node(bus)
    before = os.sched_getaffinity(0)
    near = (node_cpus(gpu_node) & before) if gpu_node is not None else set()
    if os.environ.get("ECGPU_BENCH_E2E_NUMA", "1") == "0":  # A/B switch: leave the affinity alone
        near = set()
    if near:
        os.sched_setaffinity(0, near)
    try:
        r = e2e_host_pipelines(E, M, k, m, S, erasures, dev, stripes=stripes, sync=lambda: barrier(world))
    finally:
        os.sched_setaffinity(0, before)
    r["gpu_numa_node"] = gpu_node
    r["threads_on_gpu_node"] = bool(near)
    r["thread_cpus"] = len(near) if near else len(before)
    return r


def load_traffic(name: str, workload_key: str, kernel_id: str, profiles_dir: str = ""):
    """(HBM bytes per launch, note) from the committed rocprofv3 PMC summary
    (profiles/pmc_<name>.json, written by profiles/summarize.py from separate
    --pmc FETCH_SIZE / WRITE_SIZE passes of this same bench command).  The
    bytes are given only when the record is for this workload AND for the
    kernels of the loaded library (its ecgpu_build_id(1), stored in the record
    as kernel_build_id); otherwise None and the reason."""
    p = os.path.join(profiles_dir or os.path.join(ROOT, "profiles"), f"pmc_{name}.json")
    try:
        with open(p) as f:
            d = json.load(f)
    except (OSError, ValueError) as ex:
        return None, f"no PMC record ({type(ex).__name__})"
    if d.get("workload_key") != workload_key:
        return None, f"PMC record is for workload {d.get('workload_key')}, not {workload_key}"
    if d.get("kernel_build_id") != kernel_id:
        return None, (f"PMC record measured kernel build {d.get('kernel_build_id')}, the loaded library is "
                      f"{kernel_id}: stale, not reported")
    return d.get("hbm_bytes_per_launch"), f"{d.get('from')} (kernel build {kernel_id})"


# Per configs-block entry (profiles/summarize.py relies on these counts).  The
# warm-up covers the DVFS transient a new back-to-back load starts with: the
# first 3-4 launches run at boost clock, the chip then drops its clock (1.5 GHz
# effective at launches 3-8) and recovers over ~20 launches; the multiply-dense
# C4 decode turns issue-bound in the dip (profiles/r05_c4_spread.json), so 5
# warm-ups left it timed inside the recovery.  25 puts every config at its
# settled clock, like the probes that time them in-process.
CFG_WARMUP, CFG_REPS = 25, 20
C3_RANDOM_DATA_ERASURE_SEED = 0xC3


def c3_random_data_erasure() -> int:
    """The seeded single data erasure of the C3 decode shapes (1..k-1; 0 is the
    timed decode{0})."""
    import random
    return random.Random(C3_RANDOM_DATA_ERASURE_SEED).randrange(1, 10)


def c3_decode_shapes(E, shards, S, B, dev, stream, kind, nt):
    """SURVEY.md §8d's other C3 decode shapes, on the timed slab: a lost
    parity shard (erasure {12}: the dense re-encode of row 2 from the data,
    jerasure.cpp:243-247) and a seeded single data erasure (jerasure.cpp:223-228;
    rebuilt from the other data shards and parity 0, whose Vandermonde row is
    all ones, so it is XOR-only like decode{0}).  Each rewrites its shard with
    the same bytes, so the slab stays a consistent stripe."""
    k, m = 10, 4
    M = E.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    out = {}
    j = c3_random_data_erasure()
    for name, er, what in (("C3_decode_data_random", [j], f"erasure {{{j}}} (seeded single data shard; XOR-only)"),
                           ("C3_decode_parity", [k + 2], "erasure {12} (lost parity: dense re-encode of row 2)")):
        dp = E.DecodePlan(k, m, M, er, 0, dev.index).bind_stripes(shards, S)
        dp.set_kernel(kind, nt)
        ms = time_launches(lambda: dp.launch(stream.cuda_stream), stream, CFG_REPS, warmup=CFG_WARMUP)
        e = {"workload": f"RS(10,4) decode of {what}, 4 MiB shards, {B} stripes (10 shards read, 1 written)"}
        e.update(roofline_entry((k + 1) * S * B, ms))
        out[name] = e
        dp.close()
    return out


def config_block(E, N, dev, stream, kind, nt, main=None):
    """Every BASELINE.json GPU config as its own launch (median of 20 HIP-event
    timed launches after warm-up; batches sized to 4.5-6.5 GB streamed per
    launch, like the timed C3 steps' 5.6 GB, so launch ramp and tail weigh
    the same in every config): C1's shape device-resident (RS(4,2) 64 KiB;
    C1 itself is the reference's CPU case), C2 encode, C3 encode / decode{0} (from the
    timed steps) and its other decode shapes (`main`, c3_decode_shapes),
    C4 decode{0,1,2,3} with its host-side plan cost reported separately
    (SURVEY.md §8d), C5 encode.  Runs on every rank, on its own GPU."""
    import ctypes

    import torch
    out = {}

    def encode_cfg(name, k, m, S, B, cfg_id, note=""):
        M = E.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
        slab, shards = E.alloc_stripes(B, k, m, S, dev)
        fill_random(slab, list(range(B)), cfg_id)
        p = E.encode_plan(k, m, M, dev.index).bind([st[:k] for st in shards], [st[k:] for st in shards], S)
        p.set_kernel(kind, nt)
        ms = time_launches(lambda: p.launch(stream.cuda_stream), stream, CFG_REPS, warmup=CFG_WARMUP)
        size = f"{S >> 20} MiB" if S >= 1 << 20 else f"{S >> 10} KiB"
        e = {"workload": f"RS({k},{m}) encode, {size} shards, {B} stripes{note}"}
        e.update(roofline_entry((k + m) * S * B, ms))
        p.close()
        out[name] = with_mix(e, xor_stream_probe(slab, S, k, m))  # after the timing: overwrites the parity
        del slab, shards

    # C1 is the reference's CPU-only case (BASELINE configs[0], timed as the CPU
    # baseline and through the drop-in); this is its shape device-resident
    encode_cfg("C1_encode_device", 4, 2, 64 << 10, 13653, 1,
               " (BASELINE C1's shape, device-resident; C1 itself is the CPU path)")
    encode_cfg("C2_encode", 6, 3, 1 << 20, 512, 2)
    if main is not None:
        out.update(main)
    # C4: worst-case decode, erasures {0,1,2,3} of RS(10,4) 4 MiB (10 survivors = ids 4..13)
    k, m, S, B = 10, 4, 4 << 20, 96
    M = E.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    slab, shards = E.alloc_stripes(B, k, m, S, dev)
    fill_random(slab, list(range(B)), 4)
    er = [0, 1, 2, 3]
    # host side, reported separately: the decode planning (erasures -> dm_ids ->
    # k x k GF inversion -> fused map, jerasure.cpp:84-112, :153-254) and the
    # whole plan creation (planning + coefficient tables + upload)
    n = k + m
    outs, srcs, coef = (ctypes.c_int * n)(), (ctypes.c_int * n)(), (ctypes.c_int * (n * n))()
    no, ns = ctypes.c_int(), ctypes.c_int()
    Mi, eri = N.int_array(M), N.int_array(er + [-1])
    host_us = []
    for _ in range(200):
        t0 = time.perf_counter()
        N.lib.ecgpu_decode_plan(k, m, 8, Mi, 0, eri, outs, ctypes.byref(no), srcs, ctypes.byref(ns), coef)
        host_us.append((time.perf_counter() - t0) * 1e6)
    create_us = []
    for _ in range(20):
        t0 = time.perf_counter()
        dp = E.DecodePlan(k, m, M, er, 0, dev.index)
        create_us.append((time.perf_counter() - t0) * 1e6)
        dp.close()
    dp = E.DecodePlan(k, m, M, er, 0, dev.index).bind_stripes(shards, S)
    dp.set_kernel(kind, nt)
    ms = time_launches(lambda: dp.launch(stream.cuda_stream), stream, CFG_REPS, warmup=CFG_WARMUP)
    e = {"workload": f"RS(10,4) decode of erasures {{0,1,2,3}}, 4 MiB shards, {B} stripes (10 survivors read, "
                     f"4 shards written)"}
    e.update(roofline_entry((k + len(er)) * S * B, ms))
    e["host_decode_plan_us"] = round(median(host_us), 2)
    e["host_plan_create_us"] = round(median(create_us), 2)
    e["host_note"] = ("host_decode_plan_us: ecgpu_decode_plan (survivor choice, k x k inversion, fused map) through "
                      "ctypes; host_plan_create_us: the whole DecodePlan incl. coefficient tables and their (asynchronous) upload; "
                      "medians, not in the launch time")
    dp.close()
    out["C4_decode_0123"] = with_mix(e, xor_stream_probe(slab, S, k, m))  # the same 10-read / 4-write streams
    del slab, shards
    encode_cfg("C5_encode", 12, 4, 16 << 20, 24, 5)
    torch.cuda.synchronize(dev)
    return out


# -------------------------------------------------------------------- main ----
def selftest_main(args):
    """--spawn-selftest: the multi-rank control path without a GPU."""
    rank, local, world = dist_setup()
    barrier(world)
    t = max_over_ranks(float(rank + 1), world)
    # a stand-in device identity per rank (ECGPU_SELFTEST_SAME_BUS=1: every
    # rank claims one device, which the distinct-device check must fail)
    bus = "selftest:00" if os.environ.get("ECGPU_SELFTEST_SAME_BUS") == "1" else f"selftest:{local:02d}"
    # a stand-in e2e pass per rank, through the same barrier-started timing,
    # gather and aggregation as the real N > 1 e2e leg (e2e_all_ranks)
    barrier(world)
    t0 = time.perf_counter()
    time.sleep(0.01 * (rank + 1))
    pass_ms = (time.perf_counter() - t0) * 1e3
    e2e = {"data_bytes_per_pass": 1 << 30, "host_numa_node": None, "gpu_numa_node": pci_numa_node(None),
           "encode": {"pass_ms": round(pass_ms, 2), "data_GiBps": round(1e3 / pass_ms, 2), "parity_ok": True}}
    per_rank = gather({"rank": rank, "local_rank": local, "world": world, "pid": os.getpid(), "pci_bus_id": bus,
                       "e2e": e2e}, world)
    devices_ok, devices_note = distinct_devices(per_rank, os.environ.get("ECGPU_BENCH_ONE_DEVICE") == "1")
    if rank == 0:
        e2e_per_rank = [p.pop("e2e") for p in per_rank]
        print(json.dumps({"selftest": True, "n_gpus": world, "max_over_ranks": t, "per_rank": per_rank,
                          "stripes": {r: global_stripe_ids(2, r, world) for r in range(world)},
                          "e2e_per_rank": e2e_per_rank, "e2e_aggregate": e2e_aggregate(e2e_per_rank),
                          "distinct_devices_ok": devices_ok, "distinct_devices": devices_note}), flush=True)
        if not devices_ok:
            print(f"bench.py: {devices_note}", file=sys.stderr, flush=True)
    barrier(world)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    return 0 if devices_ok else 1


def sharded_c5(E, N, dev, stream, kind, nt, rank, world, per_rank=24, launches=10):
    """BASELINE config 5 as a whole job: RS(12,4) encode of 16 MiB shards,
    `per_rank` stripes on every rank (global stripe ids round-robin, no
    collective), `launches` launches per rank bracketed by a barrier and a
    device sync on both sides, the slowest rank's time.  Every rank checks its
    first stripe against the other multiply engine.  Collective: every rank
    calls it.  Returns the entry (the same on every rank)."""
    import torch
    k, m, S = 12, 4, 16 << 20
    M = E.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    slab, shards = E.alloc_stripes(per_rank, k, m, S, dev)
    fill_random(slab, global_stripe_ids(per_rank, rank, world), 5)
    p = E.encode_plan(k, m, M, dev.index).bind([st[:k] for st in shards], [st[k:] for st in shards], S)
    p.set_kernel(kind, nt)
    for _ in range(3):
        p.launch(stream.cuda_stream)
    torch.cuda.synchronize(dev)
    barrier(world)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(launches):
        p.launch(stream.cuda_stream)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    barrier(world)
    t = max_over_ranks(elapsed, world)
    chk = torch.empty((m, S), dtype=torch.uint8, device=dev)
    ref = E.encode_plan(k, m, M, dev.index).bind([shards[0][:k]], [[chk[i] for i in range(m)]], S)
    ref.set_kernel(N.KERNEL_LDS if kind == N.KERNEL_PERM else N.KERNEL_PERM, True)
    ref.launch(stream.cuda_stream)
    torch.cuda.synchronize(dev)
    bad = 0.0 if all(bool(torch.equal(chk[i], shards[0][k + i])) for i in range(m)) else 1.0
    bad = max_over_ranks(bad, world)
    p.close()
    ref.close()
    del slab, shards, chk
    torch.cuda.empty_cache()
    per_gpu_bytes = (k + m) * S * per_rank * launches
    return {"workload": f"RS(12,4) encode, 16 MiB shards, {per_rank} stripes per GPU x {world} GPU(s), global "
                        "stripe ids round-robin, no collective (BASELINE config 5)",
            "n_gpus": world, "launches": launches, "ms_per_launch": round(t / launches * 1e3, 4),
            "data_GiBps": round(world * k * S * per_rank * launches / t / 2**30, 1),
            "hbm_frac_per_gpu": round(per_gpu_bytes / t / 1e9 / HBM_PEAK_GBS, 4),
            "timing": "host clock between barriers, slowest rank (includes launch gaps)",
            "parity_ok": bad == 0.0}


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    rehearsal = os.environ.get("ECGPU_BENCH_ONE_DEVICE") == "1"
    import torch
    count = 0 if args.spawn_selftest else torch.cuda.device_count()  # does not initialise the GPU
    mode, msg = launch_mode(args.gpus, os.environ, count, args.spawn_selftest)
    if mode == "error":
        print(f"bench.py: {msg}", file=sys.stderr, flush=True)
        return 2
    if mode == "spawn":
        return spawn_ranks(args.gpus, argv)
    if args.spawn_selftest:
        return selftest_main(args)

    rank, local, world = dist_setup()
    import erasure_coding_test_amd as E
    from erasure_coding_test_amd import _native as N

    if rehearsal:
        local = 0
    elif local >= count:
        print(f"bench.py: rank {rank} has LOCAL_RANK {local} but only {count} GPUs are visible", file=sys.stderr)
        return 2
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    C = CONFIGS[args.config]
    k, m, S = C["k"], C["m"], C["shard"]
    B = args.stripes or C["stripes"]
    erasures = C["erasures"]
    M = E.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)

    # B stripes x (k+m) shards in one HBM slab at the library's recommended
    # shard stride, ecgpu_recommended_shard_stride_km(S, k, m) = round_up(S, 256)
    # + the skew csrc/shard_stride.hpp measured for S (6 KiB at 4 MiB, 8 KiB at 16 MiB;
    # the line records it as config.shard_stride_bytes); global stripe ids
    # round-robin over ranks
    ids = global_stripe_ids(B, rank, world)
    slab, shards = E.alloc_stripes(B, k, m, S, dev)
    shard_stride = int(slab.stride(1))
    fill_random(slab, ids, C["cfg_id"])

    kind = N.KERNEL_LDS if args.kernel == "lds" else N.KERNEL_PERM
    enc = E.encode_plan(k, m, M, local).bind([st[:k] for st in shards], [st[k:] for st in shards], S)
    enc.set_kernel(kind, bool(args.nt))
    dec = None
    if erasures:
        dec = E.DecodePlan(k, m, M, erasures, 0, local).bind_stripes(shards, S)
        dec.set_kernel(kind, bool(args.nt))
    stream = torch.cuda.current_stream(dev)

    # HIP events on the launch stream, one per kernel boundary: event 0 opens
    # the region, step i's encode ends at event 2i+1 (1 + i without a decode)
    # and its decode at 2i+2, which also starts step i+1's encode (each event
    # record costs the stream ~5 us, so boundaries are not recorded twice)
    per = 2 if dec is not None else 1

    def step(i=None):
        enc.launch(stream.cuda_stream)
        if i is not None:
            evs[per * i + 1].record(stream)
        if dec is not None:
            dec.launch(stream.cuda_stream)
            if i is not None:
                evs[per * i + 2].record(stream)

    for _ in range(args.warmup):
        step()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(per * args.steps + 1)]
    for e in evs:  # torch creates the HIP event at its first record: do that here, not in the timed loop
        e.record(stream)
    torch.cuda.synchronize(dev)

    barrier(world)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    evs[0].record(stream)
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize(dev)
    # each rank's clock stops when its own GPU work has drained; the closing
    # barrier still brackets the region and the max over ranks below makes
    # the slowest rank the job's time (the barrier's own latency is not work)
    elapsed = time.perf_counter() - t0
    barrier(world)
    t = max_over_ranks(elapsed, world)

    enc_times = [evs[per * i].elapsed_time(evs[per * i + 1]) for i in range(args.steps)]
    enc_ms = median(enc_times)
    # roofline.achieved divides by the AVERAGE launch of the timed steps (the
    # bench contract); the medians stay for the like-for-like ratios against
    # the copy kernel, the XOR probe and the configs block
    enc_mean_ms = sum(enc_times) / len(enc_times)
    dec_ms = (median([evs[2 * i + 1].elapsed_time(evs[2 * i + 2]) for i in range(args.steps)]) if dec is not None
              else None)
    user_per_stripe = (2 if erasures else 1) * k * S
    value = world * args.steps * B * user_per_stripe / t / 2**30

    # independent check of the timed result on every rank: stripe 0 re-encoded
    # with the OTHER multiply engine (LDS nibble tables, gf_apply_lds), outside
    # the timed region and its statistics
    chk = torch.empty((m, S), dtype=torch.uint8, device=dev)
    ref = E.encode_plan(k, m, M, local).bind([shards[0][:k]], [[chk[i] for i in range(m)]], S)
    ref.set_kernel(N.KERNEL_LDS if kind == N.KERNEL_PERM else N.KERNEL_PERM, True)
    ref.launch(stream.cuda_stream)
    torch.cuda.synchronize(dev)
    ok = all(bool(torch.equal(chk[i], shards[0][k + i])) for i in range(m))
    # rank 0's stripe 0 for the CPU baseline (taken at every N: SURVEY.md §8d,
    # the reference CPU path timed in the same run)
    host_stripe = slab[0, :, :S].cpu().numpy() if (rank == 0 and args.cpu_seconds > 0) else None

    enc_bytes = (k + m) * S * B  # algorithmic HBM bytes per encode launch
    dec_bytes = (k + len(erasures)) * S * B if erasures else 0  # k survivors read + erased shards written
    main_entries = {}
    if not args.no_configs and args.config == "C3":
        e = {"workload": f"RS(10,4) encode, 4 MiB shards, {B} stripes (the timed steps)"}
        e.update(roofline_entry(enc_bytes, enc_ms))
        main_entries["C3_encode"] = e
        e = {"workload": f"RS(10,4) decode of erasure {{0}} (XOR-only), 4 MiB shards, {B} stripes (the timed steps)"}
        e.update(roofline_entry(dec_bytes, dec_ms))
        main_entries["C3_decode_0"] = e
        main_entries.update(c3_decode_shapes(E, shards, S, B, dev, stream, kind, bool(args.nt)))
    del enc, dec, ref
    copy = copy_ceiling(slab, S)  # after the parity checks: the copy overwrites the slab's second half
    mix = xor_stream_probe(slab, S, k, m)  # overwrites the parity shards
    if main_entries:
        with_mix(main_entries["C3_encode"], mix)
        mix_dec = xor_stream_probe(slab, S, k, 1)  # every C3 decode shape reads 10 shards and writes 1
        for name in ("C3_decode_0", "C3_decode_data_random", "C3_decode_parity"):
            with_mix(main_entries.get(name), mix_dec)
    # diagnostics only (A/B of the N > 1 e2e leg): ECGPU_BENCH_SKIP=configs,c5 drops those blocks
    skip = set(filter(None, os.environ.get("ECGPU_BENCH_SKIP", "").split(",")))
    configs = None
    if not args.no_configs and "configs" not in skip:
        del shards
        slab = None
        torch.cuda.empty_cache()
        configs = config_block(E, N, dev, stream, kind, bool(args.nt), main_entries)
    c5 = None
    if not args.no_configs and args.config == "C3" and "c5" not in skip:
        c5 = sharded_c5(E, N, dev, stream, kind, bool(args.nt), rank, world)
    # about 1.5 GiB of pinned host memory per rank at most (C3: 24 stripes, C5: 6)
    e2e_n = min(args.e2e_stripes, max(2, (3 << 29) // ((k + m) * S)))
    e2e_mine = None
    if world > 1 and args.e2e_stripes > 0:
        repeats = []
        for _ in range(max(1, int(os.environ.get("ECGPU_BENCH_E2E_REPEAT", "1") or 1))):  # diagnostics: >1 repeats
            barrier(world)
            e2e_mine = e2e_all_ranks(E, M, k, m, S, erasures, dev, local, world, e2e_n)
            barrier(world)
            repeats.append({leg: e2e_mine[leg]["pass_ms"] for leg in ("encode", "decode") if leg in e2e_mine})
        if len(repeats) > 1:
            e2e_mine["repeats_pass_ms"] = repeats

    enc_frac = enc_bytes / (enc_mean_ms / 1e3) / 1e9 / HBM_PEAK_GBS
    mine = {"rank": rank, "device": local, **device_identity(N, local), "elapsed_s": round(elapsed, 6),
            "encode_mean_ms": round(enc_mean_ms, 4), "encode_median_ms": round(enc_ms, 4),
            "encode_launch_ms": [round(x, 4) for x in enc_times],  # in step order: the DVFS recovery shows here
            "encode_frac": round(enc_frac, 4),
            "decode_median_ms": round(dec_ms, 4) if dec_ms is not None else None,
            "decode_frac": (round(dec_bytes / (dec_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4) if dec_ms is not None
                            else None),
            "stripe_ids": [ids[0], ids[-1], len(ids)], "parity_ok": ok,
            "copy_ceiling_GBps": copy["GBps"] if copy else None,
            "xor_probe_GBps": mix["GBps"] if mix else None}
    if configs:
        mine["configs"] = {name: {"median_launch_ms": e["median_launch_ms"], "frac": e["frac"]}
                           for name, e in configs.items()}
    if e2e_mine is not None:
        mine["e2e"] = e2e_mine
    # no GPU result may come from the drop-in's CPU fallback or
    # its CPU executor for small host calls (ECGPU_MIN_OFFLOAD_KIB); the
    # package keeps both off, and a nonzero count fails the run
    mine["cpu_fallbacks"] = N.fallback_count()
    mine["cpu_calls"] = N.cpu_call_count()
    per_rank = gather(mine, world)
    ok = (all(p["parity_ok"] for p in per_rank) and (c5 is None or c5["parity_ok"]) and
          all(p["cpu_fallbacks"] == 0 and p["cpu_calls"] == 0 for p in per_rank))
    devices_ok, devices_note = distinct_devices(per_rank, rehearsal)
    barrier(world)  # every rank's GPU work is done: the CPU baseline below runs alone

    workload = C["workload"].format(B=B)
    cpu_ok = None
    if rank == 0:
        cpu = cpu_share = cpu_all = cpu_o3 = None
        if host_stripe is not None:
            cpu, cpu_ok = cpu_baseline(args.cpu_seconds, host_stripe, k, m, erasures)
            share = host_cpus()
            cpu_share, ok_share = cpu_baseline(max(2.0, args.cpu_seconds / 2), host_stripe, k, m, erasures,
                                               threads=len(share), cpus=share)
            cpu_ok = cpu_ok and ok_share
            every = all_host_cpus()
            if len(every) > len(share):  # a whole host (the 8-GPU node): every core it gives us
                cpu_all, ok_all = cpu_baseline(max(2.0, args.cpu_seconds / 2), host_stripe, k, m, erasures,
                                               threads=len(every), cpus=every)
                cpu_ok = cpu_ok and ok_all
            else:  # a one-GPU lease: its share is all there is
                cpu_all = dict(cpu_share, note="the per-GPU share is every CPU this process may use here")
            from oracle.oracle import REFERENCE_O3_SO
            if host_has_avx2() and os.path.exists(REFERENCE_O3_SO):
                cpu_o3, ok_o3 = cpu_baseline(max(2.0, args.cpu_seconds / 2), host_stripe, k, m, erasures, o3=True)
                cpu_ok = cpu_ok and ok_o3
        e2e_per_rank = e2e_agg = None
        if world > 1:
            e2e_per_rank = [p.pop("e2e", None) for p in per_rank]
            e2e = e2e_per_rank[0]
            e2e_agg = e2e_aggregate(e2e_per_rank) if all(e2e_per_rank) else None
        else:
            e2e = e2e_host_pipelines(E, M, k, m, S, erasures, dev, stripes=e2e_n) if args.e2e_stripes > 0 else None
        e2e_ok = (None if not e2e else
                  all(bool(r["encode"]["parity_ok"] and r.get("decode", {}).get("rebuilt_ok", True))
                      for r in (e2e_per_rank or [e2e])))
        achieved = enc_bytes / (enc_mean_ms / 1e3) / 1e9
        achieved_median = enc_bytes / (enc_ms / 1e3) / 1e9
        wkey = f"{args.config}:{B}"
        kernel_id = N.lib.ecgpu_build_id(1).decode()
        traffic, traffic_note = load_traffic("encode", wkey, kernel_id)
        dec_traffic, dec_traffic_note = load_traffic("decode", wkey, kernel_id)
        fracs = [p["encode_frac"] for p in per_rank]
        out = {
            "metric": C["metric"],
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
            "data": "synthetic (uniform random bytes, device-generated per global stripe id)",
            "config": {"workload": workload, "k": k, "m": m, "shard_bytes": S, "stripes_per_gpu": B,
                       "shard_stride_bytes": shard_stride,
                       "erasures": erasures, "kernel": args.kernel, "nontemporal": bool(args.nt),
                       "parallelism": f"stripes round-robin over {world} GPU(s), no collective"},
            "rehearsal": rehearsal,
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_note,
                         "frac_worst_rank": min(fracs), "frac_per_rank": fracs,
                         "kernel": "gf_apply (encode launch, rank 0)", "algorithmic_bytes_per_launch": enc_bytes,
                         "mean_launch_ms": round(enc_mean_ms, 4), "median_launch_ms": round(enc_ms, 4),
                         "kernel_time_stat": f"mean of the {args.steps} timed encode launches (HIP events on the "
                                             f"launch stream); frac at the median: "
                                             f"{round(achieved_median / HBM_PEAK_GBS, 4)}",
                         # the north star's read-only accounting: data-shard bytes only, which
                         # caps at k/(k+m) of peak for any encode
                         "read_only_frac": round(k * S * B / (enc_mean_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4)},
            "copy_ceiling": copy,
            "encode_frac_of_copy": round(achieved_median / copy["GBps"], 4) if copy else None,  # medians both
            "xor_stream_probe": mix,
            "encode_vs_xor_probe": round(achieved_median / mix["GBps"], 4) if mix else None,  # medians both
            "decode_kernel": ({"erasures": erasures, "median_launch_ms": round(dec_ms, 4),
                               "algorithmic_bytes_per_launch": dec_bytes,
                               "achieved_GBps": round(dec_bytes / (dec_ms / 1e3) / 1e9, 1),
                               "traffic": dec_traffic, "traffic_source": dec_traffic_note,
                               "note": "decode{0} is XOR-only (parity 0 is the all-ones row); the decodes that "
                                       "multiply are configs.C3_decode_parity and configs.C4_decode_0123"}
                              if dec_ms is not None else None),
            "per_rank": per_rank,
            "configs": configs,
            "c5_sharded": c5,
            "cpu_baseline": cpu,
            "cpu_baseline_per_gpu_share": cpu_share,
            "cpu_baseline_all_cores": cpu_all,
            "cpu_baseline_o3": cpu_o3,
            "e2e": e2e,
            **({"e2e_per_rank": e2e_per_rank, "e2e_aggregate": e2e_agg} if world > 1 else {}),
            "cpu_fallbacks": sum(p["cpu_fallbacks"] for p in per_rank),
            "cpu_calls": sum(p["cpu_calls"] for p in per_rank),
            "selfcheck_parity_ok": ok,
            "selfcheck_vs_reference_cpu": cpu_ok,
            "e2e_ok": e2e_ok,
            "distinct_devices_ok": devices_ok,
            "distinct_devices": devices_note,
            "build_id": {"library": N.lib.ecgpu_build_id(0).decode(), "kernels": kernel_id},
        }
        print(json.dumps(out), flush=True)
        if e2e_ok is False:
            ok = False
        if not devices_ok:
            print(f"bench.py: {devices_note}", file=sys.stderr, flush=True)
            ok = False
    barrier(world)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    return 0 if ok and cpu_ok is not False else 1


if __name__ == "__main__":
    sys.exit(main())
