"""bench.py's multi-rank launch logic on the CPU (no GPU needed).

`--gpus N` must yield N ranks or fail: without WORLD_SIZE the bench spawns N
rank processes itself (before touching a GPU); with too few visible GPUs, or
a WORLD_SIZE that disagrees with --gpus, it exits non-zero.  The spawn ->
gloo rendezvous -> max-reduce -> per-rank report path runs end to end here
with --spawn-selftest.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


@pytest.mark.parametrize("gpus,env,count,want", [
    (1, {}, 1, "run"),
    (1, {}, 0, "run"),                                   # N = 1 runs in process (fails later without a GPU)
    (4, {}, 8, "spawn"),
    (4, {}, 2, "error"),                                 # fewer visible GPUs than --gpus
    (2, {"ECGPU_BENCH_ONE_DEVICE": "1"}, 1, "spawn"),    # labelled rehearsal on one device
    (2, {"ECGPU_BENCH_ONE_DEVICE": "1"}, 0, "error"),
    (8, {"WORLD_SIZE": "8"}, 8, "run"),                  # the driver's torch.distributed.run form
    (8, {"WORLD_SIZE": "4"}, 8, "error"),                # WORLD_SIZE disagrees with --gpus
    (2, {"WORLD_SIZE": "2"}, 1, "error"),
    (0, {}, 8, "error"),
])
def test_launch_mode(gpus, env, count, want):
    mode, msg = bench.launch_mode(gpus, env, count)
    assert mode == want, msg
    assert (msg != "") == (want == "error")


def test_rank_envs():
    envs = bench.rank_envs(3, 12345, {"X": "1"})
    assert [(e["RANK"], e["LOCAL_RANK"], e["WORLD_SIZE"]) for e in envs] == [("0", "0", "3"), ("1", "1", "3"),
                                                                               ("2", "2", "3")]
    assert all(e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "12345" and e["X"] == "1" for e in envs)


def test_global_stripe_ids_round_robin():
    per_rank, world = 3, 4
    owned = [bench.global_stripe_ids(per_rank, r, world) for r in range(world)]
    assert owned[1] == [1, 5, 9]
    assert sorted(i for o in owned for i in o) == list(range(per_rank * world))


def _env():
    env = dict(os.environ)
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "ECGPU_BENCH_ONE_DEVICE"):
        env.pop(v, None)
    return env


@pytest.mark.parametrize("world", [2, 3, 8])  # 8: the driver's scaling run
def test_spawn_selftest_end_to_end(world):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--spawn-selftest"],
                       capture_output=True, text=True, timeout=240, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    # stdout is exactly rank 0's one JSON line: gloo's connection reports go to stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == world and d["max_over_ranks"] == float(world)
    assert [p["rank"] for p in d["per_rank"]] == list(range(world))
    assert [p["local_rank"] for p in d["per_rank"]] == list(range(world))
    assert len({p["pid"] for p in d["per_rank"]}) == world  # one process per rank


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="checks the no-GPU refusal")
def test_gpus2_without_gpus_exits_nonzero():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], capture_output=True,
                       text=True, timeout=120, env=_env(), cwd=ROOT)
    assert r.returncode == 2
    assert "needs 2 visible GPUs" in r.stderr


def test_world_size_mismatch_exits_nonzero():
    env = _env()
    env["WORLD_SIZE"] = "3"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], capture_output=True,
                       text=True, timeout=120, env=env, cwd=ROOT)
    assert r.returncode == 2
    assert "WORLD_SIZE=3" in r.stderr


def test_distinct_devices_check():
    two = [{"rank": 0, "pci_bus_id": "0000:05:00.0"}, {"rank": 1, "pci_bus_id": "0000:05:00.0"}]
    ok, note = bench.distinct_devices(two, rehearsal=False)
    assert not ok and "ranks [0, 1] on 0000:05:00.0" in note
    assert bench.distinct_devices(two, rehearsal=True)[0]  # a labelled rehearsal shares cuda:0 on purpose
    two[1]["pci_bus_id"] = "0000:15:00.0"
    assert bench.distinct_devices(two, rehearsal=False) == (True, "2 ranks on 2 distinct GPUs (PCI bus ids)")
    two[1]["pci_bus_id"] = None
    two[1]["uuid"] = None
    assert not bench.distinct_devices(two, rehearsal=False)[0]  # unproven is a failure
    assert bench.distinct_devices(two[:1], rehearsal=False)[0]


def test_selftest_fails_ranks_on_one_device():
    """End to end through spawn -> gloo -> gather: two ranks claiming the same
    device make rank 0 exit non-zero, with the reason in the line."""
    env = _env()
    env["ECGPU_SELFTEST_SAME_BUS"] = "1"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--spawn-selftest"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 1, r.stderr[-2000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.strip()][0])
    assert d["distinct_devices_ok"] is False and "share a GPU" in r.stderr
    env["ECGPU_BENCH_ONE_DEVICE"] = "1"  # the rehearsal flag suppresses the check
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--spawn-selftest"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]


def test_cgroup_cpu_quota(tmp_path):
    assert bench.cgroup_cpu_quota(str(tmp_path)) is None  # no cgroup files: unlimited
    (tmp_path / "cpu.max").write_text("max 100000\n")
    assert bench.cgroup_cpu_quota(str(tmp_path)) is None
    (tmp_path / "cpu.max").write_text("1600000 100000\n")
    assert bench.cgroup_cpu_quota(str(tmp_path)) == 16
    (tmp_path / "cpu.max").unlink()
    (tmp_path / "cpu").mkdir()
    (tmp_path / "cpu" / "cpu.cfs_quota_us").write_text("800000\n")
    (tmp_path / "cpu" / "cpu.cfs_period_us").write_text("100000\n")
    assert bench.cgroup_cpu_quota(str(tmp_path)) == 8
    assert 1 <= len(bench.host_cpus()) <= bench.HOST_THREAD_CAP
    assert len(bench.all_host_cpus()) >= len(bench.host_cpus())


@pytest.mark.parametrize("threads", [1, 7])
def test_cpu_baseline_thread_split_keeps_parity(threads):
    """The multi-thread CPU baseline splits a stripe by byte range like the
    reference client, in whole 8-B words: 7 x 599,193 + 3 B over 7 threads is
    not, and the reference's word loops would otherwise write up to 7 B into
    the next thread's range while that thread runs (the baseline's parity
    check catches that)."""
    import numpy as np

    from oracle.oracle import Reference, Restatement, alloc_shards
    try:
        o = Reference()
    except (FileNotFoundError, OSError):
        o = Restatement()
    k, m, S = 10, 4, 7 * 599193 + 3
    rng = np.random.default_rng(5)
    data = alloc_shards(k, S)
    for d in data:
        d[:S] = rng.integers(0, 256, S, dtype=np.uint8)
    coding = alloc_shards(m, S)
    o.matrix_encode(k, m, o.vandermonde_coding_matrix(k, m), data, coding, S)
    stripe = np.stack([d[:S] for d in data] + [c[:S] for c in coding])
    cpus = sorted(os.sched_getaffinity(0))
    cpus = (cpus * threads)[:threads]
    for _ in range(3):
        base, ok = bench.cpu_baseline(0.2, stripe, k, m, [0], threads=threads, cpus=cpus)
        assert ok and base["cores"] == threads
