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
    # the N > 1 e2e leg's gather and aggregation (stand-in passes of 10 ms x (rank + 1))
    assert len(d["e2e_per_rank"]) == world and d["e2e_aggregate"]["ranks"] == world
    slowest = max(r["encode"]["pass_ms"] for r in d["e2e_per_rank"])
    assert d["e2e_aggregate"]["encode"]["slowest_pass_ms"] == round(slowest, 2) >= 10 * world
    assert d["e2e_aggregate"]["encode"]["data_GiBps"] == round(world * 1e3 / slowest, 2)


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


# ---------------------------------------------- N > 1 e2e ----
def test_parse_cpulist_and_node_lookup(tmp_path):
    import bench
    assert bench.parse_cpulist("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}
    assert bench.parse_cpulist("") == set()
    pci = tmp_path / "pci" / "0000:8e:00.0"
    pci.mkdir(parents=True)
    (pci / "numa_node").write_text("1\n")
    assert bench.pci_numa_node("0000:8E:00.0", sysfs=str(tmp_path / "pci")) == 1
    (pci / "numa_node").write_text("-1\n")  # no affinity reported
    assert bench.pci_numa_node("0000:8e:00.0", sysfs=str(tmp_path / "pci")) is None
    assert bench.pci_numa_node(None) is None and bench.pci_numa_node("0000:ff:00.0", sysfs=str(tmp_path)) is None
    node = tmp_path / "node" / "node1"
    node.mkdir(parents=True)
    (node / "cpulist").write_text("48-95,144-191\n")
    assert bench.node_cpus(1, sysfs=str(tmp_path / "node")) == set(range(48, 96)) | set(range(144, 192))
    assert bench.node_cpus(7, sysfs=str(tmp_path / "node")) == set()


def test_page_numa_node_of_own_memory():
    import numpy as np

    import bench
    a = np.ones(1 << 20, np.uint8)
    n = bench.page_numa_node(a.ctypes.data)
    assert n is None or n >= 0


def test_e2e_aggregate_is_total_over_slowest():
    import bench
    rank = lambda ms_e, ms_d, ok=True: {"data_bytes_per_pass": 10 * 2**30,  # noqa: E731
                                        "encode": {"pass_ms": ms_e, "data_GiBps": 10 / (ms_e / 1e3),
                                                   "parity_ok": ok},
                                        "decode": {"pass_ms": ms_d, "data_GiBps": 10 / (ms_d / 1e3),
                                                   "rebuilt_ok": True}}
    agg = bench.e2e_aggregate([rank(200.0, 250.0), rank(250.0, 200.0), rank(100.0, 100.0)])
    assert agg["ranks"] == 3
    assert agg["encode"]["data_GiBps"] == round(30 / 0.25, 2) and agg["encode"]["slowest_pass_ms"] == 250.0
    assert agg["decode"]["data_GiBps"] == round(30 / 0.25, 2) and agg["encode"]["ok"] and agg["decode"]["ok"]
    assert agg["encode"]["per_rank_GiBps"] == [50.0, 40.0, 100.0]
    bad = bench.e2e_aggregate([rank(1.0, 1.0), rank(1.0, 1.0, ok=False)])
    assert bad["encode"]["ok"] is False
    enc_only = bench.e2e_aggregate([{"data_bytes_per_pass": 2**30, "encode": {"pass_ms": 10.0, "data_GiBps": 100.0,
                                                                            "parity_ok": True}}])
    assert "decode" not in enc_only and enc_only["encode"]["data_GiBps"] == 100.0
