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


@pytest.mark.parametrize("world", [2, 3])
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
