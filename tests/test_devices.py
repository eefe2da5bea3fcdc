"""Which device a synchronous call runs on, and which engine its launch takes.

* ECGPU_DEVICES / ecgpu_set_devices: unchanged
  concurrent callers -- the reference client's byte-range encode pthreads,
  client_main.cpp:1074-1164 -- are spread over a device list, one entry per
  calling thread, round-robin in the order threads make their first call.
  Off by default (one device); the multi-GPU gain is unmeasured on this
  one-GPU pool, so the GPU test repeats device 0.
* The per-context plan cache is keyed on the engine and store-policy knobs
  too: a knob switched between two identical synchronous calls
  reaches the second call's launch.
"""
import os
import subprocess
import sys
import threading

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _thread_devices(N, nthreads, calls=2):
    got = [None] * nthreads

    def work(i):
        got[i] = [N.lib.ecgpu_call_device() for _ in range(calls)]
    ts = [threading.Thread(target=work, args=(i,)) for i in range(nthreads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    return got


def test_device_list_round_robin_per_thread():
    from erasure_coding_test_amd import _native as N
    try:
        N.set_devices([2, 5, 7])
        assert N.get_devices() == [2, 5, 7]
        got = _thread_devices(N, 6)
        assert all(a == b for a, b in got), got  # a thread keeps its device
        assert sorted(a for a, _ in got) == [2, 2, 5, 5, 7, 7], got  # round-robin over threads
        N.set_devices([4])
        assert [a for a, _ in _thread_devices(N, 3)] == [4, 4, 4]  # a new list re-assigns
        N.set_knob("ECGPU_DEVICE", 1)  # a forced device wins
        assert N.lib.ecgpu_call_device() == 1
    finally:
        N.reset_knob("ECGPU_DEVICE")
        N.set_devices(None)
    assert N.get_devices() == []


@pytest.mark.parametrize("env,want", [("1,1,3", [1, 1, 3]), ("0", [0]), ("1,x", []), ("", []), ("-2", [])])
def test_devices_environment(env, want):
    code = ("from erasure_coding_test_amd import _native as N\n"
            "print(N.get_devices())\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, cwd=ROOT,
                       env=dict(os.environ, ECGPU_DEVICES=env))
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip().splitlines()[-1] == str(want)


def test_set_devices_rejects_bad_arguments():
    from erasure_coding_test_amd import _native as N
    with pytest.raises(N.EcgpuError):
        N.set_devices([0, -1])
    assert N.lib.ecgpu_set_devices(-1, None) == N.ECGPU_ERR_ARG


# ------------------------------------------------------------------ GPU ----
@pytest.mark.gpu
def test_device_list_names_only_visible_devices_gpu(gpu):
    """A list naming a device this process cannot see is rejected by
    ecgpu_set_devices and ignored (with one stderr line) from ECGPU_DEVICES:
    otherwise every call on it would fail or complete on the CPU."""
    import torch

    from erasure_coding_test_amd import _native as N
    n = torch.cuda.device_count()
    with pytest.raises(N.EcgpuError, match="not visible"):
        N.set_devices([0, n])
    assert N.get_devices() == []
    N.set_devices([n - 1, 0])
    try:
        assert N.get_devices() == [n - 1, 0]
    finally:
        N.set_devices(None)
    code = ("from erasure_coding_test_amd import _native as N\n"
            "print(N.get_devices())\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, cwd=ROOT,
                       env=dict(os.environ, ECGPU_DEVICES=f"0,{n}"))
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip().splitlines()[-1] == "[]"
    assert "not visible" in r.stderr
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, cwd=ROOT,
                       env=dict(os.environ, ECGPU_DEVICES="all"))
    assert r.returncode == 0 and r.stdout.strip().splitlines()[-1] == str(list(range(n))), r.stderr[-2000:]
    # a forced ECGPU_DEVICE the process cannot see is ignored the same way
    code = ("from erasure_coding_test_amd import _native as N\n"
            "print(N.lib.ecgpu_call_device())\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, cwd=ROOT,
                       env=dict(os.environ, ECGPU_DEVICE=str(n)))
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip().splitlines()[-1] == "0" and f"ECGPU_DEVICE={n} ignored" in r.stderr


@pytest.mark.gpu
def test_concurrent_pageable_encodes_over_a_device_list_gpu(gpu, restatement):
    """8 threads, each an unchanged caller's pageable RS(10,4) 4 MiB encode,
    spread over ECGPU_DEVICES = 0,0: every thread's parity bit-exact."""
    from erasure_coding_test_amd import _native as N, jerasure as J, reed_sol as R
    from oracle.oracle import alloc_shards
    k, m, size = 10, 4, 4 << 20
    M = R.reed_sol_vandermonde_coding_matrix(k, m, 8)
    rng = np.random.default_rng(55)
    jobs = []
    for t in range(8):
        data = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(k)]
        jobs.append((data, [np.zeros(size, np.uint8) for _ in range(m)]))
    errors, devs = [], [None] * 8

    def work(i):
        try:
            devs[i] = N.lib.ecgpu_call_device()
            J.jerasure_matrix_encode(k, m, 8, M, jobs[i][0], jobs[i][1], size)
        except Exception as ex:  # noqa: BLE001 -- reported below
            errors.append(repr(ex))
    try:
        N.set_devices([0, 0])
        ts = [threading.Thread(target=work, args=(i,)) for i in range(8)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
    finally:
        N.set_devices(None)
    assert not errors, errors
    assert devs == [0] * 8
    Mn = np.array(M).reshape(m, k)
    for data, coding in jobs:
        hd = alloc_shards(k, size)
        for a, h in zip(hd, data):
            a[:size] = h
        hc = alloc_shards(m, size)
        restatement.matrix_encode(k, m, Mn, hd, hc, size)
        for got, want in zip(coding, hc):
            assert np.array_equal(got, want[:size])


@pytest.mark.gpu
def test_engine_knob_reaches_a_cached_plan_gpu(gpu, knobs):
    """a synchronous call caches its plan per context; the
    engine knob switched between two identical calls must reach the second
    call's launch (the plan key holds the engine and store policy)."""
    import torch

    from erasure_coding_test_amd import _native as N, jerasure as J, reed_sol as R
    k, m, size = 10, 4, 1 << 20
    M = R.reed_sol_vandermonde_coding_matrix(k, m, 8)
    g = torch.Generator(device=gpu).manual_seed(7)
    data = [torch.randint(0, 256, (size,), dtype=torch.uint8, device=gpu, generator=g) for _ in range(k)]
    c0 = [torch.zeros(size, dtype=torch.uint8, device=gpu) for _ in range(m)]
    c1 = [torch.zeros(size, dtype=torch.uint8, device=gpu) for _ in range(m)]
    knobs.set("ECGPU_INLINE", 0)  # the plan path (inline calls carry no plan)
    perm0, lds0 = N.lib.ecgpu_engine_launches(0), N.lib.ecgpu_engine_launches(1)
    J.jerasure_matrix_encode(k, m, 8, M, data, c0, size)
    perm1, lds1 = N.lib.ecgpu_engine_launches(0), N.lib.ecgpu_engine_launches(1)
    assert perm1 > perm0 and lds1 == lds0
    knobs.set("ECGPU_KERNEL", 1)
    J.jerasure_matrix_encode(k, m, 8, M, data, c1, size)
    assert N.lib.ecgpu_engine_launches(1) > lds1 and N.lib.ecgpu_engine_launches(0) == perm1
    for a, b in zip(c0, c1):
        assert torch.equal(a, b)
    knobs.set("ECGPU_KERNEL", 0)
    J.jerasure_matrix_encode(k, m, 8, M, data, c1, size)
    assert N.lib.ecgpu_engine_launches(0) > perm1
