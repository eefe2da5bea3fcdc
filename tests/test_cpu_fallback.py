"""SURVEY.md §8b's failure contract: "the GPU layer must add no new failure
modes; on any HIP error it falls back to the CPU and records it".

libjerasure_amd.so (ECGPU_CPU_FALLBACK=1, its default) completes a synchronous
host-memory call on the CPU -- the library's own executor of the planned map,
csrc/cpu_fallback.cpp, never oracle/ -- when a HIP error comes before any
caller byte was written; it counts the fallback (ecgpu_fallback_count) and
logs the first one.  With the knob at 0 the unchanged caller sees the old
failure channel (exit 1 / decode -1).  A call that already wrote caller
memory, or names device memory, keeps the error.

The reference's own call sequences (tests/fallback_driver.py: the client's
encode / decode, the ECX datanode's per-block region ops, the rest of the
header surface) run in subprocesses through the C++-mangled names, with
ECGPU_TEST_INJECT_HIP (the drivers set the library's in-process-only
test_inject_hip knob from it) forcing the HIP error: 1 before the first
launch, 2 the same plus the device marked lost (sticky), 3 after caller memory
was written -- recoverable unless an output is also a source.  One GPU test
takes a genuine HIP error instead: HBM filled until the staging hipMalloc
fails.
On this CPU container the HIP calls fail by themselves (no device) and the
injection changes nothing; on the MI355X box (-m gpu) the injection is what
fails them.  The outputs are checked against the golden fixtures and the
reference built in oracle/_ref.

Everything else in the suite runs with the fallback off (the Python package's
default, tests/conftest.py) and asserts the count stays 0.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(ROOT, "tests", "fallback_driver.py")
SCENARIOS = ["client", "ecx", "surface"]


def drive(scenario, fallback, inject, timeout=600, extra_env=None):
    env = dict(os.environ)
    env["ECGPU_CPU_FALLBACK"] = str(fallback)
    env["ECGPU_TEST_INJECT_HIP"] = str(inject)
    env.update(extra_env or {})
    r = subprocess.run([sys.executable, DRIVER, scenario], capture_output=True, text=True, timeout=timeout, env=env,
                       cwd=ROOT)
    out = None
    for line in r.stdout.splitlines():
        if line.startswith("{"):
            out = json.loads(line)
    return r, out


def _need_reference():
    if not os.path.exists(os.path.join(ROOT, "oracle", "_ref", "libjerasure_ref.so")):
        import refcheck
        refcheck.reference_missing("oracle/_ref/libjerasure_ref.so")


# ------------------------------------------------------------------ CPU ----
@pytest.mark.parametrize("scenario", SCENARIOS)
def test_fallback_completes_reference_sequences(scenario):
    _need_reference()
    r, out = drive(scenario, fallback=1, inject=1)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    assert out["mismatches"] == [] and out["checked"] > 0, out
    assert out["fallbacks"] >= 1
    # one stderr line per process, however many calls fell back
    assert r.stderr.count("completed on the CPU") == 1, r.stderr[-2000:]


@pytest.mark.parametrize("scenario", ["client", "ecx"])
def test_fallback_off_keeps_the_failure_channel(scenario):
    r, out = drive(scenario, fallback=0, inject=1)
    assert r.returncode == 1 and out is None, (r.stdout[-2000:], r.stderr[-2000:])
    assert "MI355X path failed (-3)" in r.stderr and "ECGPU_CPU_FALLBACK=0" in r.stderr


def test_python_package_fails_loudly_by_default():
    """The package (tests, smoke(), bench) never takes the fallback unless the
    environment asks for it."""
    code = ("import numpy as np\n"
            "from erasure_coding_test_amd import _native as N, jerasure as J, reed_sol as R\n"
            "assert N.get_knob('ECGPU_CPU_FALLBACK') == 0\n"
            "N.set_knob('ECGPU_CPU_FALLBACK', 1); N.reset_knob(None)\n"
            "assert N.get_knob('ECGPU_CPU_FALLBACK') == 0\n"
            "N.set_knob('test_inject_hip', 1)\n"
            "M = R.reed_sol_vandermonde_coding_matrix(4, 2, 8)\n"
            "d = [np.ones(4096, np.uint8) for _ in range(4)]; c = [np.zeros(4096, np.uint8) for _ in range(2)]\n"
            "try:\n"
            "    J.jerasure_matrix_encode(4, 2, 8, M, d, c, 4096)\n"
            "except N.EcgpuError as e:\n"
            "    print('raised', e)\n"
            "print('count', N.fallback_count())\n")
    env = {k: v for k, v in os.environ.items() if k not in ("ECGPU_CPU_FALLBACK", "ECGPU_TEST_INJECT_HIP")}
    env["ECGPU_TEST_INJECT_HIP"] = "1"
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "raised" in r.stdout and "count 0" in r.stdout, r.stdout


# ------------------------------------------------------------------ GPU ----
@pytest.mark.gpu
@pytest.mark.parametrize("scenario", SCENARIOS)
def test_fallback_after_injected_hip_error_gpu(scenario):
    """A transient HIP error before the first launch: every call completes on
    the CPU, bit-exact, and the device is not marked lost."""
    _need_reference()
    r, out = drive(scenario, fallback=1, inject=1)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    assert out["mismatches"] == [] and out["checked"] > 0, out
    assert out["fallbacks"] >= 1 and out["lost"] == 0, out


@pytest.mark.gpu
def test_split_call_ranges_fall_back_independently_gpu():
    """A call cut into concurrent byte ranges (ECGPU_SPLIT): each range's GPU
    attempt fails and that range completes on the CPU on its own thread; the
    call's bytes are the whole call's."""
    _need_reference()
    r, out = drive("client", fallback=1, inject=1, extra_env={"ECGPU_SPLIT": "3", "ECGPU_SPLIT_MIN_KIB": "256"})
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    assert out["mismatches"] == [] and out["fallbacks"] >= 1 and out["lost"] == 0, out


@pytest.mark.gpu
def test_sticky_error_sends_later_calls_to_the_cpu_gpu():
    r, out = drive("client", fallback=1, inject=2)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    assert out["mismatches"] == [] and out["lost"] == 1 and out["fallbacks"] >= 1, out


@pytest.mark.gpu
@pytest.mark.parametrize("scenario", ["client", "ecx"])
def test_fallback_off_exits_gpu(scenario):
    r, out = drive(scenario, fallback=0, inject=1)
    assert r.returncode == 1 and out is None, (r.stdout[-2000:], r.stderr[-2000:])
    assert "injected HIP failure" in r.stderr and "ECGPU_CPU_FALLBACK=0" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("scenario", ["client", "pinned"])
def test_partly_written_call_without_alias_completes_gpu(scenario):
    """A failure after the call started writing caller memory -- a D2H into
    an output, or the kernel writing pinned outputs in place -- is still
    completed on the CPU when no output is also a source: the map reads the
    sources only, and they are untouched."""
    _need_reference()
    r, out = drive(scenario, fallback=1, inject=3)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    assert out["mismatches"] == [] and out["checked"] > 0 and out["fallbacks"] >= 1 and out["lost"] == 0, out


@pytest.mark.gpu
@pytest.mark.parametrize("scenario", ["ecx", "pinned_alias"])
def test_partly_written_aliased_call_keeps_the_error_gpu(scenario):
    """An output that is also a source (the ECX accumulator, galois_region_xor
    r3 == r2; an in-place region multiply) has lost its original bytes once
    the call started writing it: the reference's failure channel, fallback on
    or not."""
    _need_reference()
    r, out = drive(scenario, fallback=1, inject=3)
    assert r.returncode == 1 and out is None, (r.stdout[-2000:], r.stderr[-2000:])
    assert "after caller memory was written" in r.stderr


@pytest.mark.gpu
def test_real_hip_error_hbm_full_completes_on_the_cpu_gpu():
    """A genuine HIP failure, not an injected one: HBM filled by hipMalloc
    until it fails, then the client's C3 4 MiB pageable encode +
    decode{0,1,2,3} through the mangled names -- the library's staging
    hipMalloc fails (csrc/ecgpu_runtime.hip ensure_stage) and the calls
    complete on the CPU, bit-exact against the golden digests; the device is
    not marked lost (out of memory is not sticky).  With the knob at 0 the
    unchanged caller exits 1."""
    r, out = drive("oom", fallback=1, inject=0, timeout=300)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    assert out["hbm_held"] > (100 << 30), out  # the MI355X's HBM, not a token allocation
    assert out["mismatches"] == [] and out["checked"] == 2 and out["fallbacks"] >= 2 and out["lost"] == 0, out
    assert "out of memory" in r.stderr.lower() or "hipMalloc" in r.stderr, r.stderr[-2000:]
    r, out = drive("oom", fallback=0, inject=0, timeout=300)
    assert r.returncode == 1 and out is None, (r.stdout[-2000:], r.stderr[-2000:])
    assert "ECGPU_CPU_FALLBACK=0" in r.stderr


@pytest.mark.gpu
def test_device_buffers_never_fall_back_gpu(gpu, knobs):
    import numpy as np
    import torch

    from erasure_coding_test_amd import _native as N, jerasure as J, reed_sol as R
    k, m, size = 4, 2, 4096
    M = R.reed_sol_vandermonde_coding_matrix(k, m, 8)
    d = [torch.full((size,), i + 1, dtype=torch.uint8, device=gpu) for i in range(k)]
    c = [torch.zeros(size, dtype=torch.uint8, device=gpu) for _ in range(m)]
    knobs.set("ECGPU_CPU_FALLBACK", 1)
    knobs.set("ECGPU_TEST_INJECT_HIP", 1)
    before = N.fallback_count()
    with pytest.raises(N.EcgpuError, match="injected HIP failure"):
        J.jerasure_matrix_encode(k, m, 8, M, d, c, size)
    assert N.fallback_count() == before
    knobs.reset("ECGPU_TEST_INJECT_HIP")
    J.jerasure_matrix_encode(k, m, 8, M, d, c, size)  # row 0 of the Vandermonde matrix is all ones
    assert np.array_equal(c[0].cpu().numpy(), np.full(size, 1 ^ 2 ^ 3 ^ 4, np.uint8))


def fuzz(cases, inject, seed=20261017):
    env = dict(os.environ, ECGPU_CPU_FALLBACK="1", ECGPU_TEST_INJECT_HIP=str(inject))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "fallback_fuzz.py"), str(cases), str(seed)],
                       capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]) if r.stdout.strip() else None
    return r, out


def test_fallback_fuzz_vs_reference():
    """3,000 random synchronous calls (a quarter with repeated buffers) completed
    on the CPU fallback, bytes and return codes equal to the compiled reference."""
    _need_reference()
    r, out = fuzz(3000, inject=2)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    assert out["mismatches"] == [] and out["fallbacks"] >= 2500, out
    assert all(v > 0 for v in out["kinds"].values()), out


@pytest.mark.gpu
def test_fallback_fuzz_vs_reference_gpu():
    """The same on the MI355X, each call's GPU attempt failing before its first
    launch (transient injection): the fallback decision after map_buffers."""
    _need_reference()
    r, out = fuzz(1000, inject=1, seed=77)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    assert out["mismatches"] == [] and out["fallbacks"] >= 800, out
