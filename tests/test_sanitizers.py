"""Sanitizers on the host code (the reference races on its lazy
tables and stats; the replacement must not).

tests/sanitize/host_harness.cpp drives the host-only part of libecgpu --
field tables, matrix construction and inversion, the fused decode planner
over every RS(10,4) pattern of up to 5 erasures, bit-matrix / schedule
construction, the CPU executor at every SIMD level the host has (against
the reference's sequential semantics, aliasing and > 4 output rows included)
and its bookkeeping -- built from
csrc/ with g++:

* AddressSanitizer + UndefinedBehaviorSanitizer (+ LeakSanitizer), one thread;
* ThreadSanitizer, 8 threads making their first calls concurrently.

tests/sanitize/pipeline_harness.cpp drives the threaded runtime's host-side
synchronisation (csrc/host_sync.hpp: the host pipeline's ticket / slot / D2H
worker state machine, the pipeline groups' member queues, the context pool,
the per-device upload streams) on a fake device whose streams are threads and
whose events complete after random delays, under ThreadSanitizer.  Each
stripe is checked right after the wait() that covers it.  The same harness
built with the round-2 logic restored (ECGPU_MUTANT_R2_*) must FAIL: a race
report or wrong bytes for the D2H routing, a hang for the group wake-up.

The sanitizer runtimes are linked statically so the process does not depend
on library load order.  GPU code is not built here (no device sanitizers on
this pool); CPU-only, a couple of minutes.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "erasure_coding_test_amd", "csrc")
HOST_SRCS = ["gf_host.cpp", "matrix_host.cpp", "planner.cpp", "schedule_host.cpp", "capi_host.cpp", "contract_host.cpp",
             "knobs.cpp", "cpu_fallback.cpp", "cpu_exec.cpp"]
HARNESS = os.path.join(ROOT, "tests", "sanitize", "host_harness.cpp")
PIPE_HARNESS = os.path.join(ROOT, "tests", "sanitize", "pipeline_harness.cpp")
TSAN_ENV = {"TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1"}

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")


def _build(tmp_path, name, flags):
    exe = str(tmp_path / name)
    cmd = (["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-pthread",
            f"-I{os.path.join(ROOT, 'include')}", f"-I{CSRC}"] + flags +
           [os.path.join(CSRC, s) for s in HOST_SRCS] + [HARNESS, "-o", exe])
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0 and "cannot find" in r.stderr and "-static-lib" in " ".join(flags):
        pytest.skip("static sanitizer runtime not installed")
    assert r.returncode == 0, r.stderr[-4000:]
    return exe


def _run(exe, args, env_extra):
    env = dict(os.environ, **env_extra)
    r = subprocess.run([exe] + args, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-6000:])
    assert "ERROR: AddressSanitizer" not in r.stderr
    assert "runtime error:" not in r.stderr  # UBSan
    assert "WARNING: ThreadSanitizer" not in r.stderr
    return r.stdout


def test_host_code_asan_ubsan(tmp_path):
    exe = _build(tmp_path, "harness_asan",
                 ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-static-libasan", "-static-libubsan"])
    out = _run(exe, [], {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
                         "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1"})
    assert "host harness ok" in out


def test_host_code_tsan_concurrent_first_use(tmp_path):
    exe = _build(tmp_path, "harness_tsan", ["-fsanitize=thread", "-static-libtsan"])
    out = _run(exe, ["8"], {"TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1"})
    assert "8 thread(s)" in out


def _build_pipe(tmp_path, name, flags):
    exe = str(tmp_path / name)
    cmd = (["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-pthread", "-Wall", "-Wextra", "-Werror",
            f"-I{os.path.join(ROOT, 'include')}", f"-I{CSRC}"] + flags + [PIPE_HARNESS, "-o", exe])
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0 and "cannot find" in r.stderr and "-static-lib" in " ".join(flags):
        pytest.skip("static sanitizer runtime not installed")
    assert r.returncode == 0, r.stderr[-4000:]
    return exe


TSAN = ["-fsanitize=thread", "-static-libtsan"]


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_pipeline_state_machine_tsan(tmp_path, seed):
    exe = _build_pipe(tmp_path, "pipe_tsan", TSAN)
    out = _run(exe, ["pipe", "150", str(seed)], TSAN_ENV)
    assert "pipeline harness ok: 150 runs" in out
    # both D2H routes were exercised: inline on the submitting thread and by the worker
    inline, worker = [int(w) for w in out.split() if w.isdigit()][1:3]
    assert inline > 0 and worker > 0, out


def test_group_member_queue_and_pools_tsan(tmp_path):
    exe = _build_pipe(tmp_path, "group_tsan", TSAN)
    assert "group harness ok" in _run(exe, ["group", "60", "5"], TSAN_ENV)
    assert "pool harness ok" in _run(exe, ["pool", "8"], TSAN_ENV)


def test_harness_detects_round2_d2h_routing(tmp_path):
    """Round 2 issued a pinned stripe's D2H inline whenever the worker queue
    was empty, even while the worker still held a popped job: the retire of
    the earlier slot then synced a stale event and wait() returned early.
    With that logic restored the harness must fail (TSan race report: exit
    66, or wrong bytes right after wait(): exit 2)."""
    exe = _build_pipe(tmp_path, "pipe_mutant", TSAN + ["-DECGPU_MUTANT_R2_D2H"])
    r = subprocess.run([exe, "pipe", "150", "1", "60"], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, **TSAN_ENV))
    assert r.returncode in (2, 66), (r.returncode, r.stdout[-1000:], r.stderr[-3000:])
    assert "WARNING: ThreadSanitizer: data race" in r.stderr or "stripe output wrong" in r.stderr


def test_harness_detects_round2_group_lost_wakeup(tmp_path):
    """Round 2 signalled a put() blocked on back-pressure only before the
    worker advanced next_local, never after: the put of exactly the next
    ticket could sleep forever.  With that logic restored the
    constructed case must hang (watchdog exit 3)."""
    exe = _build_pipe(tmp_path, "group_mutant", ["-DECGPU_MUTANT_R2_WAKEUP"])
    r = subprocess.run([exe, "group", "5", "1", "5"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 3 and "HANG" in r.stderr, (r.returncode, r.stderr[-2000:])
