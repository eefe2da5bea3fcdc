"""The library's CPU executor for small synchronous host-memory calls
(csrc/cpu_exec.hpp, csrc/cpu_fallback.hpp; SURVEY.md §5 "min offload size",
§7 "the fallback for tiny sizes").

A synchronous call whose buffers are all host memory and that moves fewer than
ECGPU_MIN_OFFLOAD_KIB bytes (distinct buffers x size) runs on the calling
thread's CPU -- vgf2p8affineqb on AVX-512 + GFNI hosts, the nibble split on
AVX2, else scalar -- because below the measured crossover the GPU round trip
costs more than the arithmetic.  ECGPU_GPU=0 sends every such
call there.  It is the library's own code: nothing from oracle/ or the
reference, which serve here only as the checkers.

The reference's own call sequences (tests/fallback_driver.py: the client's
encode / decode, the ECX datanode's per-block region ops, the rest of the
header surface) run in subprocesses through the C++-mangled names at every
SIMD level, against the golden fixtures and the reference built in
oracle/_ref; a 1,500-case fuzz per level against the reference.  The
Python package, the bench and the rest of the suite keep the threshold at 0
(tests/conftest.py asserts ecgpu_cpu_call_count() == 0 after every test).
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(ROOT, "tests", "fallback_driver.py")
FUZZ = os.path.join(ROOT, "tests", "fallback_fuzz.py")
LEVELS = [0, 1, 2]  # scalar, AVX2, AVX-512 + GFNI (capped at what the host has)


def _need_reference():
    if not os.path.exists(os.path.join(ROOT, "oracle", "_ref", "libjerasure_ref.so")):
        import refcheck
        refcheck.reference_missing("oracle/_ref/libjerasure_ref.so")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("ECGPU_GPU", "EC_GPU", "ECGPU_MIN_OFFLOAD_KIB", "ECGPU_CPU_SIMD", "ECGPU_TEST_INJECT_HIP",
                        "ECGPU_LINK_CALLS")}
    env["ECGPU_CPU_FALLBACK"] = "0"  # nothing may reach the CPU through the fallback here
    env.update({k: str(v) for k, v in kw.items()})
    return env


def drive(scenario, timeout=600, **kw):
    r = subprocess.run([sys.executable, DRIVER, scenario], capture_output=True, text=True, timeout=timeout,
                       env=_env(**kw), cwd=ROOT)
    out = None
    for line in r.stdout.splitlines():
        if line.startswith("{"):
            out = json.loads(line)
    return r, out


def run_py(code, timeout=300, **kw):
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=timeout,
                          env=_env(**kw), cwd=ROOT)


# ------------------------------------------------------------------ CPU ----
@pytest.mark.parametrize("level", LEVELS)
@pytest.mark.parametrize("scenario", ["client", "ecx", "surface"])
def test_cpu_executor_reference_sequences(scenario, level):
    """ECGPU_GPU=0: every call of the reference's sequences on the CPU executor
    by choice, bit-exact, none through the fallback (here any GPU attempt would
    fail -- no device, fallback off -- and the drop-in would exit 1)."""
    _need_reference()
    r, out = drive(scenario, ECGPU_GPU=0, ECGPU_CPU_SIMD=level)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    assert out["mismatches"] == [] and out["checked"] > 0, out
    assert out["fallbacks"] == 0 and out["cpu_calls"] > 0, out


@pytest.mark.parametrize("level", LEVELS)
def test_cpu_executor_fuzz_vs_reference(level):
    """1,500 random synchronous calls (encode k 1..20 x m 1..8, decodes of up to
    m + 1 erasures with return codes, dot products, region ops, a quarter with
    repeated buffers) on the CPU executor, equal to the compiled reference."""
    _need_reference()
    r = subprocess.run([sys.executable, FUZZ, "1500", str(4000 + level)], capture_output=True, text=True, timeout=600,
                       env=_env(ECGPU_GPU=0, ECGPU_CPU_SIMD=level), cwd=ROOT)
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    assert out["mismatches"] == [] and out["fallbacks"] == 0 and out["cpu_calls"] >= 1350, out  # decodes that return -1 never execute


def test_min_offload_threshold_boundary():
    """A call moving fewer than the threshold's bytes runs on the CPU; one
    moving exactly that many goes to the GPU (here: no device, fallback off, so
    it fails -- which shows it was not run on the CPU)."""
    code = ("import numpy as np\n"
            "from erasure_coding_test_amd import _native as N, galois as G\n"
            "N.set_knob('ECGPU_MIN_OFFLOAD_KIB', 1)\n"  # 1024 bytes
            "a = np.arange(512, dtype=np.uint8); b = a[::-1].copy(); c = np.zeros(512, np.uint8)\n"
            "G.galois_region_xor(a, b, c, 511)\n"  # r1, r2, r3 distinct: 3 x 511 = 1533 >= 1024 -> GPU
            "print('unexpected')\n")
    r = run_py(code)
    assert "unexpected" not in r.stdout and r.returncode != 0, (r.stdout, r.stderr[-2000:])
    code = ("import numpy as np\n"
            "from erasure_coding_test_amd import _native as N, galois as G\n"
            "N.set_knob('ECGPU_MIN_OFFLOAD_KIB', 1)\n"
            "a = np.arange(512, dtype=np.uint8); b = a[::-1].copy(); c = np.zeros(512, np.uint8)\n"
            "G.galois_region_xor(a, b, c, 341)\n"  # 3 x 341 = 1023 < 1024 -> CPU
            "assert np.array_equal(c[:341], a[:341] ^ b[:341]) and not c[341:].any()\n"
            "G.galois_region_xor(a, b, b, 511)\n"  # r3 == r2: 2 distinct x 511 = 1022 -> CPU
            "assert np.array_equal(b[:511], (a ^ a[::-1])[:511]) and b[511] == 0\n"
            "print('cpu_calls', N.cpu_call_count(), 'fallbacks', N.fallback_count())\n")
    r = run_py(code)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "cpu_calls 2 fallbacks 0" in r.stdout, r.stdout


def test_ecx_block_sequence_below_default_threshold():
    """The unchanged ECX datanode's per-block calls (349,525-B blocks, 2
    distinct buffers each) fall under the library's default threshold: with
    the GPU untouched and the fallback off they complete, bit-exact."""
    _need_reference()
    code = ("from erasure_coding_test_amd import _native as N\n"
            "N.lib.ecgpu_reset_knob(b'ECGPU_MIN_OFFLOAD_KIB')\n"
            "print(N.lib.ecgpu_min_offload_bytes())\n")
    r = run_py(code)
    default_bytes = int(r.stdout.split()[-1])
    assert default_bytes > 0, "the library's default threshold must be a measured crossover, not 0"
    r, out = drive("ecx")
    if 2 * 349525 < default_bytes:
        assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
        assert out["mismatches"] == [] and out["fallbacks"] == 0 and out["cpu_calls"] > 0, out


def test_default_threshold_follows_the_executor_simd_level():
    """ECGPU_MIN_OFFLOAD_KIB unset (-1): the measured crossover for the
    executor's SIMD level (GFNI 16 MiB, AVX2 4 MiB, scalar 256 KiB, DESIGN.md
    §8); a set value wins; the Python package's 0 sends everything to the GPU."""
    code = ("import ctypes, os\n"
            "from erasure_coding_test_amd import _native as N\n"
            "N.lib.ecgpu_reset_knob(b'ECGPU_MIN_OFFLOAD_KIB')\n"
            "lvl = ctypes.c_int(); N.lib.ecgpu_get_knob(b'ECGPU_CPU_SIMD', ctypes.byref(lvl))\n"
            "print('auto', N.lib.ecgpu_min_offload_bytes())\n"
            "N.set_knob('ECGPU_MIN_OFFLOAD_KIB', 100); print('set', N.lib.ecgpu_min_offload_bytes())\n"
            "N.reset_knob('ECGPU_MIN_OFFLOAD_KIB'); print('package', N.lib.ecgpu_min_offload_bytes())\n")
    want = {"0": 256 << 10, "1": 4 << 20}
    for level in ("0", "1"):
        r = run_py(code, ECGPU_CPU_SIMD=level)
        assert r.returncode == 0, r.stderr[-2000:]
        got = dict(line.split() for line in r.stdout.splitlines() if line.split()[0] in ("auto", "set", "package"))
        assert int(got["auto"]) == want[level] and int(got["set"]) == 100 << 10 and int(got["package"]) == 0, got
    r = run_py(code)  # the host's best level: GFNI hosts 16 MiB
    got = dict(line.split() for line in r.stdout.splitlines() if line.split()[0] in ("auto", "set", "package"))
    assert int(got["auto"]) in (256 << 10, 4 << 20, 16 << 20), got


def test_ec_gpu_alias_of_the_gpu_switch():
    """SURVEY §5 names the switch EC_GPU=0/1: it sets ECGPU_GPU when that is
    unset; ECGPU_GPU wins when both are set."""
    code = ("from erasure_coding_test_amd import _native as N\n"
            "print('gpu', N.get_knob('ECGPU_GPU'))\n")
    for env, want in (({"EC_GPU": "0"}, 0), ({"EC_GPU": "1"}, 1), ({"EC_GPU": "0", "ECGPU_GPU": "1"}, 1), ({}, 1)):
        r = run_py(code, **env)
        assert r.returncode == 0 and f"gpu {want}" in r.stdout, (env, r.stdout, r.stderr[-2000:])


def test_gpu_switch_does_not_touch_device_memory_logic():
    """ECGPU_GPU=0 is a routing switch for host memory only: the package's
    knob defaults keep it on, and a reset restores them."""
    code = ("from erasure_coding_test_amd import _native as N\n"
            "assert N.get_knob('ECGPU_GPU') == 1 and N.get_knob('ECGPU_MIN_OFFLOAD_KIB') == 0\n"
            "N.set_knob('ECGPU_MIN_OFFLOAD_KIB', 64); N.reset_knob('min_offload_kib')\n"
            "assert N.get_knob('ECGPU_MIN_OFFLOAD_KIB') == 0\n"
            "print('ok')\n")
    r = run_py(code)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]


def test_injection_knob_is_not_read_from_the_environment():
    """a stray ECGPU_TEST_INJECT_HIP in a deployed datanode's
    environment must not fail calls -- the hook is settable only in-process."""
    code = ("from erasure_coding_test_amd import _native as N\n"
            "print('inject', N.get_knob('test_inject_hip'))\n")
    r = run_py(code, ECGPU_TEST_INJECT_HIP=2)
    assert r.returncode == 0 and "inject 0" in r.stdout, (r.stdout, r.stderr[-2000:])


def test_bad_device_ordinal_does_not_mark_a_device_lost():
    """ecgpu_device_pci_bus_id(999) fails (invalid or no device) but
    leaves device 0 usable (a fresh process: in this one, earlier no-device
    calls may have marked it lost on purpose)."""
    code = ("import ctypes\n"
            "from erasure_coding_test_amd import _native as N\n"
            "buf = ctypes.create_string_buffer(64)\n"
            "assert N.lib.ecgpu_device_pci_bus_id(999, buf, 64) == N.ECGPU_ERR_HIP\n"
            "print('lost', N.lib.ecgpu_device_lost(0))\n")
    r = run_py(code)
    assert r.returncode == 0 and "lost 0" in r.stdout, (r.stdout, r.stderr[-2000:])


# ------------------------------------------------------------------ GPU ----
@pytest.mark.gpu
def test_default_threshold_client_sequence_gpu():
    """The library's defaults on the MI355X: the client's small calls (C1-C3
    golden stripes at 1-4 KiB, the golden inconsistent decodes) run on the CPU
    executor, its C3 4 MiB stripe on the GPU; every byte as the reference's."""
    _need_reference()
    r, out = drive("client")
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    assert out["mismatches"] == [] and out["fallbacks"] == 0, out
    assert 0 < out["cpu_calls"] < out["checked"], out  # some, not all (C3 4 MiB stays on the GPU)


@pytest.mark.gpu
@pytest.mark.parametrize("scenario", ["client", "ecx", "surface"])
def test_gpu_switch_off_gpu(scenario):
    _need_reference()
    r, out = drive(scenario, ECGPU_GPU=0)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    assert out["mismatches"] == [] and out["fallbacks"] == 0 and out["cpu_calls"] > 0, out


@pytest.mark.gpu
def test_device_buffers_ignore_the_cpu_routing_gpu(gpu, knobs):
    """Device memory never runs on the CPU executor, whatever the knobs say."""
    import numpy as np
    import torch

    from erasure_coding_test_amd import _native as N, jerasure as J, reed_sol as R
    k, m, size = 4, 2, 4096
    M = R.reed_sol_vandermonde_coding_matrix(k, m, 8)
    d = [torch.full((size,), i + 1, dtype=torch.uint8, device=gpu) for i in range(k)]
    c = [torch.zeros(size, dtype=torch.uint8, device=gpu) for _ in range(m)]
    knobs.set("ECGPU_GPU", 0)
    knobs.set("ECGPU_MIN_OFFLOAD_KIB", 1 << 20)
    J.jerasure_matrix_encode(k, m, 8, M, d, c, size)
    assert N.cpu_call_count() == 0
    assert np.array_equal(c[0].cpu().numpy(), np.full(size, 1 ^ 2 ^ 3 ^ 4, np.uint8))


@pytest.mark.gpu
def test_bad_device_ordinal_does_not_mark_a_device_lost_gpu(gpu):
    import ctypes

    from erasure_coding_test_amd import _native as N
    buf = ctypes.create_string_buffer(64)
    assert N.lib.ecgpu_device_pci_bus_id(99, buf, 64) == N.ECGPU_ERR_HIP
    assert N.lib.ecgpu_device_lost(0) == 0
    assert N.lib.ecgpu_device_pci_bus_id(0, buf, 64) == 0


@pytest.mark.gpu
def test_handled_hip_error_does_not_leak_into_the_callers_hip_state_gpu(gpu):
    """A HIP error the library handled (a bad ordinal here; an OOM completed on
    the CPU in deployment) is cleared from HIP's per-thread last error, which
    the caller's own HIP code in the same process shares: torch's next launch
    check used to raise the library's stale 'invalid device ordinal'."""
    import ctypes

    import torch

    from erasure_coding_test_amd import _native as N
    buf = ctypes.create_string_buffer(64)
    assert N.lib.ecgpu_device_pci_bus_id(99, buf, 64) == N.ECGPU_ERR_HIP
    hip = ctypes.CDLL("libamdhip64.so.7")
    assert hip.hipPeekAtLastError() == 0
    t = torch.full((4096,), 7, dtype=torch.uint8, device=gpu)
    torch.cuda.synchronize()
    assert int(t.sum()) == 7 * 4096


def test_decode_matrix_cache_keys_on_the_whole_coding_matrix():
    """The decoding-matrix cache (planner.cpp) must never serve one matrix's
    inversion for another with the same erasure pattern: the same patterns
    decoded under two coding matrices (the Vandermonde one and a copy with
    its rows scaled), alternately, each on inconsistent inputs so the
    survivor choice shows, against the compiled reference."""
    _need_reference()
    code = r'''
import sys, os, ctypes, numpy as np
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
from fallback_driver import LIB, REF, bind, ints, ptrs, matrix
d = bind(os.path.join(LIB, "libjerasure_amd.so")); ref = bind(os.path.join(REF, "libjerasure_ref.so"))
k, m, size = 6, 3, 4096
A = matrix(d, k, m)
B = [x if i < k else (x * 3) % 256 or 1 for i, x in enumerate(A)]  # rows 1.. differ
rng = np.random.default_rng(9)
# the two matrices decode the same inputs differently (else the test proves nothing)
probe = [rng.integers(0, 256, size + 16, dtype=np.uint8) for _ in range(k + m)]
pa, pb = [b.copy() for b in probe], [b.copy() for b in probe]
ref["decode"](k, m, 8, ints(A), 0, ints([0, 1, 2, -1]), ptrs(pa[:k]), ptrs(pa[k:]), size)
ref["decode"](k, m, 8, ints(B), 0, ints([0, 1, 2, -1]), ptrs(pb[:k]), ptrs(pb[k:]), size)
assert any(not np.array_equal(a, b) for a, b in zip(pa, pb))
bad = 0
for it in range(40):
    M = A if it % 2 == 0 else B
    er = [[0, 1, 2], [1, 4, 7], [0, 6], [2, 5, 8]][(it // 2) % 4] + [-1]
    bufs = [rng.integers(0, 256, size + 16, dtype=np.uint8) for _ in range(k + m)]  # inconsistent on purpose
    mine = [b.copy() for b in bufs]
    theirs = [b.copy() for b in bufs]
    r1 = d["decode"](k, m, 8, ints(M), 0, ints(er), ptrs(mine[:k]), ptrs(mine[k:]), size)
    r2 = ref["decode"](k, m, 8, ints(M), 0, ints(er), ptrs(theirs[:k]), ptrs(theirs[k:]), size)
    bad += (r1 != r2) or any(not np.array_equal(a[:size], b[:size]) for a, b in zip(mine, theirs))
print("bad", bad)
'''
    r = run_py(code, ECGPU_GPU=0)
    assert r.returncode == 0 and "bad 0" in r.stdout, (r.stdout[-2000:], r.stderr[-2000:])


@pytest.mark.gpu
def test_link_busy_calls_run_on_the_cpu_bit_exact_gpu():
    """ECGPU_LINK_CALLS (the C library's default 1): a large host-memory call
    arriving while another holds the device's link runs on the CPU executor.
    Four threads encode their own pageable RS(10,4) 4 MiB stripes through the
    mangled names at once (the small-call threshold at 0, so only the link
    rule routes); some calls take the CPU, and every parity equals the same
    stripe's parity computed with every call on the GPU."""
    code = r'''
import os, sys, ctypes, threading, numpy as np
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
from fallback_driver import LIB, bind, ints, ptrs, matrix
d = bind(os.path.join(LIB, "libjerasure_amd.so"))
core = ctypes.CDLL(os.path.join(LIB, "libecgpu.so"))
core.ecgpu_set_knob.argtypes = [ctypes.c_char_p, ctypes.c_int]
core.ecgpu_cpu_call_count.restype = ctypes.c_int64
k, m, S = 10, 4, 4 << 20
M = matrix(d, k, m)
core.ecgpu_set_knob(b"ECGPU_MIN_OFFLOAD_KIB", 0)
rng = np.random.default_rng(5)
stripes = [[rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)] for _ in range(4)]
core.ecgpu_set_knob(b"ECGPU_LINK_CALLS", 0)  # reference parities: every call on the GPU
want = []
for st in stripes:
    c = [np.zeros(S, np.uint8) for _ in range(m)]
    d["encode"](k, m, 8, ints(M), ptrs(st), ptrs(c), S)
    want.append(c)
before = core.ecgpu_cpu_call_count()
core.ecgpu_set_knob(b"ECGPU_LINK_CALLS", 1)
bad = []
def worker(i):
    for rep in range(6):
        c = [np.full(S, 0x5A, np.uint8) for _ in range(m)]
        d["encode"](k, m, 8, ints(M), ptrs(stripes[i]), ptrs(c), S)
        if any(not np.array_equal(a, b) for a, b in zip(c, want[i])):
            bad.append((i, rep))
ts = [threading.Thread(target=worker, args=(i,)) for i in range(4)]
[t.start() for t in ts]
[t.join() for t in ts]
print("bad", len(bad), "cpu_calls", core.ecgpu_cpu_call_count() - before)
'''
    r = run_py(code)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    words = r.stdout.split()
    assert words[words.index("bad") + 1] == "0", r.stdout
    assert 0 < int(words[words.index("cpu_calls") + 1]) < 24, r.stdout
