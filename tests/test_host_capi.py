"""Host half of the C ABI (include/ecgpu.h) against the reference's golden
vectors -- no GPU is touched.

The fused decode map (ecgpu_decode_plan) is replayed here with numpy GF(2^8)
arithmetic (products from the reference's own multiplication table) on the
golden inconsistent-input decode cases: matching the reference's digests pins
the planner's survivor choice, row_k_ones path and aliasing semantics without
a GPU.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from ecdata import CONFIGS, fnv1a64, shard_seed, splitmix_bytes

E = pytest.importorskip("erasure_coding_test_amd")
from erasure_coding_test_amd import galois, jerasure, reed_sol  # noqa: E402


def gf_combine(mul, coefs, srcs):
    out = np.zeros_like(srcs[0])
    for c, s in zip(coefs, srcs):
        if c:
            out ^= mul[c][s]
    return out


def test_scalar_field_matches_reference(golden, vectors):
    mul = vectors["gf_mul_table"]
    got = np.array([[galois.galois_single_multiply(a, b, 8) for b in range(256)] for a in range(256)], np.uint8)
    assert np.array_equal(got, mul)
    s = golden["scalar"]
    assert [galois.galois_inverse(a, 8) for a in range(256)] == s["inverse"]
    assert [galois.galois_log(v, 8) for v in range(256)] == s["log"]
    assert all(galois.galois_ilog(int(v), 8) == x for v, x in s["ilog"].items())
    assert [galois.galois_single_divide(a, 0, 8) for a in range(0, 256, 51)] == s["div_by_zero"]
    for a in range(1, 256):
        for b in (1, 2, 29, 142, 255):
            q = galois.galois_single_divide(a, b, 8)
            assert galois.galois_single_multiply(q, b, 8) == a


def test_python_mirror_covers_every_header_function():
    """The Python mirror has every function the reference headers declare
    (include/dropin/*.h carry the reference's declarations verbatim in
    signature), under the same name."""
    import importlib
    import re
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    total = 0
    for hdr in ("galois", "jerasure", "reed_sol"):
        with open(os.path.join(root, "include", "dropin", hdr + ".h")) as f:
            text = re.sub(r"/\*.*?\*/", "", f.read(), flags=re.S)
        names = set(re.findall(r"\b((?:galois|jerasure|reed_sol)_\w+)\s*\(", text))
        mod = importlib.import_module("erasure_coding_test_amd." + hdr)
        assert not [n for n in sorted(names) if not callable(getattr(mod, n, None))], hdr
        total += len(names)
    assert total == 60  # galois.h 24, jerasure.h 28, reed_sol.h 8


def test_log_tables_out_of_range():
    """The reference indexes its log tables unchecked and exits for w > 30
    (galois.cpp:269-289): the C ABI returns -1 there, the mirror raises."""
    from erasure_coding_test_amd import _native as N
    for w in (4, 8, 16):
        nwm1 = (1 << w) - 1
        assert N.lib.ecgpu_galois_log(nwm1, w) == galois.galois_log(nwm1, w) >= 0
        assert N.lib.ecgpu_galois_ilog(-nwm1, w) == galois.galois_ilog(-nwm1, w) == 1
        assert N.lib.ecgpu_galois_ilog(2 * nwm1 - 1, w) == galois.galois_ilog(2 * nwm1 - 1, w) >= 1
        for bad in (-1, nwm1 + 1, 1 << 30):
            assert N.lib.ecgpu_galois_log(bad, w) == -1
            with pytest.raises(ValueError):
                galois.galois_log(bad, w)
        for bad in (-nwm1 - 1, 2 * nwm1):
            assert N.lib.ecgpu_galois_ilog(bad, w) == -1
            with pytest.raises(ValueError):
                galois.galois_ilog(bad, w)
    assert N.lib.ecgpu_galois_log(1, 32) == -1
    with pytest.raises(ValueError):
        galois.galois_log(1, 31)


@pytest.mark.parametrize("w", [4, 8, 16, 32])
def test_field_axioms_other_widths(w):
    import random
    rnd = random.Random(w)
    hi = (1 << w) - 1 if w < 32 else 0x7FFFFFFF
    for _ in range(200):
        a, b, c = rnd.randint(1, hi), rnd.randint(1, hi), rnd.randint(1, hi)
        m = galois.galois_single_multiply
        assert m(a, b, w) == m(b, a, w)
        assert m(m(a, b, w), c, w) == m(a, m(b, c, w), w)
        assert m(a, b ^ c, w) == m(a, b, w) ^ m(a, c, w)
        inv = galois.galois_inverse(a, w)
        assert m(a, inv, w) & ((1 << w) - 1 if w < 32 else 0xFFFFFFFF) == 1


def test_vandermonde_and_r6_matrices(golden):
    for key, mat in golden["vandermonde"].items():
        k, m = map(int, key.split(","))
        got = reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
        if mat is None:
            assert got is None
        else:
            assert got == [x for row in mat for x in row], key
    for key, mat in golden["r6"].items():
        assert reed_sol.reed_sol_r6_coding_matrix(int(key), 8) == [x for row in mat for x in row]
    assert reed_sol.reed_sol_r6_coding_matrix(4, 7) is None
    assert reed_sol.reed_sol_vandermonde_coding_matrix(4, 4, 2) is None  # 2^w < rows


def test_decoding_matrices(golden):
    mats = {}
    for key, exp in golden["decoding_matrices"].items():
        km, ers = key.split(":")
        k, m = map(int, km.split(","))
        mats.setdefault(km, reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8))
        er = set(map(int, ers.split(",")))
        rc, dm, ids = jerasure.jerasure_make_decoding_matrix(k, m, 8, mats[km], [int(i in er) for i in range(k + m)])
        assert rc == exp["rc"] and ids == exp["dm_ids"], key
        assert dm == [x for row in exp["dm"] for x in row], key


def test_invert_matrix_final_state_matches_reference(reference):
    import random
    rnd = random.Random(3)
    for _ in range(50):
        n = rnd.randint(1, 8)
        mat = np.array([[rnd.choice([0, 0, 1, rnd.randrange(256)]) for _ in range(n)] for _ in range(n)])
        rc_ref, inv_ref = reference.invert_matrix(mat.copy())
        rc, inv, after = jerasure.jerasure_invert_matrix(mat.ravel().tolist(), n, 8)
        assert rc == rc_ref
        if rc == 0:
            assert inv == inv_ref.ravel().tolist()
            assert after == np.eye(n, dtype=int).ravel().tolist()  # the reference leaves I behind
        assert jerasure.jerasure_invertible_matrix(mat.ravel().tolist(), n, 8) == (1 if rc == 0 else 0)


def test_erasures_to_erased_and_multiply():
    assert jerasure.jerasure_erasures_to_erased(4, 2, [1, 4]) == [0, 1, 0, 0, 1, 0]
    assert jerasure.jerasure_erasures_to_erased(4, 2, [1, 1, 4]) == [0, 1, 0, 0, 1, 0]  # duplicates count once
    assert jerasure.jerasure_erasures_to_erased(4, 2, [0, 1, 2]) is None
    a = reed_sol.reed_sol_vandermonde_coding_matrix(4, 2, 8)
    ident = [1 if i == j else 0 for i in range(4) for j in range(4)]
    assert jerasure.jerasure_matrix_multiply(a, ident, 2, 4, 4, 4, 8) == a


@pytest.mark.parametrize("cfg", sorted(CONFIGS))
def test_encode_map_reproduces_golden(golden, vectors, cfg):
    mul = vectors["gf_mul_table"]
    k, m = CONFIGS[cfg]["k"], CONFIGS[cfg]["m"]
    M = np.array(reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)).reshape(m, k)
    for stripe in range(2):
        data = [splitmix_bytes(4096, shard_seed(cfg, stripe, s)) for s in range(k)]
        coding = np.stack([gf_combine(mul, M[i], data) for i in range(m)])
        assert np.array_equal(coding, vectors[f"enc_{cfg}_{stripe}"])


def test_decode_plan_replays_reference_decode(golden, vectors):
    mul = vectors["gf_mul_table"]
    mats = {}
    for case in golden["decode_inconsistent"]:
        k, m, cfg, size = case["k"], case["m"], case["cfg"], case["size"]
        mats.setdefault((k, m), reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8))
        plan = jerasure.decode_plan(k, m, mats[(k, m)], case["erasures"], case["row_k_ones"])
        if case["rc"] == -1:
            assert plan is None, case["erasures"]
            continue
        out_ids, src_ids, coefs = plan
        shards = [splitmix_bytes(size, shard_seed(cfg, 7, s)) for s in range(k + m)]
        result = list(shards)
        for oid, row in zip(out_ids, coefs):
            result[oid] = gf_combine(mul, row, [shards[i] for i in src_ids])
        assert [fnv1a64(x) for x in result] == case["digests"], (case["erasures"], case["row_k_ones"])


def test_recommended_stride():
    from erasure_coding_test_amd import _native as N
    # per-size skew table (shard_stride.hpp kSkewTable, profiles/r03_skew_sweep_*.jsonl), +10 KiB elsewhere
    st = N.lib.ecgpu_recommended_shard_stride
    assert st(4 << 20) == (4 << 20) + (6 << 10)
    assert st((4 << 20) + 3) == (4 << 20) + 256 + (6 << 10)
    assert st(16 << 20) == (16 << 20) + (8 << 10)
    assert st(1 << 20) == 1 << 20
    assert st(5 << 20) == (5 << 20) + (10 << 10)
    assert st(349525) == ((349525 + 255) & ~255) + (10 << 10)  # ECX block size
    # round 5: no skew up to 256 KiB (+1/16) and at 512 KiB, profiles/r05_skew_small.jsonl, r05_skew_mid.jsonl
    for small in (1, 4096, 16 << 10, 64 << 10, 100000, 256 << 10, 272 << 10, 480 << 10, 512 << 10, 544 << 10):
        assert st(small) == (small + 255) & ~255, small
    assert st((272 << 10) + 1) == (272 << 10) + 256 + (10 << 10)
    assert st((544 << 10) + 1) == (544 << 10) + 256 + (10 << 10)


def test_recommended_stride_per_scheme():
    """ecgpu_recommended_shard_stride_km: RS(10,4) (k + m = 14) keeps the
    round-3 skews at 256 / 512 KiB; other schemes and sizes take the
    size-only advice."""
    from erasure_coding_test_amd import _native as N
    km, st = N.lib.ecgpu_recommended_shard_stride_km, N.lib.ecgpu_recommended_shard_stride
    assert km(256 << 10, 10, 4) == (256 << 10) + (12 << 10)
    assert km(512 << 10, 10, 4) == (512 << 10) + (8 << 10)
    assert km(500 << 10, 12, 2) == (500 << 10) + (8 << 10)  # any k + m = 14, within 1/16
    for k, m in ((4, 2), (6, 3), (12, 4)):
        assert km(256 << 10, k, m) == 256 << 10 and km(512 << 10, k, m) == 512 << 10
    for size in (64 << 10, 1 << 20, 4 << 20, (4 << 20) + 3, 16 << 20, 349525):
        for k, m in ((10, 4), (4, 2), (6, 3), (12, 4)):
            assert km(size, k, m) == st(size), (size, k, m)
    assert km(256 << 10, 0, 4) == st(256 << 10)  # k <= 0: the size-only advice
    for size in (1, 7, 4095, 65536, (1 << 20) - 1, (3 << 20) + 17, 100 << 20):
        assert st(size) % 256 == 0 and st(size) >= size


def test_stride_skew_override(knobs):
    """The shard_skew_kib knob (ECGPU_SHARD_SKEW_KIB) replaces the per-size
    table; values outside 0..1024 are ignored."""
    from erasure_coding_test_amd import _native as N
    st = N.lib.ecgpu_recommended_shard_stride
    knobs.set("ECGPU_SHARD_SKEW_KIB", 12)
    assert st(4 << 20) == (4 << 20) + (12 << 10) and st(1 << 20) == (1 << 20) + (12 << 10)
    knobs.set("shard_skew_kib", 0)
    assert st(16 << 20) == 16 << 20
    assert N.lib.ecgpu_recommended_shard_stride_km(512 << 10, 10, 4) == 512 << 10  # the knob wins for schemes too
    for bad in (-4, 2000):
        knobs.set("ECGPU_SHARD_SKEW_KIB", bad)
        assert st(4 << 20) == (4 << 20) + (6 << 10), bad
    knobs.reset("ECGPU_SHARD_SKEW_KIB")
    assert st(4 << 20) == (4 << 20) + (6 << 10)


KNOB_ENV = """
import os, sys
sys.path.insert(0, {root!r})
from erasure_coding_test_amd import _native as N
print(N.get_knob("ECGPU_SHARD_SKEW_KIB"), N.lib.ecgpu_recommended_shard_stride(4 << 20) - (4 << 20))
"""


@pytest.mark.parametrize("env,want", [("12", "12 12288"), ("", "-1 6144"), ("x", "-1 6144"), ("12k", "-1 6144"),
                                      ("-4", "-4 6144"), ("2000", "2000 6144")])
def test_knob_environment_is_read_once_and_strictly(env, want):
    """The environment is read once, at first use, as a whole decimal integer:
    a malformed value keeps the default."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    e = dict(os.environ, ECGPU_SHARD_SKEW_KIB=env)
    r = subprocess.run([sys.executable, "-c", KNOB_ENV.format(root=root)], capture_output=True, text=True, env=e,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.split("\n")[-2] == want


def test_knobs_set_get_reset():
    from erasure_coding_test_amd import _native as N
    assert N.get_knob("cap") == N.get_knob("ECGPU_CAP")
    N.set_knob("ECGPU_CAP", 0)
    assert N.get_knob("cap") == 0
    N.reset_knob("cap")
    assert N.get_knob("ECGPU_CAP") == -1
    with pytest.raises(N.EcgpuError, match="unknown knob"):
        N.set_knob("ECGPU_NOPE", 1)
    assert N.lib.ecgpu_set_knob(b"cap", -(2**31)) == N.ECGPU_ERR_ARG  # the reserved "unset" value


NO_GPU = not os.path.exists("/dev/kfd")


@pytest.mark.skipif(not NO_GPU, reason="checks the no-GPU failure mode")
def test_hot_path_without_gpu_fails_loudly():
    """No silent success with the CPU fallback off (the package's and the test
    session's setting; tests/test_cpu_fallback.py covers it on): with no GPU
    every hot-path call returns ECGPU_ERR_HIP with a message; through the drop-in names a void
    call exits 1 with the message (the reference's convention,
    galois.cpp:330-334) and jerasure_matrix_decode returns -1 (its own
    failure result, which the client handles, client_main.cpp:2118-2124)."""
    from erasure_coding_test_amd import _native as N
    a = np.arange(64, dtype=np.uint8)
    b = np.zeros(64, np.uint8)
    before = b.copy()
    for fn, args in (("ecgpu_galois_region_xor", (a.ctypes.data, a.ctypes.data, b.ctypes.data, 64)),
                     ("ecgpu_galois_w08_region_multiply", (a.ctypes.data, 7, 64, b.ctypes.data, 0)),
                     ("ecgpu_galois_w16_region_multiply", (a.ctypes.data, 0, 64, b.ctypes.data, 0)),
                     ("ecgpu_galois_w32_region_multiply", (a.ctypes.data, 9, 64, b.ctypes.data, 1))):
        assert getattr(N.lib, fn)(*args) == -3, fn
        assert N.last_error(), fn
        assert np.array_equal(b, before), fn
    code = ("import ctypes, numpy as np\n"
            f"L = ctypes.CDLL({os.path.join(os.path.dirname(N.LIB_PATH), 'libjerasure_amd.so')!r})\n"
            "f = L._Z17galois_region_xorPcS_S_i\n"
            "f.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int]\n"
            "a = np.zeros(64, np.uint8)\n"
            "f(a.ctypes.data, a.ctypes.data, a.ctypes.data, 64)\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 1 and "MI355X path failed" in r.stderr
    code = ("import ctypes, numpy as np\n"
            f"L = ctypes.CDLL({os.path.join(os.path.dirname(N.LIB_PATH), 'libjerasure_amd.so')!r})\n"
            "vdm = L._Z34reed_sol_vandermonde_coding_matrixiii\n"
            "vdm.restype = ctypes.c_void_p\n"
            "M = vdm(4, 2, 8)\n"
            "dec = L._Z22jerasure_matrix_decodeiiiPiiS_PPcS1_i\n"
            "bufs = [np.zeros(64, np.uint8) for _ in range(6)]\n"
            "P = ctypes.c_void_p * 6\n"
            "ptrs = P(*[b.ctypes.data for b in bufs])\n"
            "er = (ctypes.c_int * 2)(0, -1)\n"
            "rc = dec(4, 2, 8, ctypes.c_void_p(M), 0, er, ptrs, ctypes.byref(ptrs, 4 * 8), 64)\n"
            "print('rc', rc)\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "rc -1" in r.stdout and "MI355X path failed" in r.stderr, (r.stdout, r.stderr)


def test_int_array_accepts_any_iterable():
    from erasure_coding_test_amd import _native as N
    assert list(N.int_array(x for x in range(3))) == [0, 1, 2]
    assert list(N.int_array(iter(range(100)))) == list(range(100))  # the numpy branch
    assert list(N.int_array([2**32 - 1])) == [-1]  # wraps like a C int
