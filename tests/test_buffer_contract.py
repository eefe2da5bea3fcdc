"""The buffer contract (csrc/buffer_contract.hpp): the regions of one call are
identical or disjoint.

The reference runs every call as sequential whole-region byte loops
(galois.cpp:452-465, :731-754; jerasure.cpp:561-620), so a written region
that partially overlaps another region of the call -- a shifted alias -- gets
bytes fixed by its loop order; the GPU kernels would return different (and
run-to-run different) bytes there.  Such calls are rejected with
ECGPU_ERR_ARG, naming the pair, before anything touches the GPU -- so the
CPU cases below run without one.  Identical pointers keep the reference's
sequential semantics (tests/test_gpu_parity.py ::test_aliased_*,
::test_host_region_ops_aliasing), and read-only overlaps are allowed.
"""
import ctypes
import random
import subprocess
import sys

import numpy as np
import pytest

E = pytest.importorskip("erasure_coding_test_amd")
from erasure_coding_test_amd import _native as N  # noqa: E402

SHIFTS = (1, 8, 4096)
SIZE = 8192


def _pp(ptrs):
    return ctypes.cast(N.ptr_array(ptrs), N.c_void_pp)


def _check(rows, nsrc, srcs, dsts, size):
    stripes = len(srcs) // nsrc
    return N.lib.ecgpu_plan_check_buffers(rows, nsrc, stripes, _pp(srcs), _pp(dsts), size)


def _brute(rows, nsrc, srcs, dsts, size):
    """The contract of ecgpu_plan_check_buffers restated pair by pair."""
    if size <= 0:
        return True
    spans = [(p, False, i // nsrc) for i, p in enumerate(srcs)] + [(p, True, i // rows) for i, p in enumerate(dsts)]
    for i, (p, wp, sp) in enumerate(spans):
        for j, (q, wq, sq) in enumerate(spans):
            if i >= j or not (wp or wq) or not (p < q + size and q < p + size):
                continue
            if p == q and wp != wq and sp == sq and rows <= 4:
                continue  # an in-place output of its own stripe, one launch
            return False
    return True


@pytest.mark.parametrize("seed", range(40))
def test_plan_check_matches_pairwise_rule(seed):
    """The O(n log n) sweep agrees with the pairwise rule on random binds."""
    rng = random.Random(seed)
    rows, nsrc, stripes = rng.randint(1, 6), rng.randint(1, 5), rng.randint(1, 4)
    size = rng.choice([1, 7, 64, 100])
    base = 1 << 20
    pool = [base + rng.randrange(0, 12) * rng.choice([1, 16, 50]) for _ in range(6)]  # clustered addresses
    pick = lambda: rng.choice(pool) if rng.random() < 0.6 else base + rng.randrange(0, 4000)
    srcs = [pick() for _ in range(stripes * nsrc)]
    dsts = [pick() for _ in range(stripes * rows)]
    for trial in range(8):
        if trial:  # perturb: make some binds legal, some not
            dsts = [d + rng.choice([0, 0, size, 2 * size + 3, 1000]) for d in dsts]
        want = _brute(rows, nsrc, srcs, dsts, size)
        rc = _check(rows, nsrc, srcs, dsts, size)
        assert (rc == 0) == want, (rows, nsrc, srcs, dsts, size, N.last_error())
        if rc:
            assert rc == N.ECGPU_ERR_ARG and "overlap" in N.last_error()


def test_plan_check_rules():
    b, S = 1 << 20, 4096
    assert _check(2, 2, [b, b + S], [b + 2 * S, b + 3 * S], S) == 0                 # disjoint
    assert _check(2, 2, [b, b + 1], [b + 2 * S, b + 3 * S], S) == 0                 # sources may overlap
    assert _check(2, 2, [b, b + S], [b + S, b + 3 * S], S) == 0                     # in place, own stripe
    assert _check(5, 2, [b, b + S], [b + S] + [b + (3 + i) * S for i in range(4)], S) == N.ECGPU_ERR_ARG  # > 4 rows
    assert "the same buffer" in N.last_error()
    assert _check(1, 1, [b, b + S], [b + S, b + 2 * S], S) == N.ECGPU_ERR_ARG      # another stripe reads it
    assert _check(1, 1, [b, b + S], [b + 2 * S, b + 2 * S], S) == N.ECGPU_ERR_ARG  # two writers
    for shift in SHIFTS:
        assert _check(1, 2, [b, b + 4 * S], [b + shift], 2 * S) == N.ECGPU_ERR_ARG
        msg = N.last_error()
        assert "ecgpu_plan_bind" in msg and f"overlap by {2 * S - shift} bytes" in msg, msg
    assert _check(1, 2, [b, b + 2 * S], [b + 1], 0) == 0                            # size 0 touches nothing


def _sync_cases(base, shift):
    """Synchronous calls whose written region is shifted against another."""
    a, c = base, base + 3 * SIZE
    M = E.reed_sol.reed_sol_vandermonde_coding_matrix(4, 2, 8)
    four = [base + i * SIZE for i in range(4)]
    return [
        ("galois_region_xor", lambda: N.lib.ecgpu_galois_region_xor(a, c, a + shift, SIZE)),
        ("galois_w08_region_multiply", lambda: N.lib.ecgpu_galois_w08_region_multiply(a, 0x1D, SIZE, a + shift, 1)),
        ("galois_w16_region_multiply", lambda: N.lib.ecgpu_galois_w16_region_multiply(a, 0x1D, SIZE, a + shift, 1)),
        ("jerasure_matrix_encode", lambda: N.lib.ecgpu_jerasure_matrix_encode(
            4, 2, 8, N.int_array(M), _pp(four), _pp([four[1] + shift, base + 5 * SIZE]), SIZE)),
        ("jerasure_matrix_decode", lambda: N.lib.ecgpu_jerasure_matrix_decode(
            4, 2, 8, N.int_array(M), 0, N.int_array([0, -1]), _pp([four[1] + shift] + four[1:]),
            _pp([base + 4 * SIZE, base + 5 * SIZE]), SIZE)),
        ("jerasure_matrix_dotprod", lambda: N.lib.ecgpu_jerasure_matrix_dotprod(
            4, 8, N.int_array(M[4:]), None, 4, _pp(four), _pp([four[3] + shift, 0]), SIZE)),
    ]


@pytest.mark.parametrize("shift", SHIFTS)
def test_sync_calls_reject_shifted_aliases_before_the_gpu(shift):
    buf = np.random.default_rng(shift).integers(0, 256, 8 * SIZE, dtype=np.uint8)
    before = buf.copy()
    for name, call in _sync_cases(buf.ctypes.data, shift):
        assert call() == N.ECGPU_ERR_ARG, name
        msg = N.last_error()
        assert msg.startswith(name) and "overlap by" in msg and "identical or disjoint" in msg, msg
    assert np.array_equal(buf, before)  # nothing written


def test_identical_aliases_pass_the_contract():
    """r3 == r1, in-place multiply, an output that is also a source: the
    contract lets them through (on a GPU they run with the reference's
    sequential semantics; here they fail later, at the missing GPU)."""
    buf = np.zeros(4 * SIZE, np.uint8)
    a, b = buf.ctypes.data, buf.ctypes.data + 2 * SIZE
    for rc in (N.lib.ecgpu_galois_region_xor(a, b, a, SIZE),
               N.lib.ecgpu_galois_w08_region_multiply(a, 7, SIZE, None, 0),
               N.lib.ecgpu_galois_w08_region_multiply(a, 7, SIZE, a, 1),
               N.lib.ecgpu_galois_region_xor(a, a + 1, b, SIZE)):  # overlapping sources are only read
        assert rc != N.ECGPU_ERR_ARG, N.last_error()


DROPIN_SHIFTED = """
import ctypes, numpy as np, sys
L = ctypes.CDLL({path!r})
a = np.arange(3 * 8192, dtype=np.uint64).view(np.uint8).copy()
p = a.ctypes.data
if sys.argv[1] == "xor":
    f = L._Z17galois_region_xorPcS_S_i
    f.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int]
    f(p, p + 2 * 8192, p + {shift}, 8192)
    print("returned")
elif sys.argv[1] == "mul":
    f = L._Z26galois_w08_region_multiplyPciiS_i
    f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    f(p, 29, 8192, p + {shift}, 1)
    print("returned")
else:
    vdm = L._Z34reed_sol_vandermonde_coding_matrixiii
    vdm.restype = ctypes.c_void_p
    M = vdm(2, 2, 8)
    dec = L._Z22jerasure_matrix_decodeiiiPiiS_PPcS1_i
    P = ctypes.c_void_p * 4
    ptrs = P(p + {shift}, p, p + 8192, p + 2 * 8192)   # data[0] (erased) shifted onto data[1]
    er = (ctypes.c_int * 2)(0, -1)
    rc = dec(2, 2, 8, ctypes.c_void_p(M), 0, er, ptrs, ctypes.byref(ptrs, 2 * 8), 4096)
    print("rc", rc)
"""


def run_dropin_shifted(kind, shift):
    code = DROPIN_SHIFTED.format(path=N.DROPIN_PATH, shift=shift)
    return subprocess.run([sys.executable, "-c", code, kind], capture_output=True, text=True, timeout=120)


@pytest.mark.parametrize("shift", SHIFTS)
def test_dropin_rejects_shifted_aliases_through_reference_channels(shift):
    """Through the reference's own names: the void region calls print the
    conflict and exit(1) (galois.cpp:330-334 convention); decode returns -1
    (client_main.cpp:2118-2124 handles it)."""
    for kind in ("xor", "mul"):
        r = run_dropin_shifted(kind, shift)
        assert r.returncode == 1 and "returned" not in r.stdout, (kind, r.stdout, r.stderr)
        assert "arguments rejected" in r.stderr and "identical or disjoint" in r.stderr, r.stderr
    r = run_dropin_shifted("decode", shift if shift < 4096 else 2048)
    assert r.returncode == 0 and "rc -1" in r.stdout, (r.stdout, r.stderr)
    assert "jerasure_matrix_decode: arguments rejected" in r.stderr, r.stderr


# ------------------------------------------------ on the GPU box (-m gpu) ----
@pytest.fixture(scope="module")
def dev_buf(gpu):
    import torch
    g = torch.Generator(device="cpu").manual_seed(5)
    return torch.randint(0, 256, (8 * SIZE,), dtype=torch.uint8, generator=g).to(gpu)


@pytest.mark.gpu
@pytest.mark.parametrize("shift", SHIFTS)
def test_shifted_aliases_rejected_on_device_buffers(dev_buf, shift):
    import torch
    before = dev_buf.clone()
    for name, call in _sync_cases(dev_buf.data_ptr(), shift):
        assert call() == N.ECGPU_ERR_ARG, name
        assert N.last_error().startswith(name) and "identical or disjoint" in N.last_error()
    torch.cuda.synchronize()
    assert torch.equal(dev_buf, before)


@pytest.mark.gpu
@pytest.mark.parametrize("shift", SHIFTS)
def test_dropin_rejects_shifted_aliases_with_a_gpu(gpu, shift):
    """The same drop-in calls as the CPU test, with a GPU present: the
    rejection does not depend on the GPU being absent."""
    test_dropin_rejects_shifted_aliases_through_reference_channels(shift)


@pytest.mark.gpu
@pytest.mark.parametrize("shift", SHIFTS)
def test_plan_bind_and_encode_batch_reject(gpu, dev_buf, shift):
    from erasure_coding_test_amd import plan
    k, m = 2, 1
    M = [1, 1]
    base = dev_buf.data_ptr()
    p = plan.encode_plan(k, m, M)
    with pytest.raises(N.EcgpuError, match="overlap by"):
        p.bind([[base, base + 2 * SIZE]], [[base + shift]], SIZE)
    p.bind([[base, base + 2 * SIZE]], [[base + 4 * SIZE]], SIZE)  # disjoint: fine
    rc = N.lib.ecgpu_encode_batch(k, m, N.int_array(M), 1, _pp([base, base + 2 * SIZE]), _pp([base + 2 * SIZE + shift]),
                                  SIZE, None)
    assert rc == N.ECGPU_ERR_ARG and "overlap by" in N.last_error()


@pytest.mark.gpu
@pytest.mark.parametrize("shift", SHIFTS)
def test_pipeline_submit_rejects_and_keeps_working(gpu, restatement, shift):
    from oracle.oracle import alloc_shards
    k, m = 4, 2
    M = E.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    slab = np.random.default_rng(shift).integers(0, 256, 8 * SIZE, dtype=np.uint8)
    data = [slab.ctypes.data + i * SIZE for i in range(k)]
    bad_coding = [data[2] + shift, slab.ctypes.data + 6 * SIZE]
    pipe = N.lib.ecgpu_pipeline_create(k, m, N.int_array(M), SIZE, 2, -1)
    grp = N.lib.ecgpu_pipeline_group_create(k, m, N.int_array(M), SIZE, 2, 1, N.int_array([0]))
    try:
        assert N.lib.ecgpu_pipeline_submit(pipe, _pp(data), _pp(bad_coding)) == N.ECGPU_ERR_ARG
        assert "coding_ptrs[0]" in N.last_error() and "data_ptrs[2]" in N.last_error()
        assert N.lib.ecgpu_pipeline_group_submit(grp, _pp(data), _pp(bad_coding)) == N.ECGPU_ERR_ARG
        # identical pointers are rejected too: the pipeline reads every source first
        assert N.lib.ecgpu_pipeline_submit(pipe, _pp(data), _pp([data[1], bad_coding[1]])) == N.ECGPU_ERR_ARG
        coding = alloc_shards(m, SIZE, 16)
        for h in (pipe, grp):
            for c in coding:
                c[:] = 0
            sub = N.lib.ecgpu_pipeline_submit if h == pipe else N.lib.ecgpu_pipeline_group_submit
            wait = N.lib.ecgpu_pipeline_wait if h == pipe else N.lib.ecgpu_pipeline_group_wait
            t = sub(h, _pp(data), _pp([c.ctypes.data for c in coding]))
            assert t == 0, N.last_error()  # the rejected stripe took no ticket
            assert wait(h, t) == 0
            ref = alloc_shards(m, SIZE, 16)
            restatement.matrix_encode(k, m, np.array(M).reshape(m, k), [slab[i * SIZE:(i + 1) * SIZE] for i in range(k)],
                                      ref, SIZE)
            for a, b in zip(coding, ref):
                assert np.array_equal(a[:SIZE], b[:SIZE])
    finally:
        N.lib.ecgpu_pipeline_destroy(pipe)
        N.lib.ecgpu_pipeline_group_destroy(grp)


@pytest.mark.gpu
@pytest.mark.parametrize("shift", SHIFTS)
def test_accumulator_rejects_a_block_inside_an_accumulator(gpu, shift):
    a = N.lib.ecgpu_accum_create(2, SIZE, -1)
    try:
        acc0 = N.lib.ecgpu_accum_device_ptr(a, 0)
        for fn in (N.lib.ecgpu_accum_add, N.lib.ecgpu_accum_add_async):
            assert fn(a, acc0 + shift, N.int_array([1, 7])) == N.ECGPU_ERR_ARG
            assert "overlap by" in N.last_error()
        assert N.lib.ecgpu_accum_sync(a) == 0
        # nothing was applied: both accumulators are still untouched
        out = np.zeros(SIZE, np.uint8)
        assert N.lib.ecgpu_accum_read(a, 0, out.ctypes.data, SIZE) == N.ECGPU_ERR
    finally:
        N.lib.ecgpu_accum_destroy(a)


@pytest.mark.gpu
@pytest.mark.parametrize("shift", (8, 64))
def test_bitmatrix_call_rejects_overlapping_devices(gpu, dev_buf, shift):
    k, m, w, ps = 2, 1, 8, 64
    M = E.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, w)
    B = E.jerasure.jerasure_matrix_to_bitmatrix(k, m, w, M)
    base = dev_buf.data_ptr()
    size = w * ps * 4
    data = [base, base + size]
    for coding in ([data[1] + shift], [data[1]]):  # shifted, and identical (the packet map models devices, not memory)
        rc = N.lib.ecgpu_jerasure_bitmatrix_encode(k, m, w, N.int_array(B), _pp(data), _pp(coding), size, ps)
        assert rc == N.ECGPU_ERR_ARG and "device pointer" in N.last_error(), N.last_error()
