"""Seeded fuzz of the synchronous hot-path calls against the reference library
compiled in place (oracle/_ref): many random shapes in one test, bytes and
return codes compared exactly.

Each case draws one of
  * jerasure_matrix_encode, k 1..16 (inline launches) and 17..24 (plans),
    m 1..8, including all-zero / aliased-free random matrices;
  * jerasure_matrix_decode, Vandermonde RS(k,m), up to m + 1 erasures (the
    last may be undecodable: the return code must match), row_k_ones 0/1;
  * galois_w08_region_multiply with and without add, galois_region_xor;
  * jerasure_matrix_dotprod with and without src_ids,
with sizes from 8 B to 2 MiB in whole 8-byte words (the reference's loops
over-run other sizes by design, galois.cpp:452-465), on device tensors,
pageable numpy arrays or pinned tensors -- so every staging mode of a
synchronous call (device, zero-copy, bounce, outputs in coherent memory,
HIP copies, pinned in place) is crossed with every shape class.
ECGPU_FUZZ_CASES sets the case count (default 1500, ~15 s on MI355X).
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ec(gpu):
    import erasure_coding_test_amd as E
    return E


# 1 MiB + 8 and 2 MiB + 16 cross inline_ok's switch for 15-16 dense sources
# (inline up to 1 MiB, plan launches above)
SIZES = [8, 24, 4096, 4104, 65536, 100000, 262144, 349528, 655360, (1 << 20) + 8, (2 << 20) + 16]


def _bufs(arrays, where, gpu):
    import torch
    if where == "device":
        return [torch.from_numpy(a.copy()).to(gpu) for a in arrays]
    if where == "pinned":
        return [torch.from_numpy(a.copy()).pin_memory() for a in arrays]
    return [a.copy() for a in arrays]


def _host(bufs):
    return [b.cpu().numpy() if hasattr(b, "cpu") else b for b in bufs]


def test_fuzz_sync_calls_vs_reference(ec, gpu, reference):
    import torch
    cases = int(os.environ.get("ECGPU_FUZZ_CASES", "1500"))
    rng = np.random.default_rng(20261016)
    kinds = {"encode": 0, "decode": 0, "region": 0, "dotprod": 0}
    for case in range(cases):
        kind = ("encode", "decode", "region", "dotprod")[int(rng.integers(0, 4))]
        where = ("device", "pageable", "pinned")[int(rng.integers(0, 3))]
        size = int(rng.choice(SIZES))
        if 100000 < size < (1 << 20) and rng.random() < 0.5:
            size = 8 * int(rng.integers(1, size // 8))  # ragged within the range, still whole words
        ctx = (case, kind, where, size)
        kinds[kind] += 1
        if kind in ("encode", "dotprod"):
            k = int(rng.integers(1, 25 if kind == "encode" else 17))
            m = int(rng.integers(1, 9))
            # random coefficients with zeros and ones mixed in
            M = [int(x) for x in rng.choice([0, 1, 2, 3, 0x8E, int(rng.integers(0, 256))], size=k * m)]
            data = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(k)]
            coding = [np.full(size, 0x5A, np.uint8) for _ in range(m)]
            if kind == "encode":
                want = [c.copy() for c in coding]
                reference.matrix_encode(k, m, np.array(M).reshape(m, k), data, want, size)
                dd, dc = _bufs(data, where, gpu), _bufs(coding, where, gpu)
                ec.jerasure.jerasure_matrix_encode(k, m, 8, M, dd, dc, size)
                torch.cuda.synchronize()
                for i, (g, w) in enumerate(zip(_host(dc), want)):
                    assert np.array_equal(g, w), ctx + (k, m, i)
            else:
                row = M[:k]
                use_ids = rng.random() < 0.5
                src_ids = [int(x) for x in rng.permutation(k + m)[:k]] if use_ids else None
                dest = int(rng.integers(0, k + m))
                if src_ids is not None and dest in src_ids:
                    dest = next(i for i in range(k + m) if i not in src_ids)
                ref_d, ref_c = [d.copy() for d in data], [c.copy() for c in coding]
                reference.matrix_dotprod(k, row, src_ids, dest, ref_d, ref_c, size)
                dd, dc = _bufs(data, where, gpu), _bufs(coding, where, gpu)
                ec.jerasure.jerasure_matrix_dotprod(k, 8, row, src_ids, dest, dd, dc, size)
                torch.cuda.synchronize()
                for i, (g, w) in enumerate(zip(_host(dd) + _host(dc), ref_d + ref_c)):
                    assert np.array_equal(g, w), ctx + (k, m, src_ids, dest, i)
        elif kind == "decode":
            k, m = int(rng.integers(2, 17)), int(rng.integers(1, 9))
            M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
            ne = int(rng.integers(1, m + 2))
            erasures = sorted(int(x) for x in rng.choice(k + m, size=min(ne, k + m), replace=False))
            rko = int(rng.integers(0, 2))
            data = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(k)]
            coding = [np.zeros(size, np.uint8) for _ in range(m)]
            reference.matrix_encode(k, m, np.array(M).reshape(m, k), data, coding, size)
            for e in erasures:
                (data + coding)[e][:] = rng.integers(0, 256, size, dtype=np.uint8)
            ref = [b.copy() for b in data + coding]
            rc_ref = reference.matrix_decode(k, m, np.array(M).reshape(m, k), rko, erasures, ref[:k], ref[k:], size)
            bufs = _bufs(data + coding, where, gpu)
            rc = ec.jerasure.jerasure_matrix_decode(k, m, 8, M, rko, erasures, bufs[:k], bufs[k:], size)
            torch.cuda.synchronize()
            assert rc == rc_ref, ctx + (k, m, erasures, rko)
            for i, (g, w) in enumerate(zip(_host(bufs), ref)):
                assert np.array_equal(g, w), ctx + (k, m, erasures, rko, i)
        else:
            a = rng.integers(0, 256, size, dtype=np.uint8)
            b = rng.integers(0, 256, size, dtype=np.uint8)
            c = int(rng.integers(0, 256))
            op = int(rng.integers(0, 3))
            ra, rb = a.copy(), b.copy()
            ga, gb = _bufs([a, b], where, gpu)
            if op == 0:
                reference.region_multiply(ra, c, size, rb, 0)
                ec.galois.galois_w08_region_multiply(ga, c, size, gb, 0)
            elif op == 1:
                reference.region_multiply(ra, c, size, rb, 1)
                ec.galois.galois_w08_region_multiply(ga, c, size, gb, 1)
            else:
                rc_ = np.zeros(size, np.uint8)
                gc = _bufs([rc_], where, gpu)[0]
                reference.region_xor(ra, rb, rc_, size)
                ec.galois.galois_region_xor(ga, gb, gc, size)
                torch.cuda.synchronize()
                assert np.array_equal(_host([gc])[0], rc_), ctx + (op,)
            torch.cuda.synchronize()
            assert np.array_equal(_host([ga])[0], ra), ctx + (op, c)
            assert np.array_equal(_host([gb])[0], rb), ctx + (op, c)
    assert all(v > cases // 8 for v in kinds.values()), kinds
