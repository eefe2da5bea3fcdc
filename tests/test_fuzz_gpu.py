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

test_fuzz_aliased_calls_vs_reference repeats buffers inside a call and
shifts one onto another (the buffer contract); ECGPU_FUZZ_ALIAS_CASES
(default 300).
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
        if case and case % 2000 == 0:  # progress for long runs under `pytest -s` (a silent run looks hung)
            print(f"fuzz: {case}/{cases} cases", flush=True)
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


def _aliased(n, rng):
    """slot i -> the slot whose buffer it uses: itself, or (with probability
    1/4) an earlier slot -- identical pointers, as a caller that passes one
    buffer twice."""
    owner = []
    for i in range(n):
        owner.append(int(rng.integers(0, i)) if i and rng.random() < 0.25 else i)
    return owner


def test_fuzz_aliased_calls_vs_reference(ec, gpu, reference):
    """Calls whose pointer arrays repeat buffers (a coding shard that is also a
    data shard, two outputs on one buffer, r3 == r1): the reference's
    sequential semantics, replayed by the planner, bit-exact on device and
    pageable buffers.  And the same calls with one buffer shifted onto
    another by 1..size-1 bytes: rejected (EcgpuError, ECGPU_ERR_ARG) with
    every buffer untouched (buffer_contract.hpp)."""
    import torch
    from erasure_coding_test_amd import _native as N
    cases = int(os.environ.get("ECGPU_FUZZ_ALIAS_CASES", "300"))
    rng = np.random.default_rng(4242)
    done = {"encode": 0, "dotprod": 0, "decode": 0, "region": 0, "rejected": 0}
    for case in range(cases):
        if case and case % 500 == 0:
            print(f"alias fuzz: {case}/{cases} cases", flush=True)
        kind = ("encode", "dotprod", "decode", "region")[int(rng.integers(0, 4))]
        where = ("device", "pageable")[int(rng.integers(0, 2))]
        size = int(rng.choice([8, 4096, 65536 + 8, 262144, (1 << 20) + 8]))
        shift = rng.random() < 0.2
        if kind == "region":
            k, m = 1, 2
        elif kind == "decode":
            k, m = int(rng.integers(2, 11)), int(rng.integers(1, 5))
        else:
            k, m = int(rng.integers(1, 13)), int(rng.integers(1, 6))
        n = k + m
        owner = _aliased(n, rng)
        uniq = sorted(set(owner))
        pool = {u: rng.integers(0, 256, size, dtype=np.uint8) for u in uniq}
        ctx = (case, kind, where, size, k, m, owner)

        def call(mod, bufs):
            d, c = bufs[:k], bufs[k:]
            if kind == "encode":
                M = [int(x) for x in rng_m.choice([0, 1, 2, 0x8E, 77], size=k * m)]
                if mod is None:
                    reference.matrix_encode(k, m, np.array(M).reshape(m, k), d, c, size)
                else:
                    mod.jerasure.jerasure_matrix_encode(k, m, 8, M, d, c, size)
                return 0
            if kind == "dotprod":
                row = [int(x) for x in rng_m.choice([0, 1, 3, 0x1D], size=k)]
                dest = int(rng_m.integers(0, n))
                if mod is None:
                    reference.matrix_dotprod(k, row, None, dest, d, c, size)
                else:
                    mod.jerasure.jerasure_matrix_dotprod(k, 8, row, None, dest, d, c, size)
                return 0
            if kind == "decode":
                M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
                er = sorted(int(x) for x in rng_m.choice(n, size=int(rng_m.integers(1, m + 1)), replace=False))
                if mod is None:
                    return reference.matrix_decode(k, m, np.array(M).reshape(m, k), 0, er, d, c, size)
                return mod.jerasure.jerasure_matrix_decode(k, m, 8, M, 0, er, d, c, size)
            op = int(rng_m.integers(0, 3))
            a, b, x = bufs[0], bufs[1], bufs[2]
            if op == 0:
                (reference.region_xor if mod is None else mod.galois.galois_region_xor)(a, b, x, size)
            else:
                f = reference.region_multiply if mod is None else mod.galois.galois_w08_region_multiply
                f(a, 0x35, size, x, op - 1)
            return 0

        # the reference on numpy views of the host pool: slot i -> pool[owner[i]]
        ref_pool = {u: v.copy() for u, v in pool.items()}
        rng_m = np.random.default_rng(case)
        rc_ref = call(None, [ref_pool[owner[i]] for i in range(n)])
        if where == "device":
            gpool = {u: torch.from_numpy(v.copy()).to(gpu) for u, v in pool.items()}
        else:
            gpool = {u: v.copy() for u, v in pool.items()}
        if shift:
            # one slot (read or written) moved onto a written slot's buffer by s bytes
            big = {u: (torch.zeros(2 * size, dtype=torch.uint8, device=gpu) if where == "device"
                       else np.zeros(2 * size, np.uint8)) for u in uniq}
            for u in uniq:
                big[u][:size] = gpool[u]
            s = int(rng.integers(1, size)) if size > 1 else 1
            victim, target = int(rng.integers(0, n)), int(rng.integers(k, n))
            if owner[victim] == owner[target]:
                continue
            bufs = [big[owner[i]][:size] for i in range(n)]
            bufs[victim] = big[owner[target]][s:s + size]
            before = {u: (big[u].cpu().numpy().copy() if where == "device" else big[u].copy()) for u in uniq}
            rng_m = np.random.default_rng(case)
            try:
                call(ec, bufs)
                raised = False
            except N.EcgpuError as ex:
                assert "identical or disjoint" in str(ex), ctx + (str(ex),)
                raised = True
            # an output may not be written (all-zero dotprod row, decode with no erasure to fill,
            # a coefficient-0 region op): the call then has no written region and may run
            if not raised:
                continue
            done["rejected"] += 1
            torch.cuda.synchronize()
            for u in uniq:
                now = big[u].cpu().numpy() if where == "device" else big[u]
                assert np.array_equal(now, before[u]), ctx + ("touched after rejection", u)
            continue
        rng_m = np.random.default_rng(case)
        rc = call(ec, [gpool[owner[i]] for i in range(n)])
        torch.cuda.synchronize()
        assert rc == rc_ref, ctx
        for u in uniq:
            got = gpool[u].cpu().numpy() if where == "device" else gpool[u]
            assert np.array_equal(got, ref_pool[u]), ctx + (u,)
        done[kind] += 1
    assert all(v > 0 for v in done.values()), done
