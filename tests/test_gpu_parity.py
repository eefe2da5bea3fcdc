"""GPU parity: the MI355X path (through the C ABI, include/ecgpu.h) against the
golden vectors made by the reference and against the CPU oracle.

Bit-exact everywhere (integer/byte work).  Small sizes compare bytes; full
BASELINE sizes compare FNV-1a digests pinned by the reference plus
size-independent properties (encode -> erase -> decode round trips).
"""
import ctypes
import itertools
import os

import numpy as np
import pytest

from ecdata import CONFIGS, fnv1a64, shard_seed, splitmix_bytes
from oracle.oracle import alloc_shards

pytestmark = pytest.mark.gpu

PAD = 16


def host_shards(cfg, stripe, count, size, first=0):
    out = alloc_shards(count, size, PAD)
    for s in range(count):
        out[s][:size] = splitmix_bytes(size, shard_seed(cfg, stripe, first + s))
    return out


def to_dev(arrs, dev):
    import torch
    return [torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in arrs]


def to_host(tensors):
    return [t.cpu().numpy() for t in tensors]


def digests(bufs, size):
    return [fnv1a64(np.asarray(b)[:size]) for b in bufs]


@pytest.fixture(scope="module")
def ec(gpu):
    import erasure_coding_test_amd as E
    return E


# ------------------------------------------------------------ golden ----
@pytest.mark.parametrize("where", ["device", "host"])
@pytest.mark.parametrize("cfg", sorted(CONFIGS))
def test_encode_small_golden(ec, gpu, golden, vectors, cfg, where):
    k, m = CONFIGS[cfg]["k"], CONFIGS[cfg]["m"]
    M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    for size in (4096, 4099, 1000, 7, 1):
        for stripe in range(2):
            data = host_shards(cfg, stripe, k, size)
            coding = alloc_shards(m, size, PAD)
            if where == "device":
                dd, dc = to_dev(data, gpu), to_dev(coding, gpu)
                ec.jerasure.jerasure_matrix_encode(k, m, 8, M, dd, dc, size)
                coding = to_host(dc)
            else:
                ec.jerasure.jerasure_matrix_encode(k, m, 8, M, data, coding, size)
            assert digests(coding, size) == golden["encode_small"][f"C{cfg}:{size}:{stripe}"], (size, stripe)
            if size == 4096:
                assert np.array_equal(np.stack([c[:size] for c in coding]), vectors[f"enc_{cfg}_{stripe}"])


def test_decode_inconsistent_golden(ec, gpu, golden):
    mats = {}
    for case in golden["decode_inconsistent"]:
        k, m, cfg, size = case["k"], case["m"], case["cfg"], case["size"]
        if (k, m) not in mats:
            mats[(k, m)] = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
        bufs = to_dev(host_shards(cfg, 7, k, size) + host_shards(cfg, 7, m, size, first=k), gpu)
        rc = ec.jerasure.jerasure_matrix_decode(k, m, 8, mats[(k, m)], case["row_k_ones"], case["erasures"],
                                                bufs[:k], bufs[k:], size)
        assert rc == case["rc"], case["erasures"]
        assert digests(to_host(bufs), size) == case["digests"], (case["erasures"], case["row_k_ones"])


@pytest.fixture(scope="module")
def c4_inputs(golden):
    """The C4 stripe of golden["c4_full_inconsistent"]: 14 x 4 MiB shards whose
    parity is NOT the data's (host, pageable)."""
    g = golden["c4_full_inconsistent"]
    k, m, size, cfg = g["k"], g["m"], g["size"], g["cfg"]
    return host_shards(cfg, 7, k, size) + host_shards(cfg, 7, m, size, first=k)


@pytest.mark.parametrize("path", ["sync-device", "sync-host", "plan-2-stripes"])
def test_c4_full_size_inconsistent_golden(ec, gpu, golden, c4_inputs, path):
    """BASELINE config 4 at its own size (RS(10,4), 4 MiB shards) on inputs that
    are not a codeword, against the reference's jerasure_matrix_decode digests:
    the survivor choice (dm_ids = the first k non-erased, jerasure.cpp:84-112),
    the row_k_ones shortcut and the re-encode of erased parity from the
    recovered data (:223-247) show in the bytes.  Through the synchronous call
    on device and on pageable host buffers, and through DecodePlan on a
    2-stripe slab (the batched launch shape the bench times)."""
    import torch
    g = golden["c4_full_inconsistent"]
    k, m, size = g["k"], g["m"], g["size"]
    M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    for case in g["cases"]:
        er, rko = case["erasures"], case["row_k_ones"]
        if path == "sync-device":
            bufs = to_dev(c4_inputs, gpu)
            rc = ec.jerasure.jerasure_matrix_decode(k, m, 8, M, rko, er, bufs[:k], bufs[k:], size)
            got = [digests(to_host(bufs), size)]
        elif path == "sync-host":
            bufs = [b.copy() for b in c4_inputs]
            rc = ec.jerasure.jerasure_matrix_decode(k, m, 8, M, rko, er, bufs[:k], bufs[k:], size)
            got = [digests(bufs, size)]
        else:
            slab, shards = ec.alloc_stripes(2, k, m, size)
            for st in shards:
                for i in range(k + m):
                    st[i].copy_(torch.from_numpy(np.ascontiguousarray(c4_inputs[i][:size])))
            ec.DecodePlan(k, m, M, er, rko).bind_stripes(shards, size).launch()
            torch.cuda.synchronize()
            rc = 0
            got = [[fnv1a64(t.cpu().numpy()) for t in st] for st in shards]
        assert rc == case["rc"], (path, er, rko)
        for d in got:
            assert d == case["digests"], (path, er, rko)


def test_dotprod_golden(ec, gpu, golden):
    for t, case in enumerate(golden["dotprod"]):
        k, m, size = case["k"], case["m"], case["size"]
        bufs = to_dev(host_shards(9, case["seed_stripe"], k, size) +
                      host_shards(9, case["seed_stripe"], m, size, first=k), gpu)
        ec.jerasure.jerasure_matrix_dotprod(k, 8, case["row"], case["src_ids"], case["dest_id"], bufs[:k], bufs[k:],
                                            size)
        assert digests(to_host(bufs), size) == case["digests"], t


def test_region_ops_golden(ec, gpu, golden):
    for case in golden["region_multiply"]:
        size, t = case["size"], case["seed_stripe"]
        src, dst = to_dev([host_shards(10, t, 1, size)[0], host_shards(10, t, 1, size, first=1)[0]], gpu)
        if case["mode"] == "r2":
            ec.galois.galois_w08_region_multiply(src, case["multby"], size, dst, case["add"])
            out = dst
        else:
            ec.galois.galois_w08_region_multiply(src, case["multby"], size, None, case["add"])
            out = src
        assert fnv1a64(out.cpu().numpy()[:size]) == case["digest"], case
    for case in golden["region_xor"]:
        size = case["size"]
        a, b, c = to_dev(host_shards(11, case["seed_stripe"], 2, size) + alloc_shards(1, size, PAD), gpu)
        ec.galois.galois_region_xor(a, b, c, size)
        assert fnv1a64(c.cpu().numpy()[:size]) == case["digest"]
        ec.galois.galois_region_xor(a, b, a, size)  # r3 aliasing r1
        assert fnv1a64(a.cpu().numpy()[:size]) == case["digest"]


def test_stats_semantics(ec, gpu, golden):
    k, m = 10, 4
    M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    ec.jerasure.jerasure_get_stats()
    data = to_dev(host_shards(3, 0, k, 4096), gpu)
    coding = to_dev(alloc_shards(m, 4096, PAD), gpu)
    ec.jerasure.jerasure_matrix_encode(k, m, 8, M, data, coding, 4096)
    assert ec.jerasure.jerasure_get_stats() == golden["stats_after_rs10_4_encode_4096"]
    ec.jerasure.jerasure_matrix_decode(k, m, 8, M, 0, [0, 1, 2, 3], data, coding, 4096)
    assert ec.jerasure.jerasure_get_stats() == golden["stats_after_rs10_4_decode_0123_4096"]


# ---------------------------------------------------- full BASELINE sizes ----
@pytest.mark.parametrize("name", ["C2", "C3", "C5"])
def test_full_size_digests(ec, gpu, golden, name):
    import torch
    g = golden["full_size"][name]
    cfg = int(name[1:])
    k, m, size = g["k"], g["m"], g["size"]
    M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    data = [splitmix_bytes(size, shard_seed(cfg, 0, s)) for s in range(k)]
    assert [fnv1a64(d) for d in data] == g["data"]
    dd = to_dev(data, gpu)
    dc = [torch.empty(size, dtype=torch.uint8, device=gpu) for _ in range(m)]
    ec.jerasure.jerasure_matrix_encode(k, m, 8, M, dd, dc, size)
    assert [fnv1a64(c.cpu().numpy()) for c in dc] == g["coding"]


@pytest.mark.parametrize("erasures", [[0], [5], [10], [0, 1, 2, 3], [3, 7, 11, 13], [9, 10, 11, 12], [0, 13]])
def test_full_size_roundtrip_rs10_4(ec, gpu, erasures):
    import torch
    k, m, size = 10, 4, 4 << 20
    M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    g = torch.Generator(device="cpu").manual_seed(sum(erasures) + 17)
    data = [torch.randint(0, 256, (size,), dtype=torch.uint8, generator=g).to(gpu) for _ in range(k)]
    coding = [torch.empty(size, dtype=torch.uint8, device=gpu) for _ in range(m)]
    ec.jerasure.jerasure_matrix_encode(k, m, 8, M, data, coding, size)
    orig = [t.clone() for t in data + coding]
    bufs = [t.clone() for t in orig]
    for e in erasures:
        bufs[e].fill_(0x5A)
    assert ec.jerasure.jerasure_matrix_decode(k, m, 8, M, 0, erasures, bufs[:k], bufs[k:], size) == 0
    for a, b in zip(bufs, orig):
        assert torch.equal(a, b)


def test_too_many_erasures_returns_minus_one(ec, gpu):
    k, m, size = 6, 3, 64
    M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    bufs = to_dev(host_shards(2, 0, k + m, size), gpu)
    before = to_host(bufs)
    assert ec.jerasure.jerasure_matrix_decode(k, m, 8, M, 0, [0, 1, 2, 3], bufs[:k], bufs[k:], size) == -1
    for a, b in zip(to_host(bufs), before):
        assert np.array_equal(a, b)


# ----------------------------------------------------- batched plan API ----
def _encode_ref(restatement, k, m, M, data, size):
    coding = alloc_shards(m, size, PAD)
    restatement.matrix_encode(k, m, np.array(M).reshape(m, k), data, coding, size)
    return coding


@pytest.mark.parametrize("kind,nt", [(0, 1), (0, 0), (1, 1), (1, 0)])
@pytest.mark.parametrize("k,m", [(4, 2), (6, 3), (10, 4), (12, 4), (16, 3), (1, 1), (3, 4)])
def test_plan_batch_kernels(ec, gpu, restatement, kind, nt, k, m):
    import torch
    size, stripes = 65536 + 48, 5
    M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8) if k > 1 else [7] * m
    hdata = [host_shards(20 + k, s, k, size) for s in range(stripes)]
    data = [to_dev(h, gpu) for h in hdata]
    coding = [[torch.zeros(size + PAD, dtype=torch.uint8, device=gpu) for _ in range(m)] for _ in range(stripes)]
    p = ec.plan.encode_plan(k, m, M).bind(data, coding, size).set_kernel(kind, bool(nt))
    p.launch()
    torch.cuda.synchronize()
    for s in range(stripes):
        ref = _encode_ref(restatement, k, m, M, hdata[s], size)
        for a, b in zip(to_host(coding[s]), ref):
            assert np.array_equal(a[:size], b[:size]), (s,)
            assert not a[size:].any()  # nothing written past the shard


@pytest.mark.parametrize("k,m", [(17, 2), (20, 4), (32, 3), (24, 6)])
def test_generic_k_and_many_rows(ec, gpu, restatement, k, m):
    size = 40000 + 5
    M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    hdata = host_shards(30, k, k, size)
    dd, dc = to_dev(hdata, gpu), to_dev(alloc_shards(m, size, PAD), gpu)
    ec.jerasure.jerasure_matrix_encode(k, m, 8, M, dd, dc, size)
    for a, b in zip(to_host(dc), _encode_ref(restatement, k, m, M, hdata, size)):
        assert np.array_equal(a[:size], b[:size])


@pytest.mark.parametrize("offset", [1, 3, 8, 15])
def test_misaligned_buffers(ec, gpu, restatement, offset):
    import torch
    k, m, size = 6, 3, 10007
    M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    hdata = host_shards(31, offset, k, size)
    base = [torch.zeros(size + 64, dtype=torch.uint8, device=gpu) for _ in range(k + m)]
    views = [b[offset:offset + size] for b in base]
    for v, h in zip(views[:k], hdata):
        v.copy_(torch.from_numpy(h[:size]))
    ec.jerasure.jerasure_matrix_encode(k, m, 8, M, views[:k], views[k:], size)
    for a, b in zip(views[k:], _encode_ref(restatement, k, m, M, hdata, size)):
        assert np.array_equal(a.cpu().numpy(), b[:size])


@pytest.mark.parametrize("where,size", [("device", 5000), ("host", 5000), ("host", 300_001)])
def test_aliased_coding_buffers_follow_sequential_semantics(ec, gpu, restatement, where, size):
    # coding[0] aliases data[2]: the reference overwrites data[2] with parity 0
    # before computing parity 1..; the fused plan must reproduce that exactly.
    # m = 6 > 4 rows: two launches, outputs through temporaries.  Host buffers
    # take the pinned bounce (small) or per-buffer pageable copies (large).
    k, m = 6, 6
    M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    hdata = host_shards(32, 0, k, size)
    hcoding = alloc_shards(m, size, PAD)
    hcoding[0] = hdata[2]
    restatement.matrix_encode(k, m, np.array(M).reshape(m, k), hdata, hcoding, size)
    ref = [x.copy() for x in hdata + hcoding[1:]]
    if where == "device":
        dd = to_dev(host_shards(32, 0, k, size), gpu)
        dc = [dd[2]] + to_dev(alloc_shards(m - 1, size, PAD), gpu)
    else:
        dd = host_shards(32, 0, k, size)
        dc = [dd[2]] + alloc_shards(m - 1, size, PAD)
    ec.jerasure.jerasure_matrix_encode(k, m, 8, M, dd, dc, size)
    got = to_host(dd + dc[1:]) if where == "device" else dd + dc[1:]
    for a, b in zip(got, ref):
        assert np.array_equal(a[:size], b[:size])


@pytest.mark.parametrize("size", [4096, 1 << 20, 3 << 20])
def test_host_region_ops_aliasing(ec, gpu, restatement, size):
    """Region ops on pageable host buffers, in place and aliased, on both sides
    of the pinned-bounce threshold (2 MiB of staged bytes)."""
    a0, b0 = host_shards(33, 0, 2, size)
    a, b = a0.copy(), b0.copy()
    ra, rb = a0.copy(), b0.copy()
    ec.galois.galois_region_xor(a, b, a, size)  # r3 aliases r1
    restatement.region_xor(ra, rb, ra, size)
    assert np.array_equal(a[:size], ra[:size])
    ec.galois.galois_w08_region_multiply(b, 0x8E, size, None, 0)  # in place
    restatement.region_multiply(rb, 0x8E, size, None, 0)
    assert np.array_equal(b[:size], rb[:size])
    ec.galois.galois_w08_region_multiply(a, 0x1D, size, b, 1)  # b ^= 0x1D * a
    restatement.region_multiply(ra, 0x1D, size, rb, 1)
    assert np.array_equal(b[:size], rb[:size])
    assert np.array_equal(a[size:], a0[size:]) and np.array_equal(b[size:], b0[size:])  # padding untouched


@pytest.mark.parametrize("kind", [0, 1])  # v_perm engine, LDS nibble-table engine
def test_decode_plan_batch_matches_jerasure(ec, gpu, kind):
    import torch
    k, m, size, stripes = 10, 4, 1 << 18, 4
    M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    g = torch.Generator(device="cpu").manual_seed(3)
    shards = []
    for _ in range(stripes):
        d = [torch.randint(0, 256, (size,), dtype=torch.uint8, generator=g).to(gpu) for _ in range(k)]
        c = [torch.empty(size, dtype=torch.uint8, device=gpu) for _ in range(m)]
        ec.jerasure.jerasure_matrix_encode(k, m, 8, M, d, c, size)
        shards.append(d + c)
    orig = [[t.clone() for t in st] for st in shards]
    for er in ([0], [0, 1, 2, 3], [2, 11], [10, 11, 12, 13], [12], [5]):
        for st in shards:
            for e in er:
                st[e].zero_()
        dp = ec.plan.DecodePlan(k, m, M, er)
        dp.bind_stripes(shards, size).set_kernel(kind, True).launch()
        torch.cuda.synchronize()
        for st, o in zip(shards, orig):
            for a, b in zip(st, o):
                assert torch.equal(a, b), er


# --------------------------------------------------- other hot-path ops ----
def test_r6_and_parity(ec, gpu, restatement):
    k, size = 8, 9999
    hdata = host_shards(33, 0, k, size)
    dd, dc = to_dev(hdata, gpu), to_dev(alloc_shards(2, size, PAD), gpu)
    assert ec.reed_sol.reed_sol_r6_encode(k, 8, dd, dc, size) == 1
    R6 = ec.reed_sol.reed_sol_r6_coding_matrix(k, 8)
    ref = _encode_ref(restatement, k, 2, R6, hdata, size)
    for a, b in zip(to_host(dc), ref):
        assert np.array_equal(a[:size], b[:size])
    par = to_dev(alloc_shards(1, size, PAD), gpu)[0]
    ec.jerasure.jerasure_do_parity(k, dd, par, size)
    x = np.zeros(size, np.uint8)
    for h in hdata:
        x ^= h[:size]
    assert np.array_equal(par.cpu().numpy()[:size], x)
    t = dd[0].clone()
    ec.reed_sol.reed_sol_galois_w08_region_multby_2(t, size)
    ref2 = hdata[0].copy()
    restatement.region_multiply(ref2, 2, size, None, 0)
    assert np.array_equal(t.cpu().numpy()[:size], ref2[:size])


# --------------------------------------------- the C++ drop-in library ----
def _dropin():
    from erasure_coding_test_amd._native import DROPIN_PATH
    L = ctypes.CDLL(DROPIN_PATH)
    pp = ctypes.POINTER(ctypes.c_void_p)
    i = ctypes.c_int
    enc = L._Z22jerasure_matrix_encodeiiiPiPPcS1_i
    enc.argtypes, enc.restype = [i, i, i, ctypes.POINTER(i), pp, pp, i], None
    vdm = L._Z34reed_sol_vandermonde_coding_matrixiii
    vdm.argtypes, vdm.restype = [i, i, i], ctypes.c_void_p
    rmul = L._Z26galois_w08_region_multiplyPciiS_i
    rmul.argtypes, rmul.restype = [ctypes.c_void_p, i, i, ctypes.c_void_p, i], None
    rxor = L._Z17galois_region_xorPcS_S_i
    rxor.argtypes, rxor.restype = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, i], None
    return L, enc, vdm, rmul, rxor


def test_dropin_cpp_encode_host_buffers(gpu, restatement):
    L, enc, vdm, _, _ = _dropin()
    k, m, size = 3, 3, (1 << 20) + 5  # the reference client's EC_K/EC_M (ych_ec_test.h:5-6)
    mp = vdm(k, m, 8)
    M = list((ctypes.c_int * (k * m)).from_address(mp))
    hdata = host_shards(34, 0, k, size)
    coding = alloc_shards(m, size, PAD)
    arr = lambda bufs: (ctypes.c_void_p * len(bufs))(*[b.ctypes.data for b in bufs])
    enc(k, m, 8, (ctypes.c_int * (k * m))(*M), arr(hdata), arr(coding), size)
    for a, b in zip(coding, _encode_ref(restatement, k, m, M, hdata, size)):
        assert np.array_equal(a[:size], b[:size])


def test_dropin_ecx_incremental_accumulate(gpu, restatement):
    # ecx_datanode_main.cpp:680-735: blocks of a 1 MiB chunk split in 3
    # (349,525 B -- not a multiple of 8) arrive one source at a time; each
    # parity accumulator is memcpy'd / XORed / multiply-added with init[].
    L, _, vdm, rmul, rxor = _dropin()
    k, m, bs = 3, 3, (1 << 20) // 3
    M = list((ctypes.c_int * (k * m)).from_address(vdm(k, m, 8)))
    blocks = host_shards(35, 0, k, bs)
    acc = alloc_shards(m, bs, 8)
    init = [0] * m
    for j in range(k):
        for i in range(m):
            c = M[i * k + j]
            if c == 1:
                if not init[i]:
                    acc[i][:bs] = blocks[j][:bs]
                    init[i] = 1
                else:
                    rxor(blocks[j].ctypes.data, acc[i].ctypes.data, acc[i].ctypes.data, bs)
            elif c != 0:
                rmul(blocks[j].ctypes.data, c, bs, acc[i].ctypes.data, init[i])
                init[i] = 1
    for a, b in zip(acc, _encode_ref(restatement, k, m, M, blocks, bs)):
        assert np.array_equal(a[:bs], b[:bs])


def test_all_erasure_patterns_rs63_device(ec, gpu):
    import torch
    k, m, size = 6, 3, 4096 + 7
    M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    data = to_dev(host_shards(2, 9, k, size), gpu)
    coding = [torch.empty(size, dtype=torch.uint8, device=gpu) for _ in range(m)]
    ec.jerasure.jerasure_matrix_encode(k, m, 8, M, data, coding, size)
    orig = [t[:size].clone() for t in data] + [t.clone() for t in coding]
    for e in range(1, m + 1):
        for er in itertools.combinations(range(k + m), e):
            bufs = [t.clone() for t in orig]
            for i in er:
                bufs[i].fill_(0xEE)
            for rko in (0, 1):
                b2 = [t.clone() for t in bufs]
                assert ec.jerasure.jerasure_matrix_decode(k, m, 8, M, rko, list(er), b2[:k], b2[k:], size) == 0
                for a, b in zip(b2, orig):
                    assert torch.equal(a, b), (er, rko)


# ------------------------------------------- ECX device accumulators ----
@pytest.mark.parametrize("k,m,bs,where", [(3, 3, (1 << 20) // 3 + 1, "host"), (3, 3, (1 << 20) // 3, "device"),
                                          (10, 4, 4 << 20, "device"), (6, 3, 1000, "host")])
def test_ecx_parity_accumulator(ec, gpu, restatement, k, m, bs, where):
    # ecx_datanode_main.cpp:680-735: block j of every source arrives in order;
    # accumulator i gets coefficient matrix[i*k + j] with first-touch init[].
    M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    blocks = host_shards(36, bs % 97, k, bs)
    acc = ec.ParityAccumulator(m, bs)
    for j in range(k):
        blk = blocks[j] if where == "host" else to_dev([blocks[j]], gpu)[0]
        acc.add(blk, [M[i * k + j] for i in range(m)])
    ref = _encode_ref(restatement, k, m, M, blocks, bs)
    for i in range(m):
        out = np.zeros(bs, np.uint8)
        assert acc.read(i, out)
        assert np.array_equal(out, ref[i][:bs]), i
    acc.close()


@pytest.mark.parametrize("where", ["host", "pinned", "device"])
@pytest.mark.parametrize("k,m,bs", [(10, 4, (1 << 20) + 5), (5, 6, 4099), (3, 3, (1 << 20) // 3)])
def test_ecx_parity_accumulator_async(ec, gpu, restatement, where, k, m, bs):
    # queued adds (copy of block j+1 overlapping the update of block j), one
    # synchronous add in the middle, two stripes through the same
    # accumulators; m = 6 > 4 aliased rows takes the synchronous fallback
    import torch
    M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    acc = ec.ParityAccumulator(m, bs)
    for stripe in range(2):
        blocks = host_shards(39, stripe, k, bs)
        for j in range(k):
            if where == "device":
                blk = to_dev([blocks[j]], gpu)[0]
            elif where == "pinned":
                blk = torch.from_numpy(np.ascontiguousarray(blocks[j])).pin_memory()
            else:
                blk = blocks[j]
            acc.add(blk, [M[i * k + j] for i in range(m)], wait=(j == k // 2))
        acc.sync()
        ref = _encode_ref(restatement, k, m, M, blocks, bs)
        for i in range(m):
            out = np.zeros(bs, np.uint8)
            assert acc.read(i, out)
            assert np.array_equal(out, ref[i][:bs]), (stripe, i)
        acc.reset()
    acc.close()


def test_ecx_accumulator_zero_coefficients_and_reset(ec, gpu, restatement):
    k, m, bs = 4, 3, 4099
    coef = [[0, 0, 0, 0], [1, 0, 7, 1], [0, 29, 1, 142]]  # row 0 never touched
    blocks = host_shards(37, 0, k, bs)
    acc = ec.ParityAccumulator(m, bs)
    for rnd in range(2):  # second round after reset must not see round-1 state
        for j in range(k):
            acc.add(blocks[j], [coef[i][j] for i in range(m)])
        assert not acc.read(0, np.zeros(bs, np.uint8))
        ref = _encode_ref(restatement, k, m, [c for row in coef for c in row], blocks, bs)
        for i in (1, 2):
            out = np.zeros(bs, np.uint8)
            assert acc.read(i, out)
            assert np.array_equal(out, ref[i][:bs])
        acc.reset()
    acc.close()


# ------------------------------------------------ concurrency, graphs ----
def test_concurrent_callers_get_independent_contexts(ec, gpu, restatement):
    # client_main.cpp:1074-1164 runs ENC_THREAD_NUM encode pthreads at once;
    # every thread here encodes its own byte range of one stripe, repeatedly.
    import threading
    k, m, size, threads = 6, 3, (1 << 20) + 13, 8
    M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    data = host_shards(38, 0, k, size)
    coding = alloc_shards(m, size, PAD)
    bounds = [(t * size // threads, (t + 1) * size // threads) for t in range(threads)]
    errors = []

    def work(lo, hi):
        try:
            n = hi - lo
            d = [np.frombuffer((ctypes.c_uint8 * n).from_address(x.ctypes.data + lo), np.uint8) for x in data]
            c = [np.frombuffer((ctypes.c_uint8 * n).from_address(x.ctypes.data + lo), np.uint8) for x in coding]
            for _ in range(5):
                ec.jerasure.jerasure_matrix_encode(k, m, 8, M, d, c, n)
        except Exception as e:  # pragma: no cover - surfaced below
            errors.append(e)

    ts = [threading.Thread(target=work, args=b) for b in bounds]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors
    for a, b in zip(coding, _encode_ref(restatement, k, m, M, data, size)):
        assert np.array_equal(a[:size], b[:size])


def test_plan_launch_is_graph_capturable(ec, gpu, restatement):
    import torch
    k, m, size, stripes = 10, 4, 1 << 16, 3
    M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    slab, shards = ec.alloc_stripes(stripes, k, m, size)
    slab.zero_()
    enc = ec.encode_plan(k, m, M).bind([st[:k] for st in shards], [st[k:] for st in shards], size)
    dec = ec.DecodePlan(k, m, M, [0, 12]).bind_stripes(shards, size)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        enc.launch()  # warm-up outside capture
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        enc.launch()
        for st in shards:  # erase, then rebuild inside the same graph
            st[0].fill_(0)
            st[12].fill_(0)
        dec.launch()
    for rnd in range(2):
        hdata = [host_shards(39, rnd * 10 + st, k, size) for st in range(stripes)]
        for st in range(stripes):
            for j in range(k):
                shards[st][j].copy_(torch.from_numpy(hdata[st][j][:size]))
        g.replay()
        torch.cuda.synchronize()
        for st in range(stripes):
            ref = _encode_ref(restatement, k, m, M, hdata[st], size)
            for i in range(m):
                assert np.array_equal(shards[st][k + i].cpu().numpy(), ref[i][:size]), (rnd, st, i)
            for j in range(k):
                assert np.array_equal(shards[st][j].cpu().numpy(), hdata[st][j][:size])


@pytest.mark.parametrize("k,m", [(4, 2), (6, 3), (10, 4), (12, 4)])
@pytest.mark.parametrize("size", [4 << 10, (64 << 10) + 48, 256 << 10, 512 << 10])
def test_scheme_aware_slab_round_trip(ec, gpu, restatement, k, m, size):
    """Round 5's layouts (shard_stride.hpp: no skew up to 256 KiB and at
    512 KiB, RS(10,4)'s own entries at 256 / 512 KiB): alloc_stripes lays the
    slab out at ecgpu_recommended_shard_stride_km, and a batched encode, an
    erasure of m shards and a batched decode on it are bit-exact against the
    oracle."""
    import torch

    from erasure_coding_test_amd import _native as N
    stripes = 3
    M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    slab, shards = ec.alloc_stripes(stripes, k, m, size)
    stride = int(N.lib.ecgpu_recommended_shard_stride_km(size, k, m))
    assert slab.stride(1) == stride and stride % 256 == 0 and stride >= size
    hdata = [host_shards(41, st, k, size) for st in range(stripes)]
    for st in range(stripes):
        for j in range(k):
            shards[st][j].copy_(torch.from_numpy(hdata[st][j][:size]))
    ec.encode_plan(k, m, M).bind([st[:k] for st in shards], [st[k:] for st in shards], size).launch()
    torch.cuda.synchronize()
    refs = [_encode_ref(restatement, k, m, M, hdata[st], size) for st in range(stripes)]
    for st in range(stripes):
        for i in range(m):
            assert np.array_equal(shards[st][k + i].cpu().numpy(), refs[st][i][:size]), (st, i)
    erased = sorted(int(x) for x in np.random.default_rng(size + k).choice(k + m, size=m, replace=False))
    for st in shards:
        for e in erased:
            st[e].fill_(0)
    ec.DecodePlan(k, m, M, erased).bind_stripes(shards, size).launch()
    torch.cuda.synchronize()
    for st in range(stripes):
        for j in range(k):
            assert np.array_equal(shards[st][j].cpu().numpy(), hdata[st][j][:size]), (st, j, erased)
        for i in range(m):
            assert np.array_equal(shards[st][k + i].cpu().numpy(), refs[st][i][:size]), (st, i, erased)


# --------------------------------------------------- host pipeline ----
@pytest.mark.parametrize("memory", ["pageable", "registered", "torch_pinned"])
def test_host_pipeline_matches_oracle(ec, gpu, restatement, memory):
    import torch
    k, m, size, stripes = 10, 4, (1 << 20) + 3, 7
    M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    data = [host_shards(40, s, k, size) for s in range(stripes)]
    coding = [alloc_shards(m, size, PAD) for _ in range(stripes)]
    if memory == "registered":
        for bufs in data + coding:
            for b in bufs:
                ec.pipeline.host_register(b)
    if memory == "torch_pinned":
        data = [[torch.from_numpy(b).pin_memory() for b in st] for st in data]
        coding = [[torch.zeros(size + PAD, dtype=torch.uint8).pin_memory() for _ in range(m)] for _ in range(stripes)]
    p = ec.HostPipeline(k, m, M, size, depth=3)
    tickets = [p.submit(data[s], coding[s]) for s in range(stripes)]
    p.wait(tickets[2])
    p.drain()
    p.close()
    for s in range(stripes):
        hd = [np.asarray(b) if not hasattr(b, "numpy") else b.numpy() for b in data[s]]
        ref = _encode_ref(restatement, k, m, M, hd, size)
        for i in range(m):
            got = coding[s][i].numpy() if hasattr(coding[s][i], "numpy") else coding[s][i]
            assert np.array_equal(got[:size], ref[i][:size]), (s, i)
    if memory == "registered":
        for bufs in data + coding:
            for b in bufs:
                ec.pipeline.host_unregister(b)


@pytest.mark.parametrize("pattern", ["alternate", "pageable_then_pinned"])
def test_host_pipeline_mixed_output_memory(ec, gpu, restatement, pattern):
    """Pageable outputs go through the pipeline's D2H worker thread, pinned
    ones inline unless a worker job is pending: stripes switching between the
    two keep submission order (depth 2 reuses slots while jobs are queued),
    and close() with stripes in flight drains them."""
    import torch
    k, m, size, stripes = 6, 3, (1 << 20) + 16, 9
    M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    data = [host_shards(70, s, k, size) for s in range(stripes)]

    def pinned_at(s):
        return s % 2 == 1 if pattern == "alternate" else s >= stripes // 2

    coding = [[torch.full((size + PAD,), 0x77, dtype=torch.uint8).pin_memory() for _ in range(m)] if pinned_at(s)
              else [np.full(size + PAD, 0x77, np.uint8) for _ in range(m)] for s in range(stripes)]
    p = ec.HostPipeline(k, m, M, size, depth=2)
    tickets = [p.submit(data[s], coding[s]) for s in range(stripes)]
    p.wait(tickets[3])
    p.close()  # stripes 4.. still in flight
    for s in range(stripes):
        ref = _encode_ref(restatement, k, m, M, data[s], size)
        for i in range(m):
            got = coding[s][i].numpy() if hasattr(coding[s][i], "numpy") else coding[s][i]
            assert np.array_equal(got[:size], ref[i][:size]), (s, i)
            assert (got[size:] == 0x77).all(), (s, i)


@pytest.fixture
def d2h_worker_delay(knobs):
    """The test_d2h_delay_us knob (a test hook with no environment variable):
    the pipeline's D2H worker sleeps 3 ms between taking a job and issuing it
    (read when a pipeline is created)."""
    knobs.set("test_d2h_delay_us", 3000)
    yield


@pytest.mark.parametrize("pattern", ["alternate", "pageable_then_pinned"])
@pytest.mark.parametrize("depth", [1, 2])
def test_host_pipeline_wait_is_exact_with_delayed_worker(ec, gpu, restatement, d2h_worker_delay, pattern, depth):
    """Round-2 race: with pinned inputs, a pinned-output
    stripe following a pageable one used to be issued inline while the D2H
    worker still held the pageable job, so wait() on the earlier ticket could
    return before its outputs landed, its slot could be reused under the
    copy, and drain() could hang.  The worker's delay makes that window 3 ms
    wide on every run.  Each stripe is checked against the oracle right after
    wait(t) -- before the next submit can reuse its slot -- and the last
    stripe is pinned after a pageable one, so drain() must return."""
    import threading

    import torch
    k, m, size, stripes = 6, 3, (1 << 20) + 16, 8
    M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    data = [[torch.from_numpy(b).pin_memory() for b in host_shards(71, s, k, size)] for s in range(stripes)]

    def pinned_at(s):
        return s % 2 == 1 if pattern == "alternate" else s == stripes - 1

    coding = [[torch.full((size + PAD,), 0x77, dtype=torch.uint8).pin_memory() for _ in range(m)] if pinned_at(s)
              else [np.full(size + PAD, 0x77, np.uint8) for _ in range(m)] for s in range(stripes)]
    assert pinned_at(stripes - 1) and not pinned_at(stripes - 2)
    refs = [_encode_ref(restatement, k, m, M, [b.numpy() for b in data[s]], size) for s in range(stripes)]

    def check(s):
        for i in range(m):
            got = coding[s][i].numpy() if hasattr(coding[s][i], "numpy") else coding[s][i]
            assert np.array_equal(got[:size], refs[s][i][:size]), (s, i)
            assert (got[size:] == 0x77).all(), (s, i)

    p = ec.HostPipeline(k, m, M, size, depth=depth)
    try:
        prev = None
        for s in range(stripes):
            t = p.submit(data[s], coding[s])
            assert t == s
            if prev is not None:
                p.wait(prev)  # the ticket before: its slot is reused by the next submit at depth 2
                check(prev)
            prev = t
        done = threading.Event()
        th = threading.Thread(target=lambda: (p.drain(), done.set()), daemon=True)
        th.start()
        th.join(60)
        assert done.is_set(), "drain() did not return"
        check(stripes - 1)
    finally:
        p.close()


@pytest.mark.parametrize("pinned", [True, False])
@pytest.mark.parametrize("pitch_pad", [0, 4096 + 3])
@pytest.mark.parametrize("size", [(1 << 20) + 7, 1 << 20])
def test_host_pipeline_stripe_slab(ec, gpu, restatement, pinned, pitch_pad, size):
    """Stripes laid out in one host slab (evenly spaced shards, as the
    reference client's stripe buffer): the pipeline moves each direction as
    ONE copy -- 2-D into skewed ring slots, or 1-D when the slab is contiguous
    and the size lets the ring slots be contiguous (ECGPU_PIPE_CONTIG, 256-B
    multiples).  Encode, then a decode pipeline over the same slab with two
    data shards and one parity shard erased, against the oracle."""
    import torch
    k, m, stripes = 10, 4, 5
    pitch = size + pitch_pad
    M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    slab = torch.zeros((stripes, k + m, pitch), dtype=torch.uint8)
    if pinned:
        slab = slab.pin_memory()
    g = torch.Generator().manual_seed(pitch_pad + pinned)
    slab[:, :k, :size] = torch.randint(0, 256, (stripes, k, size), dtype=torch.uint8, generator=g)
    p = ec.HostPipeline(k, m, M, size, depth=3)
    for s in range(stripes):
        p.submit([slab[s, j] for j in range(k)], [slab[s, k + i] for i in range(m)])
    p.drain()
    p.close()
    want = slab.clone()
    for s in range(stripes):
        hd = alloc_shards(k, size, PAD)  # padded copies: the checker may read whole words
        for j in range(k):
            hd[j][:size] = slab[s, j, :size].numpy()
        ref = _encode_ref(restatement, k, m, M, hd, size)
        for i in range(m):
            assert np.array_equal(slab[s, k + i, :size].numpy(), ref[i][:size]), (s, i)
        assert not slab[s, k:, size:].any()  # nothing written past each shard
    er = [1, 6, k + 2]
    slab[:, er, :size] = 0
    d = ec.HostPipeline.decoder(k, m, M, er, size, depth=3)
    for s in range(stripes):
        d.submit([slab[s, j] for j in range(k)], [slab[s, k + i] for i in range(m)])
    d.drain()
    d.close()
    assert torch.equal(slab, want)


# zero-copy / bounce / HIP-copy staging; 600001 and 655360 stage more than the
# bounce limit with outputs <= 1 MiB each (sources by HIP's copies, outputs
# written by the kernel into coherent pinned memory); (3 << 20) + 48 keeps
# every row 16-B aligned when unpadded, so pinned rows run the vector columns
# grid-stride over a capped grid (ECGPU_ZC_GRID) with a partial last sweep
@pytest.mark.parametrize("size", [20000, 100003, 600001, 655360, (2 << 20) + 5, (3 << 20) + 48])
@pytest.mark.parametrize("pinned", [False, True])
@pytest.mark.parametrize("pitch_pad", [0, 4099])
def test_sync_calls_on_host_stripe_slab(ec, gpu, restatement, size, pinned, pitch_pad):
    """The synchronous drop-in names on shards laid out in one host slab
    (contiguous or padded rows, pageable or pinned): every staging mode of a
    host call -- zero-copy for small calls, the pinned bounce, HIP's copies
    with 2-D runs -- for encode, a decode with non-adjacent erased rows
    (data, data, parity) and RAID-6, against the oracle; nothing is written
    past any shard."""
    import torch
    k, m = 10, 4
    pitch = size + pitch_pad
    M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    slab = torch.zeros((k + m, pitch), dtype=torch.uint8)
    if pinned:
        slab = slab.pin_memory()
    g = torch.Generator().manual_seed(size + pitch_pad + pinned)
    slab[:k, :size] = torch.randint(0, 256, (k, size), dtype=torch.uint8, generator=g)
    rows = [slab[i] for i in range(k + m)]
    ec.jerasure.jerasure_matrix_encode(k, m, 8, M, rows[:k], rows[k:], size)
    hd = alloc_shards(k, size, PAD)
    for j in range(k):
        hd[j][:size] = slab[j, :size].numpy()
    ref = _encode_ref(restatement, k, m, M, hd, size)
    for i in range(m):
        assert np.array_equal(slab[k + i, :size].numpy(), ref[i][:size]), i
    assert not slab[:, size:].any()
    want = slab.clone()
    er = [1, 6, k + 2]
    slab[er, :size] = 0
    assert ec.jerasure.jerasure_matrix_decode(k, m, 8, M, 0, er, rows[:k], rows[k:], size) == 0
    assert torch.equal(slab, want)
    slab[k:] = 0
    assert ec.reed_sol.reed_sol_r6_encode(k, 8, rows[:k], rows[k:k + 2], size) == 1
    ref6 = _encode_ref(restatement, k, 2, ec.reed_sol.reed_sol_r6_coding_matrix(k, 8), hd, size)
    for i in range(2):
        assert np.array_equal(slab[k + i, :size].numpy(), ref6[i][:size]), i
    assert not slab[:, size:].any() and not slab[k + 2:].any()


@pytest.mark.parametrize("zc", [1, 2])
@pytest.mark.parametrize("memory", ["slab_pinned", "shards_pinned", "registered", "pageable", "mixed"])
@pytest.mark.parametrize("size", [(1 << 20) + 3, 4 << 20])
def test_host_pipeline_zero_copy_modes(ec, gpu, restatement, knobs, zc, memory, size):
    """ECGPU_PIPE_ZC (round 6): 1 -- sources by DMA, the kernel writes the
    outputs into the pinned host buffers in place; 2 -- the kernel also reads
    the sources in place (no DMA).  A stripe whose buffers are not all mapped
    host memory (pageable, or a pageable output among pinned ones) takes the
    DMA path in the same pipeline.  Encode against the oracle, nothing written
    past a shard, then a decode pipeline (data, data, parity erased) restores
    every byte."""
    import torch
    knobs.set("pipe_zc", zc)
    k, m, stripes = 10, 4, 5
    pitch = size + PAD
    M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    g = torch.Generator().manual_seed(size + zc)
    if memory == "slab_pinned":
        slab = torch.full((stripes, k + m, pitch), 0x77, dtype=torch.uint8).pin_memory()
        bufs = [[slab[s, j] for j in range(k + m)] for s in range(stripes)]
    else:
        bufs = [[torch.full((pitch,), 0x77, dtype=torch.uint8) for _ in range(k + m)] for _ in range(stripes)]
        for s, st in enumerate(bufs):
            if memory == "shards_pinned" or (memory == "mixed" and s % 2 == 0):
                bufs[s] = [b.pin_memory() for b in st]
            elif memory == "mixed":  # pinned sources, one pageable output: the stripe takes the DMA path
                bufs[s] = [b.pin_memory() for b in st[:k + m - 1]] + [st[-1]]
    for st in bufs:
        for j in range(k):
            st[j][:size] = torch.randint(0, 256, (size,), dtype=torch.uint8, generator=g)
    if memory == "registered":
        for st in bufs:
            for b in st:
                ec.pipeline.host_register(b.numpy())
    try:
        p = ec.HostPipeline(k, m, M, size, depth=3)
        for st in bufs:
            p.submit(st[:k], st[k:])
        p.drain()
        p.close()
        want = [[b.clone() for b in st] for st in bufs]
        for s, st in enumerate(bufs):
            hd = alloc_shards(k, size, PAD)
            for j in range(k):
                hd[j][:size] = st[j][:size].numpy()
            ref = _encode_ref(restatement, k, m, M, hd, size)
            for i in range(m):
                got = st[k + i].numpy()
                assert np.array_equal(got[:size], ref[i][:size]), (s, i)
                assert (got[size:] == 0x77).all(), (s, i)
        er = [1, 6, k + 2]
        for st in bufs:
            for e in er:
                st[e][:size] = 0
        d = ec.HostPipeline.decoder(k, m, M, er, size, depth=2)
        for st in bufs:
            d.submit(st[:k], st[k:])
        d.drain()
        d.close()
        for s in range(stripes):
            for i in range(k + m):
                assert torch.equal(bufs[s][i], want[s][i]), (s, i)
    finally:
        if memory == "registered":
            for st in bufs:
                for b in st:
                    ec.pipeline.host_unregister(b.numpy())


@pytest.mark.parametrize("erasures", [[0], [0, 1, 2, 3], [2, 11], [10, 13], []])
def test_host_pipeline_decoder_matches_reference_decode(ec, gpu, erasures):
    import torch
    k, m, size, stripes = 10, 4, (1 << 20) + 5, 5
    M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    full = []
    for s in range(stripes):
        data = host_shards(41, s, k, size)
        coding = alloc_shards(m, size, PAD)
        ec.jerasure.jerasure_matrix_encode(k, m, 8, M, data, coding, size)
        full.append(data + coding)
    want = [[b.copy() for b in st] for st in full]
    # pinned copies with the erased shards scribbled over
    bufs = [[torch.from_numpy(b).pin_memory() for b in st] for st in full]
    for st in bufs:
        for e in erasures:
            st[e].fill_(0xA5)
    p = ec.HostPipeline.decoder(k, m, M, erasures, size, depth=2)
    for st in bufs:
        p.submit(st[:k], st[k:])
    p.drain()
    p.close()
    for s in range(stripes):
        for i in range(k + m):
            assert np.array_equal(bufs[s][i].numpy()[:size], want[s][i][:size]), (s, i)


def test_host_pipeline_decoder_rejects_undecodable(ec, gpu):
    M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(6, 3, 8)
    with pytest.raises(ec._native.EcgpuError):
        ec.HostPipeline.decoder(6, 3, M, [0, 1, 2, 3], 4096)


# ------------------------------------ multi-device group (one process) ----
# The one-GPU box repeats device 0 in the member list: the round-robin
# ticket mapping, per-member rings and out-of-order waits are what is tested
# here; members on distinct devices differ only in the device ordinal.
@pytest.mark.parametrize("memory", ["pinned", "pageable"])  # pageable: every member's D2H worker
@pytest.mark.parametrize("members", [1, 2, 3])
def test_pipeline_group_encode_round_robin(ec, gpu, restatement, members, memory):
    import torch
    k, m, size, stripes = 10, 4, (1 << 18) + 7, 8
    M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    data = [[torch.from_numpy(b) for b in host_shards(60, s, k, size)] for s in range(stripes)]
    coding = [[torch.zeros(size + PAD, dtype=torch.uint8) for _ in range(m)] for _ in range(stripes)]
    if memory == "pinned":
        data = [[b.pin_memory() for b in st] for st in data]
        coding = [[b.pin_memory() for b in st] for st in coding]
    g = ec.HostPipelineGroup(k, m, M, size, devices=[0] * members, depth=2)
    assert ec._native.lib.ecgpu_pipeline_group_size(g._g) == members
    tickets = [g.submit(data[s], coding[s]) for s in range(stripes)]
    assert tickets == list(range(stripes))
    g.wait(tickets[-1])  # a late member's ticket first, then an early one
    g.wait(tickets[1])
    g.drain()
    with pytest.raises(ec._native.EcgpuError):
        g.wait(stripes)  # never submitted
    g.close()
    for s in range(stripes):
        ref = _encode_ref(restatement, k, m, M, [b.numpy() for b in data[s]], size)
        for i in range(m):
            assert np.array_equal(coding[s][i].numpy()[:size], ref[i][:size]), (s, i)
            assert not coding[s][i].numpy()[size:].any()


@pytest.mark.parametrize("members,depth,nthreads", [(3, 2, 4), (1, 1, 6), (2, 1, 8)])
def test_pipeline_group_concurrent_submitters(ec, gpu, restatement, members, depth, nthreads):
    # per-member submit workers, no group-wide lock: host threads submit
    # interleaved stripes (pageable and pinned) into one group and wait on
    # their own tickets out of order.  More submitters than depth + 1 per
    # member is the shape of the round-2 lost wake-up (a put of
    # exactly the worker's next ticket was never re-signalled)
    import threading

    import torch
    k, m, size, per_thread = 6, 3, (1 << 17) + 3, 5
    M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    g = ec.HostPipelineGroup(k, m, M, size, devices=[0] * members, depth=depth)
    results, errors = {}, []

    def run(tid):
        try:
            mine = []
            for i in range(per_thread):
                s = tid * per_thread + i
                d = host_shards(62, s, k, size)
                c = alloc_shards(m, size, PAD)
                if s % 2:
                    d = [torch.from_numpy(b).pin_memory() for b in d]
                    c = [torch.from_numpy(b).pin_memory() for b in c]
                mine.append((s, g.submit(d, c), d, c))
            for s, t, d, c in reversed(mine):
                g.wait(t)
                results[s] = ([np.asarray(b)[:size].copy() for b in d], [np.asarray(b)[:size].copy() for b in c])
        except Exception as ex:  # reported below
            errors.append(repr(ex))

    ts = [threading.Thread(target=run, args=(i,)) for i in range(nthreads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    g.close()
    assert not errors, errors
    assert sorted(results) == list(range(per_thread * nthreads))
    for s, (d, c) in results.items():
        ref = _encode_ref(restatement, k, m, M, d, size)
        for i in range(m):
            assert np.array_equal(c[i], ref[i][:size]), (s, i)


def test_pipeline_group_decoder(ec, gpu):
    import torch
    k, m, size, stripes = 6, 3, (1 << 16) + 1, 5
    M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    full, want = [], []
    for s in range(stripes):
        d, c = host_shards(61, s, k, size), alloc_shards(m, size, PAD)
        ec.jerasure.jerasure_matrix_encode(k, m, 8, M, d, c, size)
        full.append([torch.from_numpy(b).pin_memory() for b in d + c])
        want.append([b.copy() for b in d + c])
    for st in full:
        for e in (1, 7):
            st[e].fill_(0x5A)
    g = ec.HostPipelineGroup.decoder(k, m, M, [1, 7], size, devices=[0, 0])
    for st in full:
        g.submit(st[:k], st[k:])
    g.drain()
    g.close()
    for s in range(stripes):
        for i in range(k + m):
            assert np.array_equal(full[s][i].numpy()[:size], want[s][i][:size]), (s, i)
    with pytest.raises(ec._native.EcgpuError):
        ec.HostPipelineGroup.decoder(k, m, M, [0, 1, 2, 3], size, devices=[0, 0])


# ------------------------------------------- wide words (w = 16 / 32) ----
def _ref_nsa():
    import ctypes
    import os
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref",
                        "libjerasure_ref_nsa.so")
    if not os.path.exists(path):
        import refcheck
        refcheck.reference_missing("oracle/_ref/libjerasure_ref_nsa.so")
    L = ctypes.CDLL(path)
    I, IP, PP = ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_void_p)
    L._Z22jerasure_matrix_encodeiiiPiPPcS1_i.argtypes = [I, I, I, IP, PP, PP, I]
    L._Z22jerasure_matrix_decodeiiiPiiS_PPcS1_i.argtypes = [I, I, I, IP, I, IP, PP, PP, I]
    return L


def _cints(v):
    import ctypes
    return (ctypes.c_int * len(v))(*v)


def _cptrs(bufs):
    import ctypes
    return (ctypes.c_void_p * len(bufs))(*[b.ctypes.data for b in bufs])


@pytest.mark.parametrize("w", [16, 32])
@pytest.mark.parametrize("size,offset", [(1 << 20, 0), ((1 << 20) + 8, 0), (65536 + 4, 4), (4, 0)])
def test_wide_word_matrix_coding_device(ec, gpu, w, size, offset):
    """w = 16 / 32 encode + decode on device tensors (16-B column kernel,
    word-tail kernel, misaligned base) against the reference library."""
    import torch
    assert size % (w // 8) == 0  # whole words: ragged sizes are the CPU surface's (test_surface_cpu.py)
    ref = _ref_nsa()
    k, m = 6, 3
    M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, w)
    rng = np.random.default_rng(w * 7 + size)
    data = [rng.integers(0, 256, size + 64, dtype=np.uint8) for _ in range(k)]
    coding = [np.zeros(size + 64, np.uint8) for _ in range(m)]
    ref._Z22jerasure_matrix_encodeiiiPiPPcS1_i(k, m, w, _cints(M), _cptrs(data), _cptrs(coding), size)

    def dev(a):
        t = torch.zeros(size + offset + 16, dtype=torch.uint8, device=gpu)
        v = t[offset:offset + size]
        v.copy_(torch.from_numpy(a[:size]))
        return v
    dd = [dev(a) for a in data]
    dc = [torch.full((size + offset + 16,), 0x5A, dtype=torch.uint8, device=gpu)[offset:offset + size]
          for _ in range(m)]
    ec.jerasure.jerasure_matrix_encode(k, m, w, M, dd, dc, size)
    torch.cuda.synchronize()
    for i in range(m):
        assert np.array_equal(dc[i].cpu().numpy(), coding[i][:size]), i
    # decode two data + one parity erasure
    er = [1, 4, k + 2]
    for e in er:
        (dd + dc)[e].fill_(0)
    assert ec.jerasure.jerasure_matrix_decode(k, m, w, M, 0, er, dd, dc, size) == 0
    torch.cuda.synchronize()
    for j in range(k):
        assert np.array_equal(dd[j].cpu().numpy(), data[j][:size]), j
    for i in range(m):
        assert np.array_equal(dc[i].cpu().numpy(), coding[i][:size]), i


@pytest.mark.parametrize("w", [16, 32])
@pytest.mark.parametrize("engine", ["nib", "perm"])
@pytest.mark.parametrize("k,m", [(3, 1), (5, 2), (7, 3), (9, 7), (33, 4), (40, 5)])
def test_wide_word_random_matrix_engines(ec, gpu, knobs, w, engine, k, m):
    """Random w = 16 / 32 coding matrices (zeros, units and general
    coefficients) through both column engines -- LDS nibble tables
    (gf_apply_wide_nib; k = 33 / 40 with 4 rows exceed its LDS budget and
    take v_perm) and v_perm (ECGPU_WIDE=1) -- against the reference library.
    1..4 rows per launch and a second launch for m > 4."""
    import torch
    if engine == "perm":
        knobs.set("ECGPU_WIDE", "1")
    else:
        knobs.reset("ECGPU_WIDE")
    ref = _ref_nsa()
    rng = np.random.default_rng(1000 * w + 10 * k + m)
    hi = (1 << w) - 1
    M = [int(x) for x in rng.integers(0, hi, k * m, dtype=np.uint64, endpoint=True)]
    for i in rng.choice(k * m, size=(k * m) // 4, replace=False):
        M[int(i)] = int(rng.integers(0, 2))  # zeros and units mixed in
    size = (1 << 16) + 48 + (w // 8)  # whole 16-B columns + a word tail
    data = [rng.integers(0, 256, size + 64, dtype=np.uint8) for _ in range(k)]
    coding = [np.zeros(size + 64, np.uint8) for _ in range(m)]
    ref._Z22jerasure_matrix_encodeiiiPiPPcS1_i(k, m, w, _cints([x if x < 2**31 else x - 2**32 for x in M]),
                                              _cptrs(data), _cptrs(coding), size)
    dd = [torch.from_numpy(a[:size].copy()).to(gpu) for a in data]
    dc = [torch.full((size,), 0x5A, dtype=torch.uint8, device=gpu) for _ in range(m)]
    ec.jerasure.jerasure_matrix_encode(k, m, w, [x if x < 2**31 else x - 2**32 for x in M], dd, dc, size)
    torch.cuda.synchronize()
    for i in range(m):
        assert np.array_equal(dc[i].cpu().numpy(), coding[i][:size]), i


@pytest.mark.parametrize("w,nib16,unit_knob", [(32, "1", "ECGPU_WIDE_UNITS"), (16, "0", "ECGPU_WIDE_UNITS"),
                                               (16, "1", "ECGPU_WIDE16_UNITS")])
@pytest.mark.parametrize("units", ["1", "0"])
@pytest.mark.parametrize("k,m", [(10, 4), (6, 2), (5, 3), (32, 4), (12, 6), (2, 2), (7, 3)])
def test_wide_word_unit_structured_launches(ec, gpu, knobs, w, nib16, unit_knob, units, k, m):
    """Launches whose row 0 and column 0 are all ones (every Vandermonde
    encode) run the unit forms gf_apply_wide_nib<R, 1> (w = 32, and w = 16
    with 32-bit entries) and gf_apply_wide_nib16<R, 1> (w = 16 packed pairs):
    row 0 and source 0 by XOR, the other rows of sources 1..K-1 from LDS
    (R = 2, 3, 4; m = 6 is a unit launch of rows 0-3 plus a general launch of
    rows 4-5).  Random general coefficients with zeros and units mixed in,
    against the reference library, with the unit form on and off."""
    import torch
    knobs.reset("ECGPU_WIDE")
    knobs.set("ECGPU_NIB16", nib16)
    knobs.set(unit_knob, units)
    ref = _ref_nsa()
    rng = np.random.default_rng(77 * w + 10 * k + m)
    hi = (1 << w) - 1
    M = [int(x) for x in rng.integers(2, hi, k * m, dtype=np.uint64, endpoint=True)]
    for i in rng.choice(k * m, size=(k * m) // 5, replace=False):
        M[int(i)] = int(rng.integers(0, 2))
    for j in range(k):
        M[j] = 1  # row 0
    for i in range(m):
        M[i * k] = 1  # column 0
    Mi = [x if x < 2**31 else x - 2**32 for x in M]
    size = (1 << 18) + 32 + (w // 8)
    data = [rng.integers(0, 256, size + 64, dtype=np.uint8) for _ in range(k)]
    coding = [np.zeros(size + 64, np.uint8) for _ in range(m)]
    ref._Z22jerasure_matrix_encodeiiiPiPPcS1_i(k, m, w, _cints(Mi), _cptrs(data), _cptrs(coding), size)
    dd = [torch.from_numpy(a[:size].copy()).to(gpu) for a in data]
    dc = [torch.full((size,), 0x5A, dtype=torch.uint8, device=gpu) for _ in range(m)]
    ec.jerasure.jerasure_matrix_encode(k, m, w, Mi, dd, dc, size)
    torch.cuda.synchronize()
    for i in range(m):
        assert np.array_equal(dc[i].cpu().numpy(), coding[i][:size]), i


_PIPE_SHAPES = [(1, 1), (2, 2), (3, 4), (4, 1), (5, 3), (6, 4), (7, 2), (8, 3), (9, 2), (10, 4), (11, 4), (12, 4),
                (13, 3), (14, 2), (15, 3), (16, 4), (10, 6)]


# every shape at 3 column blocks; the column loop run many times (1600
# blocks) on three shapes -- explicit lists, so no test ID exists only to skip
_PIPE_CASES = [(k, m, 3) for k, m in _PIPE_SHAPES] + [(k, m, 1600) for k, m in ((10, 4), (12, 4), (16, 4), (5, 3))]


@pytest.mark.parametrize("w", [16, 32])
@pytest.mark.parametrize("structure", ["vandermonde", "random"])
@pytest.mark.parametrize("k,m,blocks", _PIPE_CASES)
@pytest.mark.parametrize("pipe", ["2", "1"])
def test_wide_word_pipelined_launches(ec, gpu, knobs, w, structure, k, m, blocks, pipe):
    """Launches of whole 256-column blocks (4 KiB per shard each) run
    gf_apply_wide_pipe<K, R, mode> -- compile-time K, double-buffered source
    chunks, all three modes (w = 32 unit structure, w = 32 general, w = 16
    packed pairs), R = 1..4 and K = 1..16 (every chunk split: 1 + 0, 2 + 2 +
    2 + 1 ...; m = 6: a unit launch plus a general one), here plus a word tail.
    1600 blocks run the workgroups' column loop more than once (the grid is
    one resident round).  Encode and a decode of up to m erasures against the
    reference library."""
    import torch
    knobs.reset("ECGPU_WIDE")
    knobs.reset("ECGPU_NIB16")
    knobs.reset("ECGPU_WIDE_UNITS")
    knobs.set("ECGPU_WIDE_PIPE", pipe)
    ref = _ref_nsa()
    rng = np.random.default_rng(31 * w + 7 * k + m + blocks)
    if structure == "vandermonde":
        M = list(ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, w))
    else:
        hi = (1 << w) - 1
        M = [int(x) for x in rng.integers(0, hi, k * m, dtype=np.uint64, endpoint=True)]
        for i in rng.choice(k * m, size=(k * m) // 4, replace=False):
            M[int(i)] = int(rng.integers(0, 2))
        M = [x if x < 2**31 else x - 2**32 for x in M]
    size = 4096 * blocks + 2 * (w // 8)  # whole column blocks + a word tail
    data = [rng.integers(0, 256, size + 64, dtype=np.uint8) for _ in range(k)]
    coding = [np.zeros(size + 64, np.uint8) for _ in range(m)]
    ref._Z22jerasure_matrix_encodeiiiPiPPcS1_i(k, m, w, _cints(M), _cptrs(data), _cptrs(coding), size)
    dd = [torch.from_numpy(a[:size].copy()).to(gpu) for a in data]
    dc = [torch.full((size,), 0x5A, dtype=torch.uint8, device=gpu) for _ in range(m)]
    ec.jerasure.jerasure_matrix_encode(k, m, w, M, dd, dc, size)
    torch.cuda.synchronize()
    for i in range(m):
        assert np.array_equal(dc[i].cpu().numpy(), coding[i][:size]), i
    if structure != "vandermonde":
        return  # random matrices need not be MDS
    er = sorted(int(x) for x in rng.choice(k + m, size=min(m, k + m - 1), replace=False))
    for e in er:
        (dd + dc)[e].fill_(0)
    assert ec.jerasure.jerasure_matrix_decode(k, m, w, M, 0, er, dd, dc, size) == 0
    torch.cuda.synchronize()
    for j in range(k):
        assert np.array_equal(dd[j].cpu().numpy(), data[j][:size]), j
    for i in range(m):
        assert np.array_equal(dc[i].cpu().numpy(), coding[i][:size]), i


@pytest.mark.parametrize("w", [16, 32])
def test_wide_word_region_ops_device(ec, gpu, w):
    import torch
    size = 8192 + 8
    rng = np.random.default_rng(w)
    src = rng.integers(0, 256, size, dtype=np.uint8)
    dst = rng.integers(0, 256, size, dtype=np.uint8)
    mulfn = ec.galois.galois_w16_region_multiply if w == 16 else ec.galois.galois_w32_region_multiply
    W = w // 8
    c = 0xBEEF if w == 16 else 0x12345678
    sw = src.view(np.uint16 if w == 16 else np.uint32)
    dw = dst.view(np.uint16 if w == 16 else np.uint32)
    prod = np.array([ec.galois.galois_single_multiply(int(x), c, w) & 0xFFFFFFFF for x in sw], dtype=sw.dtype)
    ts, td = torch.from_numpy(src).to(gpu), torch.from_numpy(dst).to(gpu)
    mulfn(ts, c, size, td, 1)
    torch.cuda.synchronize()
    assert np.array_equal(td.cpu().numpy().view(dw.dtype), dw ^ prod)
    mulfn(ts, c, size, td, 0)
    torch.cuda.synchronize()
    assert np.array_equal(td.cpu().numpy().view(dw.dtype), prod)
    by2 = ec.reed_sol.reed_sol_galois_w16_region_multby_2 if w == 16 else ec.reed_sol.reed_sol_galois_w32_region_multby_2
    by2(ts, size)
    torch.cuda.synchronize()
    two = np.array([ec.galois.galois_single_multiply(int(x), 2, w) & 0xFFFFFFFF for x in sw], dtype=sw.dtype)
    assert np.array_equal(ts.cpu().numpy().view(sw.dtype), two)
    assert W in (2, 4)


# ------------------------------------------ GF(2) bit-matrix / schedules ----
def _np_bitmatrix_encode(k, m, w, bm, data, size, ps, init=None):
    """Plain numpy restatement of jerasure_bitmatrix_encode (jerasure.cpp:301-345):
    an output packet whose bit-matrix row is all zero is left as it was
    (`init`, zeros by default) -- the reference only memcpy's / XORs."""
    out = [np.zeros(size, np.uint8) if init is None else init[i].copy() for i in range(m)]
    for i in range(m):
        for sp in range(0, size, w * ps):
            for j in range(w):
                acc = None
                row = bm[(i * w + j) * k * w:(i * w + j + 1) * k * w]
                for x in range(k):
                    for y in range(w):
                        if row[x * w + y]:
                            src = data[x][sp + y * ps:sp + (y + 1) * ps]
                            acc = src.copy() if acc is None else acc ^ src
                if acc is not None:
                    out[i][sp + j * ps:sp + (j + 1) * ps] = acc
    return out


@pytest.mark.parametrize("k,m,w,ps", [(10, 4, 8, 2048), (6, 5, 8, 512), (4, 2, 16, 256)])
def test_bitmatrix_coding_device(ec, gpu, k, m, w, ps):
    """Device tensors through the Python mirror: bit-matrix encode (>32 output
    packet rows for m=5: two launches), dumb-schedule encode, and decode."""
    import torch
    J = ec.jerasure
    M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, w)
    bm = J.jerasure_matrix_to_bitmatrix(k, m, w, M)
    size = w * ps * 6
    rng = np.random.default_rng(k * 1000 + ps)
    data = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(k)]
    want = _np_bitmatrix_encode(k, m, w, bm, data, size, ps)
    dd = [torch.from_numpy(a).to(gpu) for a in data]
    dc = [torch.zeros(size, dtype=torch.uint8, device=gpu) for _ in range(m)]
    J.jerasure_bitmatrix_encode(k, m, w, bm, dd, dc, size, ps)
    torch.cuda.synchronize()
    for i in range(m):
        assert np.array_equal(dc[i].cpu().numpy(), want[i]), i
    dc2 = [torch.zeros(size, dtype=torch.uint8, device=gpu) for _ in range(m)]
    J.jerasure_schedule_encode(k, m, w, J.jerasure_dumb_bitmatrix_to_schedule(k, m, w, bm), dd, dc2, size, ps)
    torch.cuda.synchronize()
    for i in range(m):
        assert torch.equal(dc[i], dc2[i]), i
    er = [0, k - 1, k + m - 1][: m]
    for e in er:
        (dd + dc)[e].fill_(0x33)
    assert J.jerasure_bitmatrix_decode(k, m, w, bm, 1, er, dd, dc, size, ps) == 0
    torch.cuda.synchronize()
    for j in range(k):
        assert np.array_equal(dd[j].cpu().numpy(), data[j]), j
    for i in range(m):
        assert np.array_equal(dc[i].cpu().numpy(), want[i]), i


@pytest.mark.parametrize("kind", ["0", "3"])  # ECGPU_PACKET: unit form where the map allows, general 16-B kernel
@pytest.mark.parametrize("k", [1, 2, 6, 10, 12])
def test_vandermonde_bitmatrix_unit_form(ec, gpu, knobs, kind, k):
    """The w = 8 Vandermonde bit-matrix encode of RS(k,4): the unit-structure
    packet kernel (identity blocks of coding device 0 and data device 0 as
    plain XORs) and the general kernel, against the numpy restatement."""
    import torch
    knobs.set("ECGPU_PACKET", kind)
    m, w, ps = 4, 8, 1024
    J = ec.jerasure
    bm = J.jerasure_matrix_to_bitmatrix(k, m, w, ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, w))
    size = w * ps * 5
    rng = np.random.default_rng(700 + k)
    data = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(k)]
    want = _np_bitmatrix_encode(k, m, w, bm, data, size, ps)
    dd = [torch.from_numpy(a).to(gpu) for a in data]
    dc = [torch.full((size,), 0x5A, dtype=torch.uint8, device=gpu) for _ in range(m)]
    J.jerasure_bitmatrix_encode(k, m, w, bm, dd, dc, size, ps)
    torch.cuda.synchronize()
    for i in range(m):
        assert np.array_equal(dc[i].cpu().numpy(), want[i]), i


@pytest.mark.parametrize("kind", ["0", "1", "2", "3"])  # ECGPU_PACKET: production, 8-B lanes, unpipelined 16-B,
#                                                         general pipelined 16-B
@pytest.mark.parametrize("k,m,w,ps", [(1, 1, 3, 64), (5, 2, 3, 128), (3, 2, 5, 16), (10, 4, 8, 2048),
                                      (7, 5, 2, 48), (4, 3, 3, 8), (3, 3, 3, 5)])
def test_random_bitmatrix_packet_kernels(ec, gpu, knobs, kind, k, m, w, ps):
    """A random 0/1 bit-matrix (any w) through jerasure_bitmatrix_encode on
    every packet kernel: source-row counts below one pipelined chunk of four
    (k*w = 3), with a ragged tail (15), and whole chunks (80); 16-B, 8-B and
    byte packets; more than 8 / 16 output rows; all-zero rows leave their
    output packets untouched, as the reference does."""
    import torch
    knobs.set("ECGPU_PACKET", kind)
    rng = np.random.default_rng(k * 131 + m * 17 + w * 5 + ps)
    bm = [int(b) for b in rng.integers(0, 2, k * w * m * w)]
    size = w * ps * 7
    data = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(k)]
    init = [np.full(size, 0x5A, np.uint8) for _ in range(m)]
    want = _np_bitmatrix_encode(k, m, w, bm, data, size, ps, init)
    dd = [torch.from_numpy(a).to(gpu) for a in data]
    dc = [torch.from_numpy(a).to(gpu) for a in init]
    ec.jerasure.jerasure_bitmatrix_encode(k, m, w, bm, dd, dc, size, ps)
    torch.cuda.synchronize()
    for i in range(m):
        assert np.array_equal(dc[i].cpu().numpy(), want[i]), i


def test_scheduled_operations_accumulate_many_rows(ec, gpu):
    """XOR-into-destination ops (the destination's old content is a source)
    over 40 output packets: more rows than one launch, outputs via temps."""
    ps, npk = 64, 40
    rng = np.random.default_rng(3)
    a = rng.integers(0, 256, npk * ps, dtype=np.uint8)
    b = rng.integers(0, 256, npk * ps, dtype=np.uint8)
    ops = [(0, p, 1, p, 1) for p in range(npk)] + [(1, p, 1, (p + 1) % npk, 1) for p in range(npk)]
    want_b = b.copy().reshape(npk, ps)
    av = a.reshape(npk, ps)
    for p in range(npk):
        want_b[p] ^= av[p]
    for p in range(npk):
        want_b[(p + 1) % npk] ^= want_b[p]
    ec.jerasure.jerasure_do_scheduled_operations([a, b], ops, ps)
    assert np.array_equal(b.reshape(npk, ps), want_b)


# ------------------------------------------------ structured data patterns ----
def _pattern(name, size, shard):
    i = np.arange(size, dtype=np.int64)
    if name == "zeros":
        return np.zeros(size, np.uint8)
    if name == "ones":
        return np.full(size, 0xFF, np.uint8)
    if name == "ramp":
        return ((i + shard) & 0xFF).astype(np.uint8)
    return (1 << ((i + shard) % 8)).astype(np.uint8)  # single set bit per byte


@pytest.mark.parametrize("name", ["zeros", "ones", "ramp", "single_bit"])
@pytest.mark.parametrize("k,m", [(10, 4), (6, 3)])
def test_structured_patterns_encode_decode(ec, gpu, restatement, name, k, m):
    """SURVEY §8d correctness patterns (all-0x00, all-0xFF, ramp, single-bit)
    through the device path, against the oracle restatement, then a decode of
    m erased shards (data and parity mixed) back to the originals."""
    import torch
    size = (1 << 18) + 48
    M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    data = alloc_shards(k, size, PAD)
    for j in range(k):
        data[j][:size] = _pattern(name, size, j)
    want = _encode_ref(restatement, k, m, M, data, size)
    dd = to_dev(data, gpu)
    dc = to_dev(alloc_shards(m, size, PAD), gpu)
    ec.jerasure.jerasure_matrix_encode(k, m, 8, M, dd, dc, size)
    torch.cuda.synchronize()
    got = to_host(dc)
    for i in range(m):
        assert np.array_equal(got[i][:size], want[i][:size]), i
    er = [0, k - 1] + [k + i for i in range(m - 2)]
    for e in er:
        (dd + dc)[e].fill_(0x5C)
    assert ec.jerasure.jerasure_matrix_decode(k, m, 8, M, 0, er, dd, dc, size) == 0
    torch.cuda.synchronize()
    for j, t in enumerate(to_host(dd)):
        assert np.array_equal(t[:size], data[j][:size]), j
    for i, t in enumerate(to_host(dc)):
        assert np.array_equal(t[:size], want[i][:size]), i


@pytest.mark.parametrize("depth", [1, 4])
def test_host_pipeline_depth_and_row_k_ones(ec, gpu, restatement, depth):
    """Ring depth 1 (every submit waits for the previous stripe) and 4, and
    the decoder's row_k_ones=1 shortcut (jerasure.cpp:232-239)."""
    k, m, size, stripes = 6, 3, 65536 + 16, 5
    M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    data = [host_shards(42, s, k, size) for s in range(stripes)]
    coding = [alloc_shards(m, size, PAD) for _ in range(stripes)]
    p = ec.HostPipeline(k, m, M, size, depth=depth)
    for s in range(stripes):
        p.submit(data[s], coding[s])
    p.drain()
    p.close()
    for s in range(stripes):
        ref = _encode_ref(restatement, k, m, M, data[s], size)
        for i in range(m):
            assert np.array_equal(coding[s][i][:size], ref[i][:size]), (s, i)
    saved = [d[3].copy() for d in data]
    for d in data:
        d[3][:] = 0
    rd = ec.HostPipeline.decoder(k, m, M, [3], size, row_k_ones=1, depth=depth)
    for s in range(stripes):
        rd.submit(data[s], coding[s])
    rd.drain()
    rd.close()
    for s in range(stripes):
        assert np.array_equal(data[s][3][:size], saved[s][:size]), s


@pytest.mark.parametrize("smart", [0, 1])
def test_schedule_decode_lazy_and_cache_device(ec, gpu, smart):
    """Scheduled decoding through the Python mirror on device tensors: lazy
    (any erasure set) and the m=2 schedule cache, against the originals."""
    import torch
    J = ec.jerasure
    k, m, w, ps = 6, 2, 8, 512
    M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, w)
    bm = J.jerasure_matrix_to_bitmatrix(k, m, w, M)
    size = w * ps * 5
    rng = np.random.default_rng(7 + smart)
    data = [torch.from_numpy(rng.integers(0, 256, size, dtype=np.uint8)).to(gpu) for _ in range(k)]
    coding = [torch.zeros(size, dtype=torch.uint8, device=gpu) for _ in range(m)]
    J.jerasure_schedule_encode(k, m, w, J.jerasure_smart_bitmatrix_to_schedule(k, m, w, bm), data, coding, size, ps)
    orig = [t.clone() for t in data + coding]
    cache = J.jerasure_generate_schedule_cache(k, m, w, bm, smart)
    for er in ([0], [k], [1, 4], [2, k + 1], [k, k + 1]):
        for method in ("lazy", "cache"):
            for e in er:
                (data + coding)[e].fill_(0xEE)
            if method == "lazy":
                assert J.jerasure_schedule_decode_lazy(k, m, w, bm, er, data, coding, size, ps, smart) == 0
            else:
                assert J.jerasure_schedule_decode_cache(k, m, w, cache, er, data, coding, size, ps) == 0
            torch.cuda.synchronize()
            for i, t in enumerate(data + coding):
                assert torch.equal(t, orig[i]), (er, method, i)
    assert J.jerasure_schedule_decode_cache(k, m, w, cache, [0, 1, 2], data, coding, size, ps) == -1
    J.jerasure_free_schedule_cache(k, m, cache)


# ------------------------------------------- randomized (seeded) cases ----
# Arbitrary fused maps through the batched plan API, checked against the
# reference's own 256 x 256 product table (tests/golden vectors.npz): random
# source counts (1..20, so both the specialised K <= 16 kernels and the
# generic one), 1..7 output rows (several launches), densities of zero /
# unit / general coefficients, ragged sizes, 0..15-byte misaligned buffers.
def _random_map_case(seed):
    rng = np.random.default_rng(7000 + seed)
    K, R, stripes = int(rng.integers(1, 21)), int(rng.integers(1, 8)), int(rng.integers(1, 4))
    size = int(rng.choice([1, 15, 16, 17, 4096, (1 << 16) + 48, int(rng.integers(1, 200_000))]))
    kind = rng.choice(3, size=(R, K), p=[0.15, 0.25, 0.6])
    coefs = np.where(kind == 0, 0, np.where(kind == 1, 1, rng.integers(2, 256, size=(R, K))))
    offs = rng.integers(0, 16, size=(stripes, K + R)) if seed % 3 == 0 else np.zeros((stripes, K + R), np.int64)
    return rng, K, R, stripes, size, coefs.astype(np.int64), offs


@pytest.mark.parametrize("seed", range(40))
def test_random_fused_maps_vs_reference_table(ec, gpu, vectors, seed):
    import torch
    T = vectors["gf_mul_table"].reshape(256, 256)
    rng, K, R, stripes, size, coefs, offs = _random_map_case(seed)
    host_src = [[rng.integers(0, 256, size, dtype=np.uint8) for _ in range(K)] for _ in range(stripes)]
    bufs, srcs, dsts = [], [], []
    for s in range(stripes):
        row_s, row_d = [], []
        for j in range(K + R):
            o = int(offs[s, j])
            b = torch.full((o + size + PAD,), 0xCC, dtype=torch.uint8, device=gpu)
            bufs.append(b)
            v = b[o:o + size]
            if j < K:
                v.copy_(torch.from_numpy(host_src[s][j]))
                row_s.append(v)
            else:
                row_d.append(v)
        srcs.append(row_s)
        dsts.append(row_d)
    p = ec.plan.StripePlan(R, K, coefs.ravel().tolist()).bind(srcs, dsts, size)
    p.launch()
    torch.cuda.synchronize()
    for s in range(stripes):
        for r in range(R):
            want = np.zeros(size, np.uint8)
            for j in range(K):
                want ^= T[coefs[r, j]][host_src[s][j]]
            b = bufs[s * (K + R) + K + r].cpu().numpy()
            o = int(offs[s, K + r])
            assert np.array_equal(b[o:o + size], want), (seed, K, R, size, s, r)
            assert (b[:o] == 0xCC).all() and (b[o + size:] == 0xCC).all(), "wrote outside the region"
    p.close()


@pytest.mark.parametrize("where", ["device", "host", "pinned"])
@pytest.mark.parametrize("seed", range(16))
def test_random_fused_maps_sync_calls(ec, gpu, vectors, seed, where):
    """The same random maps through the SYNCHRONOUS surface
    (jerasure_matrix_encode with an arbitrary K x R matrix, one stripe):
    the inline-argument launches (K <= 16, one launch per 4 rows, the byte
    path for misaligned buffers), the plan path above 16 sources, and every
    host staging mode (zero-copy, bounce, HIP copies; pinned in place).  An
    all-zero row leaves its destination untouched (jerasure.cpp:561-620)."""
    import torch
    T = vectors["gf_mul_table"].reshape(256, 256)
    rng, K, R, _, size, coefs, offs = _random_map_case(seed)
    src = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(K)]
    bases, views = [], []
    for j in range(K + R):
        o = int(offs[0, j])
        if where == "device":
            b = torch.full((o + size + PAD,), 0xCC, dtype=torch.uint8, device=gpu)
        else:
            b = torch.full((o + size + PAD,), 0xCC, dtype=torch.uint8)
            if where == "pinned":
                b = b.pin_memory()
        v = b[o:o + size]
        if j < K:
            v.copy_(torch.from_numpy(src[j]))
        bases.append(b)
        views.append(v if where != "host" else v.numpy())
    ec.jerasure.jerasure_matrix_encode(K, R, 8, coefs.ravel().tolist(), views[:K], views[K:], size)
    for r in range(R):
        b = bases[K + r].cpu().numpy()
        o = int(offs[0, K + r])
        if not coefs[r].any():
            want = np.full(size, 0xCC, np.uint8)
        else:
            want = np.zeros(size, np.uint8)
            for j in range(K):
                want ^= T[coefs[r, j]][src[j]]
        assert np.array_equal(b[o:o + size], want), (seed, where, K, R, size, r)
        assert (b[:o] == 0xCC).all() and (b[o + size:] == 0xCC).all(), "wrote outside the region"
    for j in range(K):  # sources untouched
        assert np.array_equal(bases[j].cpu().numpy()[int(offs[0, j]):int(offs[0, j]) + size], src[j])


# jerasure_matrix_decode on random (k, m, erasures, row_k_ones) against the
# reference library compiled from /root/reference (oracle/_ref): decoded
# bytes must equal the reference decode on the same inputs, and the return
# code must match (including undecodable patterns).
@pytest.mark.parametrize("seed", range(24))
def test_random_decode_vs_reference(ec, gpu, reference, seed):
    rng = np.random.default_rng(9000 + seed)
    k, m = int(rng.integers(2, 15)), int(rng.integers(1, 7))
    size = 8 * int(rng.integers(1, 8192))  # whole 8-byte words: the reference's loops over-run otherwise
    M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    ne = int(rng.integers(1, m + 2))  # up to m + 1 erasures: the last may be undecodable
    erasures = sorted(int(x) for x in rng.choice(k + m, size=min(ne, k + m), replace=False))
    row_k_ones = int(rng.integers(0, 2))
    data = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(k)]
    coding = [np.zeros(size, np.uint8) for _ in range(m)]
    reference.matrix_encode(k, m, np.array(M).reshape(m, k), data, coding, size)
    for e in erasures:  # scribble over the erased shards
        (data + coding)[e][:] = rng.integers(0, 256, size, dtype=np.uint8)
    ref_bufs = [b.copy() for b in data + coding]
    got_bufs = [b.copy() for b in data + coding]
    rc_ref = reference.matrix_decode(k, m, np.array(M).reshape(m, k), row_k_ones, erasures, ref_bufs[:k],
                                     ref_bufs[k:], size)
    rc_got = ec.jerasure.jerasure_matrix_decode(k, m, 8, M, row_k_ones, erasures, got_bufs[:k], got_bufs[k:], size)
    assert rc_got == rc_ref, (k, m, erasures, row_k_ones)
    for i in range(k + m):
        assert np.array_equal(got_bufs[i], ref_bufs[i]), (k, m, erasures, row_k_ones, i)


# ------------------------------------------------ size edge cases ----
def test_empty_regions_touch_nothing(ec, gpu):
    """size 0 (the reference's loops run zero times): outputs keep their bytes,
    decode still reports success for a decodable pattern."""
    import torch
    k, m = 4, 2
    M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    dd = [torch.full((64,), 7 * i + 1, dtype=torch.uint8, device=gpu) for i in range(k)]
    dc = [torch.full((64,), 0x5A, dtype=torch.uint8, device=gpu) for _ in range(m)]
    ec.jerasure.jerasure_matrix_encode(k, m, 8, M, dd, dc, 0)
    assert ec.jerasure.jerasure_matrix_decode(k, m, 8, M, 0, [0, k], dd, dc, 0) == 0
    torch.cuda.synchronize()
    assert all(bool((c == 0x5A).all()) for c in dc)
    assert all(bool((d == 7 * i + 1).all()) for i, d in enumerate(dd))


@pytest.mark.parametrize("k,m,erasures", [(2, 1, [0]), (3, 2, [0, 2])])
def test_maximum_int_size_roundtrip(ec, gpu, k, m, erasures):
    """Shards of 2^31 - 1 bytes, the largest `int size` the reference API
    takes (134M 16-B columns plus a 15-byte tail): encode -> erase -> decode
    restores the data bit-exactly; for RS(k,1) the parity row is all ones, so
    it must equal the XOR of the data (computed by torch, independent of the
    library's kernels)."""
    import torch
    size = 2**31 - 1
    M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    g = torch.Generator(device=gpu).manual_seed(k * 10 + m)
    dd = [torch.randint(0, 256, (size,), dtype=torch.uint8, device=gpu, generator=g) for _ in range(k)]
    dc = [torch.empty(size, dtype=torch.uint8, device=gpu) for _ in range(m)]
    ec.jerasure.jerasure_matrix_encode(k, m, 8, M, dd, dc, size)
    torch.cuda.synchronize()
    if m == 1:
        x = dd[0].clone()
        for d in dd[1:]:
            x.bitwise_xor_(d)
        assert torch.equal(x, dc[0])
        del x
    keep = {e: (dd + dc)[e].clone() for e in erasures}
    for e in erasures:
        (dd + dc)[e].fill_(0)
    torch.cuda.synchronize()
    assert ec.jerasure.jerasure_matrix_decode(k, m, 8, M, 0, erasures, dd, dc, size) == 0
    torch.cuda.synchronize()
    for e, want in keep.items():
        assert torch.equal((dd + dc)[e], want), e


@pytest.mark.parametrize("w", [16, 32])
def test_maximum_int_size_wide_words(ec, gpu, w):
    """w = 16 / 32 at the largest `int size` the word size allows (2^31 - 4:
    134M 16-B columns through the LDS nibble kernels plus a 12-byte tail):
    RS(2,1)'s parity row is all ones, so the parity must equal the torch XOR
    of the data; then RS(2,1) decode of data shard 0 restores it."""
    import torch
    k, m, size = 2, 1, 2**31 - 4
    M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, w)
    g = torch.Generator(device=gpu).manual_seed(w)
    dd = [torch.randint(0, 256, (size,), dtype=torch.uint8, device=gpu, generator=g) for _ in range(k)]
    dc = [torch.empty(size, dtype=torch.uint8, device=gpu)]
    ec.jerasure.jerasure_matrix_encode(k, m, w, M, dd, dc, size)
    torch.cuda.synchronize()
    assert torch.equal(torch.bitwise_xor(dd[0], dd[1]), dc[0])
    keep = dd[0].clone()
    dd[0].fill_(0)
    assert ec.jerasure.jerasure_matrix_decode(k, m, w, M, 0, [0], dd, dc, size) == 0
    torch.cuda.synchronize()
    assert torch.equal(dd[0], keep)


def test_maximum_int_size_bitmatrix(ec, gpu):
    """Bit-matrix packet coding at the largest `int size` that is whole
    super-packets for w = 8, packetsize 8 KiB (2^31 - 64 KiB; 16.8M packet
    columns of 16 B): RS(2,1)'s bit-matrix is two identity blocks, so every
    parity packet row is the XOR of the data rows -- the torch XOR of the
    shards -- and the bit-matrix decode of data shard 0 restores it."""
    import torch
    k, m, w, ps = 2, 1, 8, 8192
    size = 2**31 - w * ps
    J = ec.jerasure
    bm = J.jerasure_matrix_to_bitmatrix(k, m, w, ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, w))
    g = torch.Generator(device=gpu).manual_seed(3)
    dd = [torch.randint(0, 256, (size,), dtype=torch.uint8, device=gpu, generator=g) for _ in range(k)]
    dc = [torch.empty(size, dtype=torch.uint8, device=gpu)]
    J.jerasure_bitmatrix_encode(k, m, w, bm, dd, dc, size, ps)
    torch.cuda.synchronize()
    assert torch.equal(torch.bitwise_xor(dd[0], dd[1]), dc[0])
    keep = dd[0].clone()
    dd[0].fill_(0)
    assert J.jerasure_bitmatrix_decode(k, m, w, bm, 0, [0], dd, dc, size, ps) == 0
    torch.cuda.synchronize()
    assert torch.equal(dd[0], keep)


@pytest.mark.parametrize("k", [15, 16])
@pytest.mark.parametrize("size", [(1 << 20) - 48, (2 << 20) + 16])
def test_dense_wide_k_calls_inline_or_plan(ec, gpu, restatement, k, size):
    """Calls with 15-16 sources and 4+ dense rows run inline up to 1 MiB and
    as a plan launch above (inline_ok: those inline kernels spill their
    tables); both sides of the switch, device buffers and pageable host
    buffers, against the oracle."""
    import torch
    m = 5  # a full 4-row launch plus one more
    rng = np.random.default_rng(k * 1000 + size % 997)
    M = [int(x) for x in rng.integers(2, 256, k * m)]
    data = host_shards(80, k, k, size)
    ref = _encode_ref(restatement, k, m, M, data, size)
    dd = to_dev([d[:size] for d in data], gpu)
    dc = [torch.zeros(size, dtype=torch.uint8, device=gpu) for _ in range(m)]
    ec.jerasure.jerasure_matrix_encode(k, m, 8, M, dd, dc, size)
    torch.cuda.synchronize()
    for i in range(m):
        assert np.array_equal(dc[i].cpu().numpy(), ref[i][:size]), i
    hc = alloc_shards(m, size, PAD)
    ec.jerasure.jerasure_matrix_encode(k, m, 8, M, data, hc, size)
    for i in range(m):
        assert np.array_equal(hc[i][:size], ref[i][:size]), i
