"""Split synchronous calls (ECGPU_SPLIT, csrc/ecgpu_runtime.hip execute_split):
a host-memory call cut into 16-B-aligned byte ranges run concurrently, each
on its own context and device (on this one-GPU box: N contexts on cuda:0).

Byte columns are independent, so a split call must give exactly the bytes of
the whole call: w = 8 encode / decode against the oracle on pageable and
pinned host slabs with ragged sizes; w = 16 / 32 region multiplies and an
aliased region XOR against the same call unsplit; the byte counters counted
once; device-buffer calls untouched by the knob.
"""
import numpy as np
import pytest

from oracle.oracle import alloc_shards

pytestmark = pytest.mark.gpu

PAD = 16


@pytest.fixture(scope="module")
def ec(gpu):
    import erasure_coding_test_amd as E
    return E


@pytest.fixture
def split(knobs):
    def on(ways, min_kib=64):
        knobs.set("ECGPU_SPLIT", ways)
        knobs.set("ECGPU_SPLIT_MIN_KIB", min_kib)
    return on


def _slab(k, m, size, pinned, seed):
    import torch
    slab = torch.zeros((k + m, size + 4099), dtype=torch.uint8)
    if pinned:
        slab = slab.pin_memory()
    g = torch.Generator().manual_seed(seed)
    slab[:k, :size] = torch.randint(0, 256, (k, size), dtype=torch.uint8, generator=g)
    return slab


@pytest.mark.parametrize("ways", [2, 3, 8])
@pytest.mark.parametrize("size", [(1 << 20) + 13, (3 << 20) + 48, 700001])
@pytest.mark.parametrize("pinned", [False, True])
def test_split_encode_decode_match_reference(ec, gpu, restatement, split, ways, size, pinned):
    import torch
    k, m = 10, 4
    M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    slab = _slab(k, m, size, pinned, size + ways)
    rows = [slab[i] for i in range(k + m)]
    split(ways)
    ec.jerasure.jerasure_matrix_encode(k, m, 8, M, rows[:k], rows[k:], size)
    hd = alloc_shards(k, size, PAD)
    for j in range(k):
        hd[j][:size] = slab[j, :size].numpy()
    ref = alloc_shards(m, size, PAD)
    restatement.matrix_encode(k, m, np.array(M).reshape(m, k), hd, ref, size)
    for i in range(m):
        assert np.array_equal(slab[k + i, :size].numpy(), ref[i][:size]), i
    assert not slab[:, size:].any()  # nothing past any shard
    want = slab.clone()
    er = [1, 6, k + 2]
    slab[er, :size] = 0
    assert ec.jerasure.jerasure_matrix_decode(k, m, 8, M, 0, er, rows[:k], rows[k:], size) == 0
    assert torch.equal(slab, want)


@pytest.mark.parametrize("w", [8, 16, 32])
def test_split_region_ops_equal_whole_calls(ec, gpu, split, knobs, w):
    size = (2 << 20) + 24  # a whole number of words at every w, not of 16-B ranges
    rng = np.random.default_rng(w)
    src = rng.integers(0, 256, size + PAD, dtype=np.uint8)
    dst0 = rng.integers(0, 256, size + PAD, dtype=np.uint8)
    c = {8: 0x8E, 16: 0xBEEF, 32: 0x1234567}[w]
    mul = {8: ec.galois.galois_w08_region_multiply, 16: ec.galois.galois_w16_region_multiply,
           32: ec.galois.galois_w32_region_multiply}[w]
    outs = []
    for ways in (0, 4):
        knobs.set("ECGPU_SPLIT", ways)
        knobs.set("ECGPU_SPLIT_MIN_KIB", 64)
        d = dst0.copy()
        mul(src, c, size, d, 1)  # d ^= c * src
        a, b = src.copy(), dst0.copy()
        ec.galois.galois_region_xor(a, b, a, size)  # r3 == r1: a ^= b
        outs.append((d, a))
    assert np.array_equal(outs[0][0], outs[1][0])
    assert np.array_equal(outs[0][1], outs[1][1])
    assert np.array_equal(outs[1][0][size:], dst0[size:])  # tail untouched


def test_split_counts_bytes_once(ec, gpu, split):
    k, m, size = 6, 3, (2 << 20) + 7
    M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    data = [np.random.default_rng(j).integers(0, 256, size + PAD, dtype=np.uint8) for j in range(k)]
    coding = alloc_shards(m, size, PAD)
    ec.jerasure.jerasure_get_stats()  # reset
    ec.jerasure.jerasure_matrix_encode(k, m, 8, M, data, coding, size)
    whole = ec.jerasure.jerasure_get_stats()
    split(4)
    ec.jerasure.jerasure_matrix_encode(k, m, 8, M, data, coding, size)
    assert ec.jerasure.jerasure_get_stats() == whole


def test_split_leaves_device_calls_whole(ec, gpu, restatement, split):
    import torch
    k, m, size = 10, 4, (1 << 20) + 3
    M = ec.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    hd = alloc_shards(k, size, PAD)
    for j in range(k):
        hd[j][:size] = np.random.default_rng(100 + j).integers(0, 256, size, dtype=np.uint8)
    data = [torch.from_numpy(h).to(gpu) for h in hd]
    coding = [torch.zeros(size + PAD, dtype=torch.uint8, device=gpu) for _ in range(m)]
    split(8)
    ec.jerasure.jerasure_matrix_encode(k, m, 8, M, data, coding, size)
    ref = alloc_shards(m, size, PAD)
    restatement.matrix_encode(k, m, np.array(M).reshape(m, k), hd, ref, size)
    for i in range(m):
        assert np.array_equal(coding[i].cpu().numpy()[:size], ref[i][:size]), i
