"""Pin the oracle: the C restatement (oracle/ec_oracle.c) against the golden
vectors generated from the reference itself (tests/golden/make_golden.py),
and -- where the reference build exists -- against the reference directly."""
import itertools
import random

import numpy as np
import pytest

from ecdata import CONFIGS, fnv1a64, shard_seed, splitmix_bytes
from oracle.oracle import alloc_shards


def shards(cfg, stripe, count, size, first=0, pad=16):
    out = alloc_shards(count, size, pad)
    for s in range(count):
        out[s][:size] = splitmix_bytes(size, shard_seed(cfg, stripe, first + s))
    return out


def test_splitmix_matches_c(restatement):
    for n in (0, 1, 7, 8, 9, 1000, 4099):
        a = splitmix_bytes(n, shard_seed(2, 3, 4))
        b = np.zeros(n, np.uint8)
        restatement.fill(b, shard_seed(2, 3, 4))
        assert np.array_equal(a, b)
        assert fnv1a64(a) == restatement.fnv1a64(a)


def test_scalar_kats(restatement, golden, vectors):
    s = golden["scalar"]
    kat = s["kat"]
    R = restatement
    assert R.gf_mul(2, 0x80) == kat["mul_2_0x80"] == 29
    assert R.gf_mul(3, 7) == kat["mul_3_7"] == 9
    assert R.gf_inverse(2) == kat["inverse_2"] == 142
    assert R.gf_div(1, 147) == kat["div_1_147"] == 79
    assert R.gf_log(2) == kat["log_2"] == 1
    assert R.gf_ilog(1) == kat["ilog_1"] == 2
    mul = np.array([[R.gf_mul(a, b) for b in range(256)] for a in range(256)], np.uint8)
    assert np.array_equal(mul, vectors["gf_mul_table"])
    assert [R.gf_inverse(a) for a in range(256)] == s["inverse"]
    assert [R.gf_log(v) for v in range(256)] == s["log"]
    assert all(R.gf_ilog(int(v)) == x for v, x in s["ilog"].items())
    assert [R.gf_div(a, 0) for a in range(0, 256, 51)] == s["div_by_zero"]


def test_vandermonde_matrices(restatement, golden):
    for key, mat in golden["vandermonde"].items():
        k, m = map(int, key.split(","))
        got = restatement.vandermonde_coding_matrix(k, m)
        assert (got is None) == (mat is None), key
        if mat is not None:
            assert got.tolist() == mat, key


def test_survey_kat_rows(restatement):
    # SURVEY.md §8c known answers
    assert restatement.vandermonde_coding_matrix(4, 2).tolist() == [[1, 1, 1, 1], [1, 70, 143, 200]]
    assert restatement.vandermonde_coding_matrix(10, 4)[3].tolist() == [1, 220, 166, 123, 82, 143, 245, 40, 167, 122]


def test_decoding_matrices(restatement, golden):
    cache = {}
    for key, exp in golden["decoding_matrices"].items():
        km, ers = key.split(":")
        k, m = map(int, km.split(","))
        if km not in cache:
            cache[km] = restatement.vandermonde_coding_matrix(k, m)
        er = set(map(int, ers.split(",")))
        erased = [1 if i in er else 0 for i in range(k + m)]
        rc, dm, ids = restatement.make_decoding_matrix(k, m, cache[km], erased)
        assert rc == exp["rc"], key
        assert ids == exp["dm_ids"], key
        assert dm.tolist() == exp["dm"], key


@pytest.mark.parametrize("cfg", sorted(CONFIGS))
def test_encode_small_vectors(restatement, golden, vectors, cfg):
    k, m = CONFIGS[cfg]["k"], CONFIGS[cfg]["m"]
    M = restatement.vandermonde_coding_matrix(k, m)
    for size in (4096, 4099, 1000, 7, 1):
        for stripe in range(2):
            data = shards(cfg, stripe, k, size)
            coding = alloc_shards(m, size)
            restatement.matrix_encode(k, m, M, data, coding, size)
            assert [fnv1a64(c[:size]) for c in coding] == golden["encode_small"][f"C{cfg}:{size}:{stripe}"]
            if size == 4096:
                assert np.array_equal(np.stack([c[:size] for c in coding]), vectors[f"enc_{cfg}_{stripe}"])


def test_decode_inconsistent_inputs(restatement, golden):
    mats = {}
    for case in golden["decode_inconsistent"]:
        k, m, cfg, size = case["k"], case["m"], case["cfg"], case["size"]
        if (k, m) not in mats:
            mats[(k, m)] = restatement.vandermonde_coding_matrix(k, m)
        data = shards(cfg, 7, k, size)
        coding = shards(cfg, 7, m, size, first=k)
        rc = restatement.matrix_decode(k, m, mats[(k, m)], case["row_k_ones"], case["erasures"], data, coding, size)
        assert rc == case["rc"], case["erasures"]
        assert [fnv1a64(x[:size]) for x in data + coding] == case["digests"], (case["erasures"], case["row_k_ones"])


def test_decode_inconsistent_full_size_c4(restatement, golden):
    """BASELINE config 4 at 4 MiB on inputs that are not a codeword: the
    restatement's survivor choice and re-encode against the reference's
    digests (golden["c4_full_inconsistent"])."""
    g = golden["c4_full_inconsistent"]
    k, m, size = g["k"], g["m"], g["size"]
    M = restatement.vandermonde_coding_matrix(k, m)
    for case in g["cases"]:
        data = shards(g["cfg"], 7, k, size)
        coding = shards(g["cfg"], 7, m, size, first=k)
        rc = restatement.matrix_decode(k, m, M, case["row_k_ones"], case["erasures"], data, coding, size)
        assert rc == case["rc"]
        assert [fnv1a64(x[:size]) for x in data + coding] == case["digests"], (case["erasures"], case["row_k_ones"])


def test_dotprod_cases(restatement, golden):
    for t, case in enumerate(golden["dotprod"]):
        k, m, size = case["k"], case["m"], case["size"]
        data = shards(9, case["seed_stripe"], k, size)
        coding = shards(9, case["seed_stripe"], m, size, first=k)
        restatement.matrix_dotprod(k, case["row"], case["src_ids"], case["dest_id"], data, coding, size)
        assert [fnv1a64(x[:size]) for x in data + coding] == case["digests"], t


def test_region_ops(restatement, golden):
    for case in golden["region_multiply"]:
        size, t = case["size"], case["seed_stripe"]
        src = shards(10, t, 1, size)[0]
        dst = shards(10, t, 1, size, first=1)[0]
        if case["mode"] == "r2":
            restatement.region_multiply(src, case["multby"], size, dst, case["add"])
            out = dst
        else:
            restatement.region_multiply(src, case["multby"], size, None, case["add"])
            out = src
        assert fnv1a64(out[:size]) == case["digest"], case
    for case in golden["region_xor"]:
        size = case["size"]
        a, b = shards(11, case["seed_stripe"], 2, size)
        c = alloc_shards(1, size)[0]
        restatement.region_xor(a, b, c, size)
        assert fnv1a64(c[:size]) == case["digest"]


def test_multithreaded_encode_matches(restatement):
    k, m, size = 6, 3, 100003
    M = restatement.vandermonde_coding_matrix(k, m)
    data = shards(2, 5, k, size)
    c1, c2 = alloc_shards(m, size), alloc_shards(m, size)
    restatement.matrix_encode(k, m, M, data, c1, size)
    assert restatement.matrix_encode_mt(k, m, M, data, c2, size, 7) == 0
    for a, b in zip(c1, c2):
        assert np.array_equal(a[:size], b[:size])


def test_restatement_vs_reference_random(restatement, reference):
    rnd = random.Random(7)
    for t in range(30):
        k = rnd.randint(2, 14)
        m = rnd.randint(1, 5)
        M = reference.vandermonde_coding_matrix(k, m)
        assert np.array_equal(M, restatement.vandermonde_coding_matrix(k, m))
        size = rnd.choice([8, 64, 1024, 1000, 333])
        data = shards(12, t, k, size)
        c1, c2 = alloc_shards(m, size), alloc_shards(m, size)
        reference.matrix_encode(k, m, M, data, c1, size)
        restatement.matrix_encode(k, m, M, data, c2, size)
        for a, b in zip(c1, c2):
            assert np.array_equal(a[:size], b[:size])
        er = rnd.sample(range(k + m), rnd.randint(1, m))
        d1 = [x.copy() for x in data] + [x.copy() for x in c1]
        d2 = [x.copy() for x in data] + [x.copy() for x in c1]
        for e in er:
            d1[e][:size] = 0xAA
            d2[e][:size] = 0x55
        rko = rnd.randint(0, 1)
        r1 = reference.matrix_decode(k, m, M, rko, er, d1[:k], d1[k:], size)
        r2 = restatement.matrix_decode(k, m, M, rko, er, d2[:k], d2[k:], size)
        assert r1 == r2 == 0
        for a, b, orig in zip(d1, d2, data + c1):
            assert np.array_equal(a[:size], b[:size])
            assert np.array_equal(a[:size], orig[:size])


def test_all_erasure_patterns_rs63_roundtrip(restatement):
    k, m, size = 6, 3, 256
    M = restatement.vandermonde_coding_matrix(k, m)
    data = shards(2, 1, k, size)
    coding = alloc_shards(m, size)
    restatement.matrix_encode(k, m, M, data, coding, size)
    orig = [x.copy() for x in data + coding]
    for e in range(1, m + 1):
        for er in itertools.combinations(range(k + m), e):
            bufs = [x.copy() for x in orig]
            for i in er:
                bufs[i][:size] = 0
            assert restatement.matrix_decode(k, m, M, 0, list(er), bufs[:k], bufs[k:], size) == 0
            for a, b in zip(bufs, orig):
                assert np.array_equal(a[:size], b[:size])
