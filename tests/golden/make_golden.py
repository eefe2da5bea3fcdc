"""Generate the golden fixtures in tests/golden/ from the REFERENCE itself.

Runs only where /root/reference exists: it drives oracle/_ref/libjerasure_ref.so
(the reference's src/erasure_coding/*.cpp compiled unchanged by oracle/Makefile)
on deterministic inputs (tests/ecdata.py) and records inputs' seeds plus the
reference's outputs.  Nothing of the reference's source is stored -- only data.

    make -C oracle && python tests/golden/make_golden.py

Outputs:
  golden.json  -- KATs, matrices, decode matrices, digests, stats
  vectors.npz  -- raw parity bytes for the small-shard stripes (allow_pickle=False)
"""
from __future__ import annotations

import itertools
import json
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

from oracle.oracle import Reference, alloc_shards  # noqa: E402
from ecdata import CONFIGS, fnv1a64, shard_seed, splitmix_bytes  # noqa: E402

PAD = 16


def shards_from_seeds(cfg, stripe, count, size, first=0):
    out = alloc_shards(count, size, PAD)
    for s in range(count):
        out[s][:size] = splitmix_bytes(size, shard_seed(cfg, stripe, first + s))
    return out


def main():
    ref = Reference()
    g = {"generator": "tests/golden/make_golden.py", "source": "oracle/_ref/libjerasure_ref.so (reference compiled -O2)"}
    vec = {}

    # ---- 1. scalar field -------------------------------------------------
    mul = np.array([[ref.gf_mul(a, b) for b in range(256)] for a in range(256)], dtype=np.uint8)
    vec["gf_mul_table"] = mul
    g["scalar"] = {
        "kat": {"mul_2_0x80": ref.gf_mul(2, 0x80), "mul_3_7": ref.gf_mul(3, 7), "inverse_2": ref.gf_inverse(2),
                "div_1_147": ref.gf_div(1, 147), "log_2": ref.gf_log(2), "ilog_1": ref.gf_ilog(1)},
        "inverse": [ref.gf_inverse(a) for a in range(256)],
        "div_by_zero": [ref.gf_div(a, 0) for a in range(0, 256, 51)],
        "log": [ref.gf_log(v) for v in range(256)],
        "ilog": {str(v): ref.gf_ilog(v) for v in range(-255, 510)},
    }

    # ---- 2. coding matrices ---------------------------------------------
    mats = {}
    for k in range(2, 17):
        for m in range(1, 9):
            M = ref.vandermonde_coding_matrix(k, m)
            mats[f"{k},{m}"] = None if M is None else M.tolist()
    g["vandermonde"] = mats
    g["r6"] = {str(k): ref.r6_coding_matrix(k).tolist() for k in range(2, 17)}

    # ---- 3. decode matrices ---------------------------------------------
    dec = {}
    for (k, m) in [(6, 3), (4, 2), (10, 4)]:
        M = ref.vandermonde_coding_matrix(k, m)
        sets = []
        for e in range(1, m + 1):
            sets += list(itertools.combinations(range(k + m), e))
        if k == 10:
            rnd = random.Random(10 * 4)
            sets = [(0,), (0, 1, 2, 3), (9, 10, 11, 12), (3, 7, 11, 13)] + rnd.sample(sets, 40)
        for s in sets:
            erased = [1 if i in s else 0 for i in range(k + m)]
            if not any(erased[:k]):
                continue
            rc, dm, ids = ref.make_decoding_matrix(k, m, M, erased)
            dec[f"{k},{m}:{','.join(map(str, s))}"] = {"rc": rc, "dm": dm.tolist(), "dm_ids": ids}
    g["decoding_matrices"] = dec

    # ---- 4. encode vectors (small shards, exact bytes; ragged sizes digests)
    enc = {}
    for cfg, c in CONFIGS.items():
        k, m = c["k"], c["m"]
        M = ref.vandermonde_coding_matrix(k, m)
        for size in (4096, 4099, 1000, 7, 1):
            for stripe in range(2):
                data = shards_from_seeds(cfg, stripe, k, size)
                coding = alloc_shards(m, size, PAD)
                ref.matrix_encode(k, m, M, data, coding, size)
                key = f"C{cfg}:{size}:{stripe}"
                enc[key] = [fnv1a64(x[:size]) for x in coding]
                if size == 4096:
                    vec[f"enc_{cfg}_{stripe}"] = np.stack([x[:size] for x in coding])
    g["encode_small"] = enc

    # ---- 5. decode on INCONSISTENT inputs (pins survivor choice/semantics)
    dcases = []
    rnd = random.Random(2024)
    for (cfg, k, m) in [(2, 6, 3), (3, 10, 4), (1, 4, 2)]:
        M = ref.vandermonde_coding_matrix(k, m)
        sets = []
        for e in range(1, m + 2):  # includes one-too-many (returns -1)
            sets += list(itertools.combinations(range(k + m), e))
        if k == 10:
            sets = [(0,), (0, 1, 2, 3), (10,), (0, 13), (9, 10, 11, 12), (1, 2, 3, 4, 5)] + rnd.sample(sets, 30)
        for s in sets:
            for rko in (0, 1):
                size = 1000
                data = shards_from_seeds(cfg, 7, k, size)
                coding = shards_from_seeds(cfg, 7, m, size, first=k)  # NOT a codeword on purpose
                rc = ref.matrix_decode(k, m, M, rko, list(s), data, coding, size)
                dcases.append({"cfg": cfg, "k": k, "m": m, "erasures": list(s), "row_k_ones": rko, "size": size,
                               "rc": rc, "digests": [fnv1a64(x[:size]) for x in data + coding]})
    g["decode_inconsistent"] = dcases

    # ---- 6. dotprod cases ----------------------------------------------
    dots = []
    for t in range(40):
        k, m = rnd.choice([(4, 2), (6, 3), (10, 4)])
        row = [rnd.choice([0, 0, 1, 1, 2, 3, 29, 142, 255, rnd.randrange(256)]) for _ in range(k)]
        use_ids = rnd.random() < 0.5
        src_ids = rnd.sample(range(k + m), k) if use_ids else None
        dest = rnd.randrange(k + m)
        size = rnd.choice([1, 8, 100, 1000, 4096])
        data = shards_from_seeds(9, t, k, size)
        coding = shards_from_seeds(9, t, m, size, first=k)
        ref.matrix_dotprod(k, row, src_ids, dest, data, coding, size)
        dots.append({"k": k, "m": m, "row": row, "src_ids": src_ids, "dest_id": dest, "size": size, "seed_stripe": t,
                     "digests": [fnv1a64(x[:size]) for x in data + coding]})
    g["dotprod"] = dots

    # ---- 7. region ops ---------------------------------------------------
    regs = []
    for t, (c, add, size, mode) in enumerate(itertools.product([0, 1, 2, 29, 142, 255], [0, 1], [1, 13, 4096, 4099],
                                                             ["r2", "inplace"])):
        src = shards_from_seeds(10, t, 1, size)[0]
        dst = shards_from_seeds(10, t, 1, size, first=1)[0]
        if mode == "r2":
            ref.region_multiply(src, c, size, dst, add)
            out = dst
        else:
            ref.region_multiply(src, c, size, None, add)
            out = src
        regs.append({"multby": c, "add": add, "size": size, "mode": mode, "seed_stripe": t, "digest": fnv1a64(out[:size])})
    xors = []
    for t, size in enumerate([1, 8, 13, 4096, 4099]):
        a, b = shards_from_seeds(11, t, 2, size)
        c = alloc_shards(1, size, PAD)[0]
        ref.region_xor(a, b, c, size)
        xors.append({"size": size, "seed_stripe": t, "digest": fnv1a64(c[:size])})
    g["region_multiply"] = regs
    g["region_xor"] = xors

    # ---- 8. full-size digests (valid codewords) --------------------------
    full = {}
    for cfg in (2, 3, 5):
        c = CONFIGS[cfg]
        k, m, size = c["k"], c["m"], c["size"]
        M = ref.vandermonde_coding_matrix(k, m)
        data = shards_from_seeds(cfg, 0, k, size)
        coding = alloc_shards(m, size, PAD)
        ref.matrix_encode(k, m, M, data, coding, size)
        full[f"C{cfg}"] = {"k": k, "m": m, "size": size, "stripe": 0,
                           "data": [fnv1a64(x[:size]) for x in data], "coding": [fnv1a64(x[:size]) for x in coding]}
    g["full_size"] = full

    # ---- 8b. C4 at its BASELINE size on INCONSISTENT inputs --------------
    # RS(10,4) 4 MiB shards whose parity is NOT the data's: the reference's
    # survivor choice (dm_ids = the first k non-erased, jerasure.cpp:84-112),
    # its row_k_ones shortcut and the re-encode of erased parity from the
    # RECOVERED data (:223-247) all show in the bytes, at the size whose
    # launches differ from the 1000-B cases' (plan / batched path).
    k, m, size = 10, 4, 4 << 20
    M = ref.vandermonde_coding_matrix(k, m)
    c4 = []
    for erasures, rko in (([0, 1, 2, 3], 0), ([0, 1, 2, 3], 1), ([12], 0), ([1, 4, 11, 13], 0), ([2, 10], 1)):
        data = shards_from_seeds(4, 7, k, size)
        coding = shards_from_seeds(4, 7, m, size, first=k)  # NOT a codeword on purpose
        rc = ref.matrix_decode(k, m, M, rko, erasures, data, coding, size)
        c4.append({"erasures": erasures, "row_k_ones": rko, "rc": rc, "stripe": 7,
                   "digests": [fnv1a64(x[:size]) for x in data + coding]})
    g["c4_full_inconsistent"] = {"k": k, "m": m, "size": size, "cfg": 4, "cases": c4}

    # ---- 9. stats semantics (jerasure.cpp:1143-1151 fill order) ----------
    ref.get_stats()
    k, m = 10, 4
    M = ref.vandermonde_coding_matrix(k, m)
    data = shards_from_seeds(3, 0, k, 4096)
    coding = alloc_shards(m, 4096, PAD)
    ref.matrix_encode(k, m, M, data, coding, 4096)
    g["stats_after_rs10_4_encode_4096"] = ref.get_stats()
    ref.matrix_decode(k, m, M, 0, [0, 1, 2, 3], data, coding, 4096)
    g["stats_after_rs10_4_decode_0123_4096"] = ref.get_stats()

    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(g, f, indent=None, separators=(",", ":"))
    np.savez_compressed(os.path.join(HERE, "vectors.npz"), **vec)
    print("wrote", os.path.join(HERE, "golden.json"), "and vectors.npz")


if __name__ == "__main__":
    main()
