"""A/B the gf_apply kernel variants on the MI355X in ONE process (interleaved
rounds in a freshly shuffled order each round, median of each), against a
streaming-copy reference with the same byte volume.  Workload = the bench's: RS(10,4), 4 MiB shards, 24 stripes.

    python tools/tune_kernels.py [--rounds 15] [--stripes 24]

Prints one JSON object per variant: median/min launch ms and GB/s of
algorithmic HBM traffic ((K+R) * S per stripe; copy: 2 * S per pair).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import erasure_coding_test_amd as E  # noqa: E402
from erasure_coding_test_amd import _native as N  # noqa: E402

L = ctypes.CDLL(os.path.join(N.LIB_DIR, "libecgpu_diag.so"))
L.ecgpu_diag_launch.restype = ctypes.c_int
L.ecgpu_diag_launch.argtypes = [ctypes.c_int] * 5 + [ctypes.c_void_p] * 4 + [
    ctypes.c_int, ctypes.c_longlong, ctypes.c_ulonglong, ctypes.c_ulonglong, ctypes.c_int, ctypes.c_void_p,
    ctypes.c_void_p]
P3 = {}  # id(qtab tensor) -> 3-bit-slice tables of the same coefficients


def tables(coefs):
    gm = E.galois.galois_single_multiply
    q, nib, p3 = [], [], []
    for c in coefs:
        for p in range(4):
            q.append(sum(gm(c, e << (2 * p), 8) << (8 * e) for e in range(4)))
        nib += [gm(c, x, 8) for x in range(16)] + [gm(c, x << 4, 8) for x in range(16)]
        # P3 layout (ecgpu_runtime.hip build_tables): T0lo T0hi T1lo T1hi T2 pad pad pad
        w = lambda vals: sum(v << (8 * e) for e, v in enumerate(vals))
        t0 = [gm(c, e, 8) for e in range(8)]
        t1 = [gm(c, e << 3, 8) for e in range(8)]
        t2 = [gm(c, e << 6, 8) for e in range(4)]
        p3 += [w(t0[:4]), w(t0[4:]), w(t1[:4]), w(t1[4:]), w(t2), 0, 0, 0]
    qt = torch.tensor(q, dtype=torch.int64).to(torch.int32).cuda()
    P3[id(qt)] = torch.tensor(p3, dtype=torch.int64).to(torch.int32).cuda()
    return qt, torch.tensor(nib, dtype=torch.uint8).cuda()


def masks(coefs):
    unit = sum(1 << i for i, c in enumerate(coefs) if c == 1)
    zero = sum(1 << i for i, c in enumerate(coefs) if c == 0)
    return unit, zero


def ptr_table(ptrs):
    return torch.tensor(ptrs, dtype=torch.int64).cuda()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=15)
    ap.add_argument("--stripes", type=int, default=24)
    ap.add_argument("--pads", default="0", help="comma list of per-shard padding bytes (shard stride = S + pad)")
    ap.add_argument("--lds", default="", help="comma list of dynamic LDS bytes per block (occupancy caps); "
                    "each value runs the variants again under ECGPU_DIAG_LDS")
    ap.add_argument("--only", default="", help="comma list of substrings; keep variants matching any")
    args = ap.parse_args()
    k, m, S, B = 10, 4, 4 << 20, args.stripes
    results = []
    for pad in [int(p) for p in args.pads.split(",")]:
        if args.lds:
            for lds in args.lds.split(","):
                os.environ["ECGPU_DIAG_LDS"] = lds
                for r in run_layout(args, k, m, S, B, pad):
                    r["lds"] = int(lds)
                    results.append(r)
            os.environ.pop("ECGPU_DIAG_LDS", None)
        else:
            results += run_layout(args, k, m, S, B, pad)
    for r in results:
        print(json.dumps(r))


def run_layout(args, k, m, S, B, pad):
    slab = torch.empty((B, k + m, S + pad), dtype=torch.uint8, device="cuda")
    slab.random_(0, 256, generator=torch.Generator(device="cuda").manual_seed(5))
    addr = lambda s, i: slab[s, i].data_ptr()
    M = E.reed_sol.reed_sol_vandermonde_coding_matrix(k, m, 8)
    q_enc, n_enc = tables(M)
    u_enc, z_enc = masks(M)
    src_enc = ptr_table([addr(s, j) for s in range(B) for j in range(k)])
    dst_enc = ptr_table([addr(s, k + i) for s in range(B) for i in range(m)])
    dec_rows = {"ones": [1] * k, "dense": [150, 119, 240, 20, 249, 36, 126, 92, 191, 156]}
    src_dec = ptr_table([addr(s, j) for s in range(B) for j in range(1, k + 1)])
    dst_dec = ptr_table([addr(s, 0) for s in range(B)])
    src_cp = ptr_table([addr(s, i) for s in range(B) for i in range(7)])
    dst_cp = ptr_table([addr(s, 7 + i) for s in range(B) for i in range(7)])
    stream = torch.cuda.current_stream().cuda_stream

    variants = []
    for ntb in range(4):  # copy reference: cache policy bits (loads / stores)
        variants.append((f"copy vec1 ldnt{ntb & 1} stnt{ntb >> 1}", 1, 1, 1, 1, ntb, None, None, src_cp, dst_cp,
                         7 * B, 0, 0, 2 * S * 7 * B, 1))
    for nt in (1, 0):
        for vec in (1, 2):
            for mode, mname in ((2, "allperm"), (3, "xoronly")):
                variants.append((f"enc perm vec{vec} {mname} nt{nt}", 0, 10, 4, vec, mode, q_enc, n_enc, src_enc,
                                 dst_enc, B, u_enc, z_enc, (k + m) * S * B, nt))
        for bps in (16, 32, 64, 128):
            for mode, mname in ((2, "allperm"), (3, "xoronly")):
                variants.append((f"enc stream bps{bps} {mname} nt{nt}", 3, 10, 4, bps, mode, q_enc, n_enc, src_enc,
                                 dst_enc, B, u_enc, z_enc, (k + m) * S * B, nt))
    for nt in (1, 0):
        for um, uname in ((0, "none"), (1, "col0"), (3, "rs")):
            variants.append((f"enc apply {uname} nt{nt}", 4, 10, 4, 1, um, q_enc, n_enc, src_enc, dst_enc, B, u_enc,
                             z_enc, (k + m) * S * B, nt))
        variants.append((f"enc apply rs occ8 nt{nt}", 6, 10, 4, 1, 3, q_enc, n_enc, src_enc, dst_enc, B, u_enc,
                         z_enc, (k + m) * S * B, nt))
        variants.append((f"enc apply rs stripefast nt{nt}", 5, 10, 4, 1, 3, q_enc, n_enc, src_enc, dst_enc, B, u_enc,
                         z_enc, (k + m) * S * B, nt))
    # production body with the round-1 2-bit-slice tables (A/B vs "enc apply rs nt1")
    variants.append(("enc apply2 rs nt1", 10, 10, 4, 1, 3, q_enc, n_enc, src_enc, dst_enc, B, u_enc, z_enc,
                     (k + m) * S * B, 1))
    variants.append(("enc lds nt1", 2, 10, 4, 1, 0, q_enc, n_enc, src_enc, dst_enc, B, u_enc, z_enc,
                     (k + m) * S * B, 1))
    for name, row in dec_rows.items():
        qd, nd = tables(row)
        ud, zd = masks(row)
        variants.append((f"dec1 {name} vec1 allperm nt1", 0, 10, 1, 1, 2, qd, nd, src_dec, dst_dec, B, ud, zd,
                         (k + 1) * S * B, 1))
        for var, tag in ((4, ""), (5, " stripefast"), (6, " occ8")):
            variants.append((f"dec1 {name} apply {'all' if name == 'ones' else 'none'}{tag} nt1", var, 10, 1, 1,
                             4 if name == "ones" else 0, qd, nd, src_dec, dst_dec, B, ud, zd, (k + 1) * S * B, 1))
        variants.append((f"dec1 {name} apply2 nt1", 10, 10, 1, 1, 4 if name == "ones" else 0, qd, nd, src_dec,
                         dst_dec, B, ud, zd, (k + 1) * S * B, 1))
        for bps in (32, 64):
            variants.append((f"dec1 {name} stream bps{bps} nt1", 3, 10, 1, bps, 2, qd, nd, src_dec, dst_dec, B, ud,
                             zd, (k + 1) * S * B, 1))

    for flags in range(4):
        tag = ("stripe" if flags & 1 else "col") + ("/occ8" if flags & 2 else "/occ7")
        variants.append((f"F enc {tag}", 7, 10, 4, flags, 3, q_enc, n_enc, src_enc, dst_enc, B, u_enc, z_enc,
                         (k + m) * S * B, 1))
        qd, nd = tables(dec_rows["ones"])
        ud, zd = masks(dec_rows["ones"])
        variants.append((f"F dec1 {tag}", 7, 10, 1, flags, 4, qd, nd, src_dec, dst_dec, B, ud, zd,
                         (k + 1) * S * B, 1))
    for vec in (1, 2, 4):
        variants.append((f"V enc vec{vec}", 8, 10, 4, vec, 3, q_enc, n_enc, src_enc, dst_enc, B, u_enc, z_enc,
                         (k + m) * S * B, 1))
        qd, nd = tables(dec_rows["ones"])
        ud, zd = masks(dec_rows["ones"])
        variants.append((f"V dec1 vec{vec}", 8, 10, 1, vec, 4, qd, nd, src_dec, dst_dec, B, ud, zd,
                         (k + 1) * S * B, 1))
    only = [o for o in args.only.split(",")] if args.only else [""]
    # access-pattern probe (XOR-only, per-lane K reads + R writes)
    for K2, R2 in ((1, 1), (2, 1), (2, 2), (4, 1), (1, 4), (4, 4), (7, 7), (10, 1), (10, 4), (13, 1)):
        st = ptr_table([addr(s, j) for s in range(B) for j in range(K2)])
        dt = ptr_table([addr(s, K2 + i) for s in range(B) for i in range(R2)])
        variants.append((f"P xor K{K2} R{R2}", 9, K2, R2, 1, 3, q_enc, n_enc, st, dt, B, 0, 0, (K2 + R2) * S * B, 1))
    # read-only probes: K streams read, nothing written (diag variants 11 / 12)
    for K2 in (1, 4, 10, 14):
        st = ptr_table([addr(s, j) for s in range(B) for j in range(K2)])
        dt = ptr_table([addr(s, 0) for s in range(B)])
        variants.append((f"R regs K{K2}", 11, K2, 1, 1, 0, q_enc, n_enc, st, dt, B, 0, 0, K2 * S * B, 1))
        for nt in (1, 0):
            variants.append((f"R glds K{K2} nt{nt}", 12, K2, 1, 1, 0, q_enc, n_enc, st, dt, B, 0, 0, K2 * S * B, nt))
    # cache-policy / load-path factorial of the production combine (diag 13 / 14)
    qd1, nd1 = tables(dec_rows["ones"])
    ud1, zd1 = masks(dec_rows["ones"])
    for var, path in ((13, "regs"), (14, "dma")):
        for ntb in range(4):
            tag = f"ldnt{ntb & 1} stnt{ntb >> 1}"
            variants.append((f"X enc {path} {tag}", var, 10, 4, ntb, 3, q_enc, n_enc, src_enc, dst_enc, B, u_enc,
                             z_enc, (k + m) * S * B, 1))
            variants.append((f"X dec1 {path} {tag}", var, 10, 1, ntb, 4, qd1, nd1, src_dec, dst_dec, B, ud1, zd1,
                             (k + 1) * S * B, 1))
    # other launch shapes of the BASELINE configs, same factorial (register loads)
    M63 = E.reed_sol.reed_sol_vandermonde_coding_matrix(6, 3, 8)
    q63, n63 = tables(M63)
    u63, z63 = masks(M63)
    src63 = ptr_table([addr(s, j) for s in range(B) for j in range(6)])
    dst63 = ptr_table([addr(s, 6 + i) for s in range(B) for i in range(3)])
    dense4 = [150, 119, 240, 20, 249, 36, 126, 92, 191, 156, 234, 203, 20, 62, 66, 253, 51, 81, 244, 150,
              105, 20, 32, 68, 153, 129, 237, 70, 41, 130, 20, 169, 197, 111, 35, 89, 161, 75, 98, 136]
    q4d, n4d = tables(dense4)
    u4d, z4d = masks(dense4)
    src4d = ptr_table([addr(s, j) for s in range(B) for j in range(4, 14)])
    dst4d = ptr_table([addr(s, i) for s in range(B) for i in range(4)])
    qdd, ndd = tables(dec_rows["dense"])
    udd, zdd = masks(dec_rows["dense"])
    for ntb in range(4):
        tag = f"ldnt{ntb & 1} stnt{ntb >> 1}"
        variants.append((f"Y enc63 {tag}", 13, 6, 3, ntb, 3, q63, n63, src63, dst63, B, u63, z63, 9 * S * B, 1))
        variants.append((f"Y dec4dense {tag}", 13, 10, 4, ntb, 0, q4d, n4d, src4d, dst4d, B, u4d, z4d,
                         14 * S * B, 1))
        variants.append((f"Y dec1dense {tag}", 13, 10, 1, ntb, 0, qdd, ndd, src_dec, dst_dec, B, udd, zdd,
                         11 * S * B, 1))
    # explicit cache bits (diag variant 15, inline-asm loads / stores)
    lnames = ["nt", "sc1nt", "sc0sc1nt", "sc0sc1", "sc1"]
    snames = ["nt", "sc1", "sc0sc1", "sc0sc1nt", "sc1nt"]
    for lp in range(5):
        for sp in range(5):
            variants.append((f"C enc L{lnames[lp]} S{snames[sp]}", 15, 10, 4, lp, sp, q_enc, n_enc, src_enc, dst_enc,
                             B, u_enc, z_enc, (k + m) * S * B, 1))
            variants.append((f"C dec1 L{lnames[lp]} S{snames[sp]}", 15, 10, 1, lp, sp, qd1, nd1, src_dec, dst_dec, B,
                             ud1, zd1, (k + 1) * S * B, 1))
    variants = [v for v in variants if any(o in v[0] for o in only)]
    times = {v[0]: [] for v in variants}
    import random
    order = list(variants)
    if True:
        for rnd in range(args.rounds + 2):
            # shuffled every round: a kernel pays for the dirty lines its
            # predecessor left behind, so a fixed order biases the medians
            random.Random(rnd).shuffle(order)
            for v in order:
                name, var, K, R, vec, mode, qt, nb, st, dt, stripes, um, zm, nbytes, nt = v
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                rc = L.ecgpu_diag_launch(var, K, R, vec, mode, qt.data_ptr() if qt is not None else None,
                                         nb.data_ptr() if nb is not None else None, st.data_ptr(), dt.data_ptr(),
                                         stripes, S, um, zm, nt, stream,
                                         P3[id(qt)].data_ptr() if qt is not None else None)
                e1.record()
                assert rc == 0, (name, rc)
                torch.cuda.synchronize()
                if rnd >= 2:
                    times[name].append(e0.elapsed_time(e1))
    out = []
    for v in variants:
        t = times[v[0]]
        med = statistics.median(t)
        out.append({"variant": v[0], "pad": pad, "median_ms": round(med, 4), "min_ms": round(min(t), 4),
                    "GBps_median": round(v[-2] / med / 1e6, 1), "GBps_best": round(v[-2] / min(t) / 1e6, 1)})
    del slab
    torch.cuda.empty_cache()
    return out


if __name__ == "__main__":
    main()
