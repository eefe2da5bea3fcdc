"""Subprocess driver of the CPU-fallback tests (tests/test_cpu_fallback.py):
the reference's own callers' call sequences through libjerasure_amd.so's
C++-mangled names, checked against golden fixtures and the reference built
here (oracle/_ref, as the checker).

    python tests/fallback_driver.py client|ecx|surface|pinned|pinned_alias|oom

Run with ECGPU_TEST_INJECT_HIP (this driver's variable: it sets the library's
test-only test_inject_hip knob, which no deployment's environment can) and
ECGPU_CPU_FALLBACK in the environment; prints
one JSON line {"scenario", "checked", "mismatches", "fallbacks", "lost"} and
exits 0 when every output matched (the drop-in itself exits 1 where a call
cannot complete).  No torch: the drop-in is loaded the way an unchanged C++
caller loads it.

* client -- the reference client's calls (client_main.cpp:1060, :2118,
  :1670): reed_sol_vandermonde_coding_matrix, jerasure_matrix_encode on C1-C3
  golden stripes at 4096 / 4099 / 1000 B, every golden inconsistent decode
  (return code and bytes), and a C3 4 MiB encode + decode{0,1,2,3} round trip
  on one malloc'd stripe buffer (the staged large-call path).
* ecx -- the ECX datanode's per-block sequence (ecx_datanode_main.cpp:
  699-734): RS(3,3) blocks of 349,525 B arriving one source at a time, each
  parity block memcpy'd / galois_region_xor'd / galois_w08_region_multiply'd
  with init[], against the reference's encode of the same blocks; plus the
  golden region-op cases.
* surface -- the rest of the header surface on the fallback: w = 16 / 32
  region multiplies and matrix encode, dot products, bit-matrix and schedule
  encode, RAID-6, against the reference (-fno-strict-aliasing build for w = 16).
* pinned / pinned_alias -- registered host buffers the kernel writes in place:
  an encode (outputs identical to no source: recoverable after a partial
  write) and an in-place region multiply (the output is the source: not).
* oom -- GPU only: HBM filled by hipMalloc until it fails, then the client's
  C3 4 MiB encode + decode{0,1,2,3}: the library's staging hipMalloc fails for
  real.
"""
from __future__ import annotations

import ctypes
import json
import os
import sys

import numpy as np

TESTS = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(TESTS)
sys.path.insert(0, TESTS)
from ecdata import CONFIGS, fnv1a64, shard_seed, splitmix_bytes  # noqa: E402

LIB = os.path.join(ROOT, "erasure_coding_test_amd", "lib")
REF = os.path.join(ROOT, "oracle", "_ref")
I = ctypes.c_int
P = ctypes.c_void_p
PP = ctypes.POINTER(ctypes.c_void_p)
IP = ctypes.POINTER(ctypes.c_int)

# mangled names (include/dropin/*.h)
SIGS = {
    "vdm": ("_Z34reed_sol_vandermonde_coding_matrixiii", P, [I, I, I]),
    "encode": ("_Z22jerasure_matrix_encodeiiiPiPPcS1_i", None, [I, I, I, IP, PP, PP, I]),
    "decode": ("_Z22jerasure_matrix_decodeiiiPiiS_PPcS1_i", I, [I, I, I, IP, I, IP, PP, PP, I]),
    "dotprod": ("_Z23jerasure_matrix_dotprodiiPiS_iPPcS1_i", None, [I, I, IP, IP, I, PP, PP, I]),
    "rmul8": ("_Z26galois_w08_region_multiplyPciiS_i", None, [P, I, I, P, I]),
    "rmul16": ("_Z26galois_w16_region_multiplyPciiS_i", None, [P, I, I, P, I]),
    "rmul32": ("_Z26galois_w32_region_multiplyPciiS_i", None, [P, I, I, P, I]),
    "rxor": ("_Z17galois_region_xorPcS_S_i", None, [P, P, P, I]),
    "to_bitmatrix": ("_Z28jerasure_matrix_to_bitmatrixiiiPi", P, [I, I, I, IP]),
    "bm_encode": ("_Z25jerasure_bitmatrix_encodeiiiPiPPcS1_ii", None, [I, I, I, IP, PP, PP, I, I]),
    "smart_sched": ("_Z36jerasure_smart_bitmatrix_to_scheduleiiiPi", P, [I, I, I, IP]),
    "sched_encode": ("_Z24jerasure_schedule_encodeiiiPPiPPcS2_ii", None, [I, I, I, P, PP, PP, I, I]),
    "r6": ("_Z18reed_sol_r6_encodeiiPPcS0_i", I, [I, I, PP, PP, I]),
}


def bind(path):
    L = ctypes.CDLL(path)
    f = {}
    for key, (name, res, args) in SIGS.items():
        fn = getattr(L, name)
        fn.restype, fn.argtypes = res, args
        f[key] = fn
    return f


def ptrs(bufs):
    return (P * len(bufs))(*[b.ctypes.data for b in bufs])


def ints(v):
    return (I * len(v))(*v)


def matrix(f, k, m, w=8):
    p = f["vdm"](k, m, w)
    return list((I * (k * m)).from_address(p))


def shards(cfg, stripe, count, size, first=0, pad=16):
    out = []
    for s in range(count):
        b = np.zeros(size + pad, np.uint8)
        b[:size] = splitmix_bytes(size, shard_seed(cfg, stripe, first + s))
        out.append(b)
    return out


class Run:
    def __init__(self, name):
        self.name, self.checked, self.mismatches = name, 0, []

    def check(self, ok, what):
        self.checked += 1
        if not ok:
            self.mismatches.append(what)


def client(d, golden, run):
    for cfg in (1, 2, 3):
        k, m = CONFIGS[cfg]["k"], CONFIGS[cfg]["m"]
        M = matrix(d, k, m)
        for size in (4096, 4099, 1000):
            for stripe in range(2):
                data = shards(cfg, stripe, k, size)
                coding = [np.zeros(size + 16, np.uint8) for _ in range(m)]
                d["encode"](k, m, 8, ints(M), ptrs(data), ptrs(coding), size)
                run.check([fnv1a64(c[:size]) for c in coding] == golden["encode_small"][f"C{cfg}:{size}:{stripe}"],
                          f"encode C{cfg} {size} stripe {stripe}")
    mats = {}
    for case in golden["decode_inconsistent"]:
        k, m, cfg, size = case["k"], case["m"], case["cfg"], case["size"]
        if (k, m) not in mats:
            mats[(k, m)] = matrix(d, k, m)
        bufs = shards(cfg, 7, k, size) + shards(cfg, 7, m, size, first=k)
        rc = d["decode"](k, m, 8, ints(mats[(k, m)]), case["row_k_ones"], ints(case["erasures"] + [-1]),
                         ptrs(bufs[:k]), ptrs(bufs[k:]), size)
        run.check(rc == case["rc"], f"decode rc {case['erasures']}")
        if rc == 0:
            run.check([fnv1a64(b[:size]) for b in bufs] == case["digests"],
                      f"decode bytes {case['cfg']} {case['erasures']} rko {case['row_k_ones']}")
    # one client stripe buffer, C3 at 4 MiB: the large staged path, then a round trip
    k, m, size = 10, 4, 4 << 20
    M = matrix(d, k, m)
    slab = np.zeros((k + m) * size, np.uint8)
    sh = [slab[i * size:(i + 1) * size] for i in range(k + m)]
    for i in range(k):
        sh[i][:] = splitmix_bytes(size, shard_seed(3, 0, i))
    d["encode"](k, m, 8, ints(M), ptrs(sh[:k]), ptrs(sh[k:]), size)
    run.check([fnv1a64(c) for c in sh[k:]] == golden["full_size"]["C3"]["coding"], "C3 4 MiB encode digests")
    keep = [s.copy() for s in sh[:4]]
    for s in sh[:4]:
        s[:] = 0xEE
    rc = d["decode"](k, m, 8, ints(M), 0, ints([0, 1, 2, 3, -1]), ptrs(sh[:k]), ptrs(sh[k:]), size)
    run.check(rc == 0 and all(np.array_equal(a, b) for a, b in zip(sh[:4], keep)), "C3 4 MiB decode{0,1,2,3}")


def ecx(d, ref, golden, run):
    k, m, bs = 3, 3, (1 << 20) // 3  # the reference client's EC_K / EC_M; 349,525 B blocks
    M = matrix(d, k, m)
    blocks = shards(40, 0, k, bs)
    acc = [np.zeros(bs + 8, np.uint8) for _ in range(m)]
    init = [0] * m
    for j in range(k):  # ecx_datanode_main.cpp:699-734, block j of source j
        for i in range(m):
            c = M[i * k + j]
            if c == 1:
                if not init[i]:
                    acc[i][:bs] = blocks[j][:bs]
                    init[i] = 1
                else:
                    d["rxor"](blocks[j].ctypes.data, acc[i].ctypes.data, acc[i].ctypes.data, bs)
            if c not in (0, 1):
                d["rmul8"](blocks[j].ctypes.data, c, bs, acc[i].ctypes.data, init[i])
                init[i] = 1
    want = [np.zeros(bs + 16, np.uint8) for _ in range(m)]
    ref["encode"](k, m, 8, ints(M), ptrs(blocks), ptrs(want), bs)
    for i in range(m):
        run.check(np.array_equal(acc[i][:bs], want[i][:bs]), f"ECX parity block {i}")
    for case in golden["region_multiply"]:
        size, t = case["size"], case["seed_stripe"]
        src = shards(10, t, 1, size)[0]
        dst = shards(10, t, 1, size, first=1)[0]
        if case["mode"] == "r2":
            d["rmul8"](src.ctypes.data, case["multby"], size, dst.ctypes.data, case["add"])
            out = dst
        else:
            d["rmul8"](src.ctypes.data, case["multby"], size, None, case["add"])
            out = src
        run.check(fnv1a64(out[:size]) == case["digest"], f"region multiply {case}")
    for case in golden["region_xor"]:
        size = case["size"]
        a, b = shards(11, case["seed_stripe"], 2, size)
        c = np.zeros(size + 16, np.uint8)
        d["rxor"](a.ctypes.data, b.ctypes.data, c.ctypes.data, size)
        run.check(fnv1a64(c[:size]) == case["digest"], f"region xor {size}")
        d["rxor"](a.ctypes.data, b.ctypes.data, a.ctypes.data, size)  # r3 == r1
        run.check(fnv1a64(a[:size]) == case["digest"], f"region xor r3 == r1 {size}")


def surface(d, ref, ref_nsa, run):
    rng = np.random.default_rng(5)
    size = 64 << 10
    for w, fn in ((16, "rmul16"), (32, "rmul32")):
        r = ref_nsa if w == 16 else ref
        for add in (0, 1):
            src = rng.integers(0, 256, size + 16, dtype=np.uint8)
            dst = rng.integers(0, 256, size + 16, dtype=np.uint8)
            a, b = dst.copy(), dst.copy()
            d[fn](src.ctypes.data, 0x1234 + w, size, a.ctypes.data, add)
            r[fn](src.ctypes.data, 0x1234 + w, size, b.ctypes.data, add)
            run.check(np.array_equal(a[:size], b[:size]), f"w{w} region multiply add={add}")
        k, m = 6, 3
        M = matrix(d, k, m, w)
        data = [rng.integers(0, 256, size + 16, dtype=np.uint8) for _ in range(k)]
        c1 = [np.zeros(size + 16, np.uint8) for _ in range(m)]
        c2 = [np.zeros(size + 16, np.uint8) for _ in range(m)]
        d["encode"](k, m, w, ints(M), ptrs(data), ptrs(c1), size)
        r["encode"](k, m, w, ints(M), ptrs(data), ptrs(c2), size)
        run.check(all(np.array_equal(a[:size], b[:size]) for a, b in zip(c1, c2)), f"w{w} matrix encode")
    k, m, w, ps = 5, 2, 8, 1024
    M = matrix(d, k, m)
    bmp = d["to_bitmatrix"](k, m, w, ints(M))
    BM = list((I * (k * m * w * w)).from_address(bmp))
    bsize = w * ps * 3
    data = [rng.integers(0, 256, bsize, dtype=np.uint8) for _ in range(k)]
    c1 = [np.zeros(bsize, np.uint8) for _ in range(m)]
    c2 = [np.zeros(bsize, np.uint8) for _ in range(m)]
    d["bm_encode"](k, m, w, ints(BM), ptrs(data), ptrs(c1), bsize, ps)
    ref["bm_encode"](k, m, w, ints(BM), ptrs(data), ptrs(c2), bsize, ps)
    run.check(all(np.array_equal(a, b) for a, b in zip(c1, c2)), "bit-matrix encode")
    sched = d["smart_sched"](k, m, w, ints(BM))
    c3 = [np.zeros(bsize, np.uint8) for _ in range(m)]
    d["sched_encode"](k, m, w, sched, ptrs(data), ptrs(c3), bsize, ps)
    run.check(all(np.array_equal(a, b) for a, b in zip(c3, c2)), "schedule encode")
    r6a = [np.zeros(size, np.uint8) for _ in range(2)]
    r6b = [np.zeros(size, np.uint8) for _ in range(2)]
    data = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(4)]
    ra = d["r6"](4, 8, ptrs(data), ptrs(r6a), size)
    rb = ref["r6"](4, 8, ptrs(data), ptrs(r6b), size)
    run.check(ra == rb == 1 and all(np.array_equal(a, b) for a, b in zip(r6a, r6b)), "RAID-6 encode")
    row = [1, 0, 71, 1, 200]
    dst1 = rng.integers(0, 256, size, dtype=np.uint8)
    dst2 = dst1.copy()
    data = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(5)]
    d["dotprod"](5, 8, ints(row), None, 5, ptrs(data), ptrs([dst1]), size)
    ref["dotprod"](5, 8, ints(row), None, 5, ptrs(data), ptrs([dst2]), size)
    run.check(np.array_equal(dst1, dst2), "dot product")
    # aliasing: a coding buffer that is also a data buffer follows the
    # reference's sequential semantics (jerasure.cpp:285-299)
    k, m = 6, 3
    M = matrix(d, k, m)

    def aliased_encode(lib):
        data = [np.array(x) for x in shards(41, 0, k, size, pad=0)]
        coding = [data[3], np.zeros(size, np.uint8), np.zeros(size, np.uint8)]
        lib["encode"](k, m, 8, ints(M), ptrs(data), ptrs(coding), size)
        return np.concatenate(data + coding[1:]).tobytes()

    run.check(aliased_encode(d) == aliased_encode(ref), "encode with coding[0] == data[3]")
    src = rng.integers(0, 256, size, dtype=np.uint8)
    a, b = src.copy(), src.copy()
    d["rmul8"](a.ctypes.data, 77, size, None, 1)
    ref["rmul8"](b.ctypes.data, 77, size, None, 1)
    run.check(np.array_equal(a, b), "in-place region multiply")


def set_injection(core):
    """ECGPU_TEST_INJECT_HIP -> the library's test_inject_hip knob."""
    v = int(os.environ.get("ECGPU_TEST_INJECT_HIP", "0") or 0)
    if v:
        core.ecgpu_set_knob.argtypes = [ctypes.c_char_p, ctypes.c_int]
        assert core.ecgpu_set_knob(b"test_inject_hip", v) == 0


def register(core, arrays):
    """hipHostRegister each array (ecgpu_host_register): pinned host memory
    the kernels read and write in place."""
    core.ecgpu_host_register.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    for a in arrays:
        assert core.ecgpu_host_register(a.ctypes.data, a.nbytes) == 0


def pinned(d, ref, core, run):
    """RS(6,3) 1 MiB encode on registered (pinned) buffers: the inline kernel
    writes the coding shards in place over PCIe, so a failure after that
    point has partly written caller memory -- recoverable, since no output is
    also a source (the map reads the sources only)."""
    k, m, size = 6, 3, 1 << 20
    M = matrix(d, k, m)
    data = shards(2, 0, k, size, pad=0)
    coding = [np.full(size, 0xA5, np.uint8) for _ in range(m)]
    register(core, data + coding)
    d["encode"](k, m, 8, ints(M), ptrs(data), ptrs(coding), size)
    want = [np.zeros(size, np.uint8) for _ in range(m)]
    ref["encode"](k, m, 8, ints(M), ptrs(data), ptrs(want), size)
    for i in range(m):
        run.check(np.array_equal(coding[i], want[i]), f"pinned encode coding {i}")


def pinned_alias(d, ref, core, run):
    """In-place region multiply (r2 = NULL, galois.cpp:429) of a registered
    buffer: the output IS the source, so once the kernel started writing it
    the CPU can no longer recompute it -- the call keeps the error."""
    size = 1 << 20
    buf = np.random.default_rng(3).integers(0, 256, size, dtype=np.uint8)
    want = buf.copy()
    register(core, [buf])
    d["rmul8"](buf.ctypes.data, 77, size, None, 0)
    ref["rmul8"](want.ctypes.data, 77, size, None, 0)
    run.check(np.array_equal(buf, want), "pinned in-place region multiply")


def fill_hbm(hip, leave=16 << 20):
    """Allocates device memory until less than `leave` bytes are free, so the
    library's own staging hipMalloc (tens of MiB for a C3 call) fails for real
    (SURVEY §8b's contract on a genuine HIP error, not an injected one) while
    the HIP runtime keeps the few MiB its own bookkeeping needs (with HBM
    exhausted to the last MiB the runtime itself crashed, round 6).  Returns
    the byte count held and the allocations."""
    hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    hip.hipMemGetInfo.argtypes = [ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t)]
    free, total = ctypes.c_size_t(), ctypes.c_size_t()
    held, keep = 0, []
    chunk = 64 << 30
    while chunk >= (1 << 20):
        assert hip.hipMemGetInfo(ctypes.byref(free), ctypes.byref(total)) == 0
        if free.value < leave + chunk:
            chunk //= 2
            continue
        p = ctypes.c_void_p()
        if hip.hipMalloc(ctypes.byref(p), chunk) == 0:
            keep.append(p)
            held += chunk
        else:
            hip.hipGetLastError()
            chunk //= 2
    return held, keep


def oom(d, core, golden, run):
    """The client's C3 calls (client_main.cpp:1060, :2118) on one malloc'd
    stripe buffer with HBM full: every staging hipMalloc fails."""
    hip = ctypes.CDLL("libamdhip64.so.7")  # the runtime libecgpu.so is bound to (already loaded)
    k, m, size = 10, 4, 4 << 20
    M = matrix(d, k, m)
    # warm the library first (context, stream, the inline kernels' code
    # object): the same calls at 64 KiB shards, staged in coherent pinned host
    # memory (no HBM), on the GPU whatever the small-call threshold
    core.ecgpu_set_knob.argtypes = [ctypes.c_char_p, ctypes.c_int]
    core.ecgpu_set_knob(b"ECGPU_MIN_OFFLOAD_KIB", 0)
    small = [np.full(64 << 10, i, np.uint8) for i in range(k + m)]
    d["encode"](k, m, 8, ints(M), ptrs(small[:k]), ptrs(small[k:]), 64 << 10)
    assert d["decode"](k, m, 8, ints(M), 0, ints([0, 1, 2, 3, -1]), ptrs(small[:k]), ptrs(small[k:]), 64 << 10) == 0
    core.ecgpu_reset_knob.argtypes = [ctypes.c_char_p]
    core.ecgpu_reset_knob(b"ECGPU_MIN_OFFLOAD_KIB")
    print("oom: library warm", file=sys.stderr, flush=True)
    held, keep = fill_hbm(hip)
    run.held = held
    print(f"oom: {held >> 20} MiB of HBM held", file=sys.stderr, flush=True)
    slab = np.zeros((k + m) * size, np.uint8)
    sh = [slab[i * size:(i + 1) * size] for i in range(k + m)]
    for i in range(k):
        sh[i][:] = splitmix_bytes(size, shard_seed(3, 0, i))
    d["encode"](k, m, 8, ints(M), ptrs(sh[:k]), ptrs(sh[k:]), size)
    run.check([fnv1a64(c) for c in sh[k:]] == golden["full_size"]["C3"]["coding"], "C3 4 MiB encode digests (HBM full)")
    keep_data = [s.copy() for s in sh[:4]]
    for s in sh[:4]:
        s[:] = 0xEE
    rc = d["decode"](k, m, 8, ints(M), 0, ints([0, 1, 2, 3, -1]), ptrs(sh[:k]), ptrs(sh[k:]), size)
    run.check(rc == 0 and all(np.array_equal(a, b) for a, b in zip(sh[:4], keep_data)),
              "C3 4 MiB decode{0,1,2,3} (HBM full)")
    hip.hipFree.argtypes = [ctypes.c_void_p]
    for p in keep:
        hip.hipFree(p)


def main():
    import faulthandler
    faulthandler.enable()  # a crash names the line it happened on
    scenario = sys.argv[1]
    with open(os.path.join(TESTS, "golden", "golden.json")) as fh:
        golden = json.load(fh)
    d = bind(os.path.join(LIB, "libjerasure_amd.so"))
    core = ctypes.CDLL(os.path.join(LIB, "libecgpu.so"))  # the instance the drop-in links
    set_injection(core)
    run = Run(scenario)
    if scenario == "client":
        client(d, golden, run)
    elif scenario == "ecx":
        ecx(d, bind(os.path.join(REF, "libjerasure_ref.so")), golden, run)
    elif scenario == "surface":
        surface(d, bind(os.path.join(REF, "libjerasure_ref.so")), bind(os.path.join(REF, "libjerasure_ref_nsa.so")),
                run)
    elif scenario == "pinned":
        pinned(d, bind(os.path.join(REF, "libjerasure_ref.so")), core, run)
    elif scenario == "pinned_alias":
        pinned_alias(d, bind(os.path.join(REF, "libjerasure_ref.so")), core, run)
    elif scenario == "oom":
        oom(d, core, golden, run)
    else:
        raise SystemExit(f"unknown scenario {scenario}")
    core.ecgpu_fallback_count.restype = ctypes.c_int64
    core.ecgpu_cpu_call_count.restype = ctypes.c_int64
    core.ecgpu_device_lost.restype = ctypes.c_int
    print(json.dumps({"scenario": scenario, "checked": run.checked, "mismatches": run.mismatches[:20],
                      "fallbacks": int(core.ecgpu_fallback_count()), "cpu_calls": int(core.ecgpu_cpu_call_count()),
                      "lost": int(core.ecgpu_device_lost(0)), "hbm_held": getattr(run, "held", None)}),
          flush=True)
    return 0 if not run.mismatches else 3


if __name__ == "__main__":
    sys.exit(main())
