"""ctypes front-end to the parity checker.  TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline
leg may import this module; the product package ``erasure_coding_test_amd``
never does.

Two interchangeable back-ends with one interface:

* :class:`Restatement` -- ``oracle/libecoracle.so``, our C restatement of the
  reference's w=8 path (``oracle/ec_oracle.c``; every function cites the
  reference file:line it follows).
* :class:`Reference` -- ``oracle/_ref/libjerasure_ref.so``, the reference's own
  ``src/erasure_coding/{galois,jerasure,reed_sol}.cpp`` compiled unchanged by
  ``oracle/Makefile`` (C++-mangled symbols, bound here by mangled name).

Buffers are numpy ``uint8`` arrays.  The reference's 8-byte loops over-run
sizes that are not a multiple of 8 (galois.cpp:452-465, :748-753), so callers
that hand ragged sizes to :class:`Reference` must pad every buffer by >= 8
bytes (:func:`alloc_shards` does).
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
RESTATEMENT_SO = os.path.join(HERE, "libecoracle.so")
REFERENCE_SO = os.path.join(HERE, "_ref", "libjerasure_ref.so")
REFERENCE_O3_SO = os.path.join(HERE, "_ref", "libjerasure_ref_o3.so")  # -O3 -march=x86-64-v3

_c_int_p = ctypes.POINTER(ctypes.c_int)
_libc = ctypes.CDLL(None)
_libc.free.argtypes = [ctypes.c_void_p]


def _ptrs(arrays: Sequence[np.ndarray]):
    arr = (ctypes.c_void_p * max(1, len(arrays)))()
    for i, a in enumerate(arrays):
        arr[i] = a.ctypes.data
    return arr


def _ints(values) -> ctypes.Array:
    vals = [int(v) for v in np.asarray(values).ravel()]
    arr = (ctypes.c_int * max(1, len(vals)))()
    for i, v in enumerate(vals):
        arr[i] = v
    return arr


def alloc_shards(n: int, size: int, pad: int = 16) -> list:
    """n zeroed shards of `size` bytes, each with `pad` spare bytes behind it."""
    return [np.zeros(size + pad, dtype=np.uint8) for _ in range(n)]


# --------------------------------------------------------------------------
class Restatement:
    """oracle/ec_oracle.c through ctypes."""

    kind = "port"

    def __init__(self, path: str = RESTATEMENT_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: run `make -C oracle`")
        L = ctypes.CDLL(path)
        self.L = L
        for name in ("orc_gf_mul", "orc_gf_div"):
            getattr(L, name).argtypes = [ctypes.c_int, ctypes.c_int]
            getattr(L, name).restype = ctypes.c_int
        for name in ("orc_gf_inverse", "orc_gf_log", "orc_gf_ilog"):
            getattr(L, name).argtypes = [ctypes.c_int]
            getattr(L, name).restype = ctypes.c_int
        L.orc_vandermonde_coding_matrix.argtypes = [ctypes.c_int, ctypes.c_int, _c_int_p]
        L.orc_invert_matrix.argtypes = [_c_int_p, _c_int_p, ctypes.c_int]
        L.orc_make_decoding_matrix.argtypes = [ctypes.c_int, ctypes.c_int, _c_int_p, _c_int_p, _c_int_p, _c_int_p]
        L.orc_erasures_to_erased.argtypes = [ctypes.c_int, ctypes.c_int, _c_int_p, _c_int_p]
        L.orc_region_multiply.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_long, ctypes.c_void_p, ctypes.c_int]
        L.orc_region_multiply.restype = None
        L.orc_region_xor.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long]
        L.orc_region_xor.restype = None
        pp = ctypes.POINTER(ctypes.c_void_p)
        L.orc_matrix_dotprod.argtypes = [ctypes.c_int, _c_int_p, _c_int_p, ctypes.c_int, pp, pp, ctypes.c_long]
        L.orc_matrix_dotprod.restype = None
        L.orc_matrix_encode.argtypes = [ctypes.c_int, ctypes.c_int, _c_int_p, pp, pp, ctypes.c_long]
        L.orc_matrix_encode.restype = None
        L.orc_matrix_encode_mt.argtypes = [ctypes.c_int, ctypes.c_int, _c_int_p, pp, pp, ctypes.c_long, ctypes.c_int]
        L.orc_matrix_decode.argtypes = [ctypes.c_int, ctypes.c_int, _c_int_p, ctypes.c_int, _c_int_p, pp, pp, ctypes.c_long]
        L.orc_splitmix_fill.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_uint64]
        L.orc_splitmix_fill.restype = None
        L.orc_fnv1a64.argtypes = [ctypes.c_void_p, ctypes.c_long]
        L.orc_fnv1a64.restype = ctypes.c_uint64

    # -- scalar ---------------------------------------------------------
    def gf_mul(self, a, b): return self.L.orc_gf_mul(a, b)
    def gf_div(self, a, b): return self.L.orc_gf_div(a, b)
    def gf_inverse(self, a): return self.L.orc_gf_inverse(a)
    def gf_log(self, v): return self.L.orc_gf_log(v)
    def gf_ilog(self, v): return self.L.orc_gf_ilog(v)

    # -- matrices -------------------------------------------------------
    def vandermonde_coding_matrix(self, k: int, m: int) -> Optional[np.ndarray]:
        out = (ctypes.c_int * (k * m))()
        if self.L.orc_vandermonde_coding_matrix(k, m, out) != 0:
            return None
        return np.frombuffer(out, dtype=np.int32).copy().reshape(m, k)

    def invert_matrix(self, mat: np.ndarray):
        n = mat.shape[0]
        a, inv = _ints(mat), (ctypes.c_int * (n * n))()
        rc = self.L.orc_invert_matrix(a, inv, n)
        return rc, np.frombuffer(inv, dtype=np.int32).copy().reshape(n, n)

    def make_decoding_matrix(self, k: int, m: int, matrix: np.ndarray, erased: Sequence[int]):
        dm, ids = (ctypes.c_int * (k * k))(), (ctypes.c_int * k)()
        rc = self.L.orc_make_decoding_matrix(k, m, _ints(matrix), _ints(erased), dm, ids)
        return rc, np.frombuffer(dm, dtype=np.int32).copy().reshape(k, k), list(ids)

    # -- regions --------------------------------------------------------
    def region_multiply(self, src, c, n, r2, add):
        self.L.orc_region_multiply(src.ctypes.data, c, n, None if r2 is None else r2.ctypes.data, add)

    def region_xor(self, r1, r2, r3, n):
        self.L.orc_region_xor(r1.ctypes.data, r2.ctypes.data, r3.ctypes.data, n)

    def matrix_dotprod(self, k, row, src_ids, dest_id, data, coding, size):
        ids = None if src_ids is None else _ints(src_ids)
        self.L.orc_matrix_dotprod(k, _ints(row), ids, dest_id, _ptrs(data), _ptrs(coding), size)

    def matrix_encode(self, k, m, matrix, data, coding, size):
        self.L.orc_matrix_encode(k, m, _ints(matrix), _ptrs(data), _ptrs(coding), size)

    def matrix_encode_mt(self, k, m, matrix, data, coding, size, nthreads):
        return self.L.orc_matrix_encode_mt(k, m, _ints(matrix), _ptrs(data), _ptrs(coding), size, nthreads)

    def matrix_decode(self, k, m, matrix, row_k_ones, erasures, data, coding, size):
        er = list(erasures) + [-1]
        return self.L.orc_matrix_decode(k, m, _ints(matrix), row_k_ones, _ints(er), _ptrs(data), _ptrs(coding), size)

    # -- synthetic data -------------------------------------------------
    def fill(self, buf: np.ndarray, seed: int, n: Optional[int] = None):
        self.L.orc_splitmix_fill(buf.ctypes.data, buf.size if n is None else n, seed & (2**64 - 1))

    def fnv1a64(self, buf: np.ndarray, n: Optional[int] = None) -> int:
        return int(self.L.orc_fnv1a64(buf.ctypes.data, buf.size if n is None else n))


# --------------------------------------------------------------------------
class Reference:
    """The reference coding library compiled from /root/reference (w=8 calls)."""

    kind = "reference"
    W = 8

    def __init__(self, path: str = REFERENCE_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: build with `make -C oracle` where /root/reference exists")
        L = ctypes.CDLL(path)
        self.L = L
        pp = ctypes.POINTER(ctypes.c_void_p)
        i = ctypes.c_int

        def bind(mangled, args, res=ctypes.c_int):
            f = getattr(L, mangled)
            f.argtypes, f.restype = args, res
            return f

        self._mul = bind("_Z22galois_single_multiplyiii", [i, i, i])
        self._div = bind("_Z20galois_single_divideiii", [i, i, i])
        self._inv = bind("_Z14galois_inverseii", [i, i])
        self._log = bind("_Z10galois_logii", [i, i])
        self._ilog = bind("_Z11galois_ilogii", [i, i])
        self._vdm = bind("_Z34reed_sol_vandermonde_coding_matrixiii", [i, i, i], ctypes.c_void_p)
        self._r6 = bind("_Z25reed_sol_r6_coding_matrixii", [i, i], ctypes.c_void_p)
        self._invert = bind("_Z22jerasure_invert_matrixPiS_ii", [_c_int_p, _c_int_p, i, i])
        self._mkdec = bind("_Z29jerasure_make_decoding_matrixiiiPiS_S_S_", [i, i, i, _c_int_p, _c_int_p, _c_int_p, _c_int_p])
        self._rmul = bind("_Z26galois_w08_region_multiplyPciiS_i", [ctypes.c_void_p, i, i, ctypes.c_void_p, i], None)
        self._rxor = bind("_Z17galois_region_xorPcS_S_i", [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, i], None)
        self._dot = bind("_Z23jerasure_matrix_dotprodiiPiS_iPPcS1_i", [i, i, _c_int_p, _c_int_p, i, pp, pp, i], None)
        self._enc = bind("_Z22jerasure_matrix_encodeiiiPiPPcS1_i", [i, i, i, _c_int_p, pp, pp, i], None)
        self._dec = bind("_Z22jerasure_matrix_decodeiiiPiiS_PPcS1_i", [i, i, i, _c_int_p, i, _c_int_p, pp, pp, i])
        self._stats = bind("_Z18jerasure_get_statsPd", [ctypes.POINTER(ctypes.c_double)], None)
        self._r6enc = bind("_Z18reed_sol_r6_encodeiiPPcS0_i", [i, i, pp, pp, i])

    def gf_mul(self, a, b): return self._mul(a, b, 8)
    def gf_div(self, a, b): return self._div(a, b, 8)
    def gf_inverse(self, a): return self._inv(a, 8)
    def gf_log(self, v): return self._log(v, 8)
    def gf_ilog(self, v): return self._ilog(v, 8)

    def _take_matrix(self, p, rows, cols):
        if not p:
            return None
        out = np.ctypeslib.as_array(ctypes.cast(p, _c_int_p), shape=(rows * cols,)).astype(np.int32).reshape(rows, cols)
        _libc.free(p)
        return out

    def vandermonde_coding_matrix(self, k, m):
        return self._take_matrix(self._vdm(k, m, 8), m, k)

    def r6_coding_matrix(self, k):
        return self._take_matrix(self._r6(k, 8), 2, k)

    def invert_matrix(self, mat):
        n = mat.shape[0]
        a, inv = _ints(mat), (ctypes.c_int * (n * n))()
        rc = self._invert(a, inv, n, 8)
        return rc, np.frombuffer(inv, dtype=np.int32).copy().reshape(n, n)

    def make_decoding_matrix(self, k, m, matrix, erased):
        dm, ids = (ctypes.c_int * (k * k))(), (ctypes.c_int * k)()
        rc = self._mkdec(k, m, 8, _ints(matrix), _ints(erased), dm, ids)
        return rc, np.frombuffer(dm, dtype=np.int32).copy().reshape(k, k), list(ids)

    def region_multiply(self, src, c, n, r2, add):
        self._rmul(src.ctypes.data, c, n, None if r2 is None else r2.ctypes.data, add)

    def region_xor(self, r1, r2, r3, n):
        self._rxor(r1.ctypes.data, r2.ctypes.data, r3.ctypes.data, n)

    def matrix_dotprod(self, k, row, src_ids, dest_id, data, coding, size):
        ids = None if src_ids is None else _ints(src_ids)
        self._dot(k, 8, _ints(row), ids, dest_id, _ptrs(data), _ptrs(coding), size)

    def matrix_encode(self, k, m, matrix, data, coding, size):
        self._enc(k, m, 8, _ints(matrix), _ptrs(data), _ptrs(coding), size)

    def matrix_decode(self, k, m, matrix, row_k_ones, erasures, data, coding, size):
        er = list(erasures) + [-1]
        return self._dec(k, m, 8, _ints(matrix), row_k_ones, _ints(er), _ptrs(data), _ptrs(coding), size)

    def r6_encode(self, k, data, coding, size):
        return self._r6enc(k, 8, _ptrs(data), _ptrs(coding), size)

    def get_stats(self):
        d = (ctypes.c_double * 3)()
        self._stats(d)
        return list(d)


def shard_seed(cfg: int, stripe: int, shard: int) -> int:
    """SURVEY.md §8d seed: 0xEC00_0000 ^ (cfg<<32) ^ (stripe<<8) ^ shard."""
    return (0xEC000000 ^ (cfg << 32) ^ (stripe << 8) ^ shard) & (2**64 - 1)


def best_available():
    """The compiled reference when its build exists, else the restatement."""
    try:
        return Reference()
    except (FileNotFoundError, OSError):
        return Restatement()
