"""jerasure.h surface (reference include/jerasure.h:113-282) over the C ABI.

Same names, argument order and meaning as the reference:
``data_ptrs`` / ``coding_ptrs`` are sequences of k / m shard buffers (CUDA
tensors are used in place; CPU tensors or numpy arrays are staged through
HBM), ``matrix`` is the flat row-major m x k coding matrix, ``erasures`` the
erased ids (a trailing -1 is optional).  Encode/decode/dotprod run on the
MI355X for w = 8, 16 and 32 (w = 16 / 32: size a whole number of words) and
are synchronous; a HIP failure raises ``EcgpuError`` (the C library's CPU
fallback is off in this package unless ECGPU_CPU_FALLBACK is set).  Where the reference calls exit(1) (bad w) this raises
ValueError; where it returns -1 this returns -1.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

from . import _native as N
from ._buffers import addr, addrs


def _erasure_list(erasures: Sequence[int]) -> list:
    er = [int(e) for e in erasures]
    if not er or er[-1] != -1:
        er.append(-1)
    return er


def jerasure_matrix_encode(k: int, m: int, w: int, matrix, data_ptrs, coding_ptrs, size: int) -> None:
    if w not in (8, 16, 32):
        raise ValueError("jerasure_matrix_encode: w must be 8, 16 or 32")
    rc = N.lib.ecgpu_jerasure_matrix_encode(k, m, w, N.int_array(matrix), N.ptr_array(addrs(data_ptrs)),
                                            N.ptr_array(addrs(coding_ptrs)), size)
    N.check(rc, "jerasure_matrix_encode")


def jerasure_matrix_decode(k: int, m: int, w: int, matrix, row_k_ones: int, erasures, data_ptrs, coding_ptrs,
                           size: int) -> int:
    if w not in (8, 16, 32):
        return -1  # jerasure.cpp:165
    rc = N.lib.ecgpu_jerasure_matrix_decode(k, m, w, N.int_array(matrix), row_k_ones,
                                            N.int_array(_erasure_list(erasures)), N.ptr_array(addrs(data_ptrs)),
                                            N.ptr_array(addrs(coding_ptrs)), size)
    return N.check(rc, "jerasure_matrix_decode")


def jerasure_matrix_dotprod(k: int, w: int, matrix_row, src_ids: Optional[Sequence[int]], dest_id: int, data_ptrs,
                            coding_ptrs, size: int) -> None:
    if w not in (1, 8, 16, 32):  # jerasure.cpp:569-572
        raise ValueError("jerasure_matrix_dotprod: w must be 1, 8, 16 or 32")
    ids = None if src_ids is None else N.int_array(src_ids)
    rc = N.lib.ecgpu_jerasure_matrix_dotprod(k, w, N.int_array(matrix_row), ids, dest_id,
                                             N.ptr_array(addrs(data_ptrs)), N.ptr_array(addrs(coding_ptrs)), size)
    N.check(rc, "jerasure_matrix_dotprod")


def jerasure_do_parity(k: int, data_ptrs, parity_ptr, size: int) -> None:
    N.check(N.lib.ecgpu_jerasure_do_parity(k, N.ptr_array(addrs(data_ptrs)), addr(parity_ptr), size),
            "jerasure_do_parity")


def jerasure_make_decoding_matrix(k: int, m: int, w: int, matrix, erased) -> Tuple[int, List[int], List[int]]:
    dm, ids = (N.c_int * (k * k))(), (N.c_int * k)()
    rc = N.lib.ecgpu_jerasure_make_decoding_matrix(k, m, w, N.int_array(matrix), N.int_array(erased), dm, ids)
    return rc, list(dm), list(ids)


def jerasure_invert_matrix(mat, rows: int, w: int) -> Tuple[int, List[int], List[int]]:
    """Returns (rc, inverse, mat-after) -- the reference destroys mat in place."""
    a, inv = N.int_array(mat), (N.c_int * (rows * rows))()
    rc = N.lib.ecgpu_jerasure_invert_matrix(a, inv, rows, w)
    return rc, list(inv), list(a)[: rows * rows]


def jerasure_invertible_matrix(mat, rows: int, w: int) -> int:
    return N.lib.ecgpu_jerasure_invertible_matrix(N.int_array(mat), rows, w)


def jerasure_erasures_to_erased(k: int, m: int, erasures) -> Optional[List[int]]:
    return N.take_int_matrix(N.lib.ecgpu_jerasure_erasures_to_erased(k, m, N.int_array(_erasure_list(erasures))),
                             k + m)


def jerasure_matrix_multiply(m1, m2, r1: int, c1: int, r2: int, c2: int, w: int) -> List[int]:
    return N.take_int_matrix(N.lib.ecgpu_jerasure_matrix_multiply(N.int_array(m1), N.int_array(m2), r1, c1, r2, c2,
                                                                  w), r1 * c2)


def jerasure_get_stats() -> List[float]:
    """[bytes XORed, bytes GF-multiplied, bytes copied] since the last call (jerasure.cpp:1143-1151 order)."""
    out = (N.ctypes.c_double * 3)()
    N.lib.ecgpu_jerasure_get_stats(out)
    return list(out)


def decode_plan(k: int, m: int, matrix, erasures, row_k_ones: int = 0):
    """The single fused linear map jerasure_matrix_decode applies: returns
    (out_ids, src_ids, coefs[n_out][n_src]) over shard ids, or None where the
    reference decode returns -1."""
    n = k + m
    out_ids, src_ids = (N.c_int * n)(), (N.c_int * n)()
    n_out, n_src = N.c_int(0), N.c_int(0)
    coefs = (N.c_int * (n * n))()
    rc = N.lib.ecgpu_decode_plan(k, m, 8, N.int_array(matrix), row_k_ones, N.int_array(_erasure_list(erasures)),
                                 out_ids, N.ctypes.byref(n_out), src_ids, N.ctypes.byref(n_src), coefs)
    if rc == N.ECGPU_ERR:
        return None
    N.check(rc, "ecgpu_decode_plan")
    no, ns = n_out.value, n_src.value
    return (list(out_ids)[:no], list(src_ids)[:ns], [list(coefs[r * ns:(r + 1) * ns]) for r in range(no)])


# ------------------------------------------------ GF(2) bit-matrix coding ----
# jerasure.cpp:257-345, :623-703, :1034-1124, :1153-1192, :1346-1363.  The
# matrices are host math; encode / decode / schedules execute on the MI355X as
# one fused GF(2) packet map per call (size must be whole super-packets,
# size % (w * packetsize) == 0).  A schedule is a list of 5-tuples
# (src device, src packet, dst device, dst packet, xor?) -- the reference's
# int** operations without the -1 terminator.

def jerasure_matrix_to_bitmatrix(k: int, m: int, w: int, matrix) -> Optional[List[int]]:
    return N.take_int_matrix(N.lib.ecgpu_jerasure_matrix_to_bitmatrix(k, m, w, N.int_array(matrix)),
                             k * m * w * w)


def jerasure_make_decoding_bitmatrix(k: int, m: int, w: int, matrix, erased) -> Tuple[int, List[int], List[int]]:
    n = k * w * k * w
    dm, ids = (N.c_int * n)(), (N.c_int * k)()
    rc = N.lib.ecgpu_jerasure_make_decoding_bitmatrix(k, m, w, N.int_array(matrix), N.int_array(erased), dm, ids)
    return rc, list(dm), list(ids)


def jerasure_invert_bitmatrix(mat, rows: int) -> Tuple[int, List[int]]:
    inv = (N.c_int * (rows * rows))()
    return N.lib.ecgpu_jerasure_invert_bitmatrix(N.int_array(mat), inv, rows), list(inv)


def jerasure_invertible_bitmatrix(mat, rows: int) -> int:
    return N.lib.ecgpu_jerasure_invertible_bitmatrix(N.int_array(mat), rows)


def _check_packets(fn: str, size: int, w: int, packetsize: int) -> None:
    if packetsize <= 0 or size % (w * packetsize):
        raise ValueError(f"{fn}: size % (w*packetsize) must be 0")


def jerasure_bitmatrix_dotprod(k: int, w: int, bitmatrix_row, src_ids: Optional[Sequence[int]], dest_id: int,
                               data_ptrs, coding_ptrs, size: int, packetsize: int) -> None:
    _check_packets("jerasure_bitmatrix_dotprod", size, w, packetsize)
    ids = None if src_ids is None else N.int_array(src_ids)
    N.check(N.lib.ecgpu_jerasure_bitmatrix_dotprod(k, w, N.int_array(bitmatrix_row), ids, dest_id,
                                                   N.ptr_array(addrs(data_ptrs)), N.ptr_array(addrs(coding_ptrs)),
                                                   size, packetsize), "jerasure_bitmatrix_dotprod")


def jerasure_bitmatrix_encode(k: int, m: int, w: int, bitmatrix, data_ptrs, coding_ptrs, size: int,
                              packetsize: int) -> None:
    _check_packets("jerasure_bitmatrix_encode", size, w, packetsize)
    N.check(N.lib.ecgpu_jerasure_bitmatrix_encode(k, m, w, N.int_array(bitmatrix), N.ptr_array(addrs(data_ptrs)),
                                                  N.ptr_array(addrs(coding_ptrs)), size, packetsize),
            "jerasure_bitmatrix_encode")


def jerasure_bitmatrix_decode(k: int, m: int, w: int, bitmatrix, row_k_ones: int, erasures, data_ptrs, coding_ptrs,
                              size: int, packetsize: int) -> int:
    _check_packets("jerasure_bitmatrix_decode", size, w, packetsize)
    rc = N.lib.ecgpu_jerasure_bitmatrix_decode(k, m, w, N.int_array(bitmatrix), row_k_ones,
                                               N.int_array(_erasure_list(erasures)), N.ptr_array(addrs(data_ptrs)),
                                               N.ptr_array(addrs(coding_ptrs)), size, packetsize)
    return N.check(rc, "jerasure_bitmatrix_decode")


class _Schedule:
    """A schedule as the reference's int** (malloc-free: ctypes-owned rows)."""

    def __init__(self, ops):
        self.rows = [(N.c_int * 5)(*op) for op in ops] + [(N.c_int * 5)(-1, 0, 0, 0, 0)]
        self.table = (N.c_void_p * len(self.rows))(*[N.ctypes.addressof(r) for r in self.rows])


def jerasure_do_scheduled_operations(ptrs, operations, packetsize: int) -> None:
    sched = _Schedule(operations)
    N.check(N.lib.ecgpu_jerasure_do_scheduled_operations(N.ptr_array(addrs(ptrs)), sched.table, packetsize),
            "jerasure_do_scheduled_operations")


def jerasure_schedule_encode(k: int, m: int, w: int, schedule, data_ptrs, coding_ptrs, size: int,
                             packetsize: int) -> None:
    _check_packets("jerasure_schedule_encode", size, w, packetsize)
    sched = _Schedule(schedule)
    N.check(N.lib.ecgpu_jerasure_schedule_encode(k, m, w, sched.table, N.ptr_array(addrs(data_ptrs)),
                                                 N.ptr_array(addrs(coding_ptrs)), size, packetsize),
            "jerasure_schedule_encode")


def _take_schedule(addr: int) -> List[Tuple[int, int, int, int, int]]:
    """Copy a malloc'd int** schedule into tuples and free it."""
    if not addr:
        return None
    rows = N.ctypes.cast(addr, N.ctypes.POINTER(N.ctypes.POINTER(N.c_int)))
    ops, i = [], 0
    while rows[i][0] >= 0:
        ops.append(tuple(rows[i][j] for j in range(5)))
        i += 1
    N.lib.ecgpu_jerasure_free_schedule(addr)
    return ops


def jerasure_dumb_bitmatrix_to_schedule(k: int, m: int, w: int, bitmatrix) -> List[Tuple[int, int, int, int, int]]:
    """jerasure.cpp:1194-1224: one copy then XORs per output packet row."""
    return _take_schedule(N.lib.ecgpu_jerasure_dumb_bitmatrix_to_schedule(k, m, w, N.int_array(bitmatrix)))


def jerasure_smart_bitmatrix_to_schedule(k: int, m: int, w: int, bitmatrix) -> List[Tuple[int, int, int, int, int]]:
    """jerasure.cpp:1226-1344: rows built from an earlier row where cheaper."""
    return _take_schedule(N.lib.ecgpu_jerasure_smart_bitmatrix_to_schedule(k, m, w, N.int_array(bitmatrix)))


def jerasure_schedule_decode_lazy(k: int, m: int, w: int, bitmatrix, erasures, data_ptrs, coding_ptrs, size: int,
                                  packetsize: int, smart: int) -> int:
    """jerasure.cpp:935-961: decoding schedule built on the host, run on the MI355X."""
    _check_packets("jerasure_schedule_decode_lazy", size, w, packetsize)
    rc = N.lib.ecgpu_jerasure_schedule_decode_lazy(k, m, w, N.int_array(bitmatrix),
                                                   N.int_array(_erasure_list(erasures)), N.ptr_array(addrs(data_ptrs)),
                                                   N.ptr_array(addrs(coding_ptrs)), size, packetsize, smart)
    return N.check(rc, "jerasure_schedule_decode_lazy")


class ScheduleCache:
    """jerasure_generate_schedule_cache (jerasure.cpp:997-1032; m must be 2):
    decoding schedules for every one- and two-erasure pattern."""

    def __init__(self, k: int, m: int, w: int, bitmatrix, smart: int = 1):
        self.k, self.m, self.w = k, m, w
        self._c = N.lib.ecgpu_jerasure_generate_schedule_cache(k, m, w, N.int_array(bitmatrix), smart)
        if not self._c:
            raise ValueError("jerasure_generate_schedule_cache: m must be 2")

    def decode(self, erasures, data_ptrs, coding_ptrs, size: int, packetsize: int) -> int:
        """jerasure_schedule_decode_cache (jerasure.cpp:963-995); -1 for more than two erasures."""
        _check_packets("jerasure_schedule_decode_cache", size, self.w, packetsize)
        rc = N.lib.ecgpu_jerasure_schedule_decode_cache(self.k, self.m, self.w, self._c,
                                                        N.int_array(_erasure_list(erasures)),
                                                        N.ptr_array(addrs(data_ptrs)), N.ptr_array(addrs(coding_ptrs)),
                                                        size, packetsize)
        return N.check(rc, "jerasure_schedule_decode_cache")

    def close(self) -> None:
        if getattr(self, "_c", None):
            N.lib.ecgpu_jerasure_free_schedule_cache(self.k, self.m, self._c)
            self._c = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# The reference's names for the schedule-cache and schedule lifetime calls
# (jerasure.h:116-119, :185).  Schedules here are Python lists, so freeing one is a
# no-op; a cache owns C memory and is released by jerasure_free_schedule_cache
# (or when it is garbage-collected).
def jerasure_generate_schedule_cache(k: int, m: int, w: int, bitmatrix, smart: int) -> Optional[ScheduleCache]:
    """jerasure.cpp:997-1032: None (the reference's NULL) unless m == 2."""
    try:
        return ScheduleCache(k, m, w, bitmatrix, smart)
    except ValueError:
        return None


def jerasure_schedule_decode_cache(k: int, m: int, w: int, scache: ScheduleCache, erasures, data_ptrs, coding_ptrs,
                                   size: int, packetsize: int) -> int:
    """jerasure.cpp:963-995 with a cache from jerasure_generate_schedule_cache."""
    if (scache.k, scache.m, scache.w) != (k, m, w):
        raise ValueError("jerasure_schedule_decode_cache: cache was built for another (k, m, w)")
    return scache.decode(erasures, data_ptrs, coding_ptrs, size, packetsize)


def jerasure_free_schedule_cache(k: int, m: int, cache: Optional[ScheduleCache]) -> None:
    """jerasure.cpp:543-560."""
    if cache is not None:
        cache.close()


def jerasure_free_schedule(schedule) -> None:
    """jerasure.cpp:534-541: schedules are Python lists here; nothing to free."""


def jerasure_print_matrix(matrix, rows: int, cols: int, w: int, file=None) -> None:
    """jerasure.cpp:46-68: entries as unsigned ints right-aligned to the width
    of 2^w - 1 (10 for w = 32), one row per line."""
    import sys
    out = file or sys.stdout
    fw = 10 if w == 32 else len(str((1 << w) - 1))
    for i in range(rows):
        out.write(" ".join(f"{matrix[i * cols + j] & 0xFFFFFFFF:>{fw}}" for j in range(cols)) + "\n")


def jerasure_print_bitmatrix(bitmatrix, rows: int, cols: int, w: int, file=None) -> None:
    """jerasure.cpp:70-82: w x w blocks, a space between block columns and an
    empty line between block rows."""
    import sys
    out = file or sys.stdout
    for i in range(rows):
        if i and i % w == 0:
            out.write("\n")
        out.write("".join((" " if j and j % w == 0 else "") + str(bitmatrix[i * cols + j]) for j in range(cols)) + "\n")
