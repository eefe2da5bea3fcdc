"""galois.h surface (reference include/galois.h:41-95) over the C ABI.

Scalar field ops run on the host (csrc/gf_host.cpp); the region ops run on
the MI355X.  Where the reference prints an error and exits (log tables for
w > 30) the mirror raises ValueError.
"""
from __future__ import annotations

from . import _native as N
from ._buffers import addr


def galois_single_multiply(a: int, b: int, w: int) -> int:
    """a * b in GF(2^w) (galois.cpp:322-360)."""
    return N.lib.ecgpu_galois_single_multiply(a, b, w)


def galois_single_divide(a: int, b: int, w: int) -> int:
    """a / b in GF(2^w); -1 for b = 0 (galois.cpp:367-398)."""
    return N.lib.ecgpu_galois_single_divide(a, b, w)


def galois_inverse(a: int, w: int) -> int:
    """1 / a in GF(2^w); -1 for a = 0 (galois.cpp:597-603)."""
    return N.lib.ecgpu_galois_inverse(a, w)


def _log_width(fn: str, w: int) -> None:
    if not 1 <= w <= 30:  # galois.cpp:273-274, 284-285: "w is too big", exit(1)
        raise ValueError(f"{fn}: w = {w} has no log tables (w <= 30)")


def galois_log(value: int, w: int) -> int:
    """Discrete log of value, 0 <= value < 2^w (galois.cpp:280-289)."""
    _log_width("galois_log", w)
    if not 0 <= value < (1 << w):
        raise ValueError(f"galois_log: value {value} outside [0, 2^{w})")
    return N.lib.ecgpu_galois_log(value, w)


def galois_ilog(value: int, w: int) -> int:
    """Antilog, -(2^w - 1) <= value < 2(2^w - 1) like the reference's offset table (galois.cpp:269-278)."""
    _log_width("galois_ilog", w)
    nwm1 = (1 << w) - 1
    if not -nwm1 <= value < 2 * nwm1:
        raise ValueError(f"galois_ilog: value {value} outside [-{nwm1}, {2 * nwm1})")
    return N.lib.ecgpu_galois_ilog(value, w)


def galois_create_log_tables(w: int) -> int:
    """0, or -1 where the reference cannot build them (w > 30) (galois.cpp:152-191)."""
    return N.lib.ecgpu_galois_create_log_tables(w)


def galois_create_mult_tables(w: int) -> int:
    """0, or -1 for w >= 14 (galois.cpp:218-267)."""
    return N.lib.ecgpu_galois_create_mult_tables(w)


def galois_create_split_w8_tables() -> int:
    """Builds the seven byte-pair product tables of GF(2^32) once: 0, or -1 if
    they cannot be allocated (galois.cpp:756-789)."""
    return N.lib.ecgpu_galois_create_split_w8_tables()


def galois_logtable_multiply(x: int, y: int, w: int) -> int:
    """galois.cpp:193-203 (the product, whichever table computes it)."""
    return 0 if x == 0 or y == 0 else N.lib.ecgpu_galois_single_multiply(x, y, w)


def galois_logtable_divide(x: int, y: int, w: int) -> int:
    """galois.cpp:205-216: -1 for y = 0."""
    return N.lib.ecgpu_galois_single_divide(x, y, w)


def galois_multtable_multiply(x: int, y: int, w: int) -> int:
    """galois.cpp:362-365."""
    return N.lib.ecgpu_galois_single_multiply(x, y, w)


def galois_multtable_divide(x: int, y: int, w: int) -> int:
    """galois.cpp:410-413."""
    return N.lib.ecgpu_galois_single_divide(x, y, w)


def galois_shift_multiply(x: int, y: int, w: int) -> int:
    """Table-free shift-and-reduce multiply (galois.cpp:292-320)."""
    return N.lib.ecgpu_galois_shift_multiply(x, y, w)


def galois_shift_inverse(y: int, w: int) -> int:
    """galois.cpp:605-625."""
    return N.lib.ecgpu_galois_shift_inverse(y, w)


def galois_shift_divide(a: int, b: int, w: int) -> int:
    """galois.cpp:400-408: -1 for b = 0, 0 for a = 0."""
    if b == 0:
        return -1
    if a == 0:
        return 0
    return N.lib.ecgpu_galois_shift_multiply(a, N.lib.ecgpu_galois_shift_inverse(b, w), w)


def galois_split_w8_multiply(x: int, y: int) -> int:
    """The w = 32 product assembled from the 8-bit split tables (galois.cpp:791-810;
    computed directly before galois_create_split_w8_tables, where the reference
    would dereference NULL)."""
    return N.lib.ecgpu_galois_split_w8_multiply(x, y)


def _table(ptr, n: int, offset: int = 0):
    """A read-only numpy view of a library-owned table (lives as long as the library)."""
    if not ptr:
        return None
    import ctypes
    import numpy as np
    base = ctypes.cast(ctypes.addressof(ptr.contents) - 4 * offset, N.c_int_p)
    a = np.ctypeslib.as_array(base, shape=(n,))
    a.flags.writeable = False
    return a


def galois_get_mult_table(w: int):
    """2^(2w) products indexed (x << w) | y, or None for w >= 14 (galois.cpp:627-635)."""
    return _table(N.lib.ecgpu_galois_get_mult_table(w), 1 << (2 * w)) if 0 < w < 14 else None


def galois_get_div_table(w: int):
    """2^(2w) quotients indexed (x << w) | y, or None for w >= 14 (galois.cpp:637-645)."""
    return _table(N.lib.ecgpu_galois_get_div_table(w), 1 << (2 * w)) if 0 < w < 14 else None


def galois_get_log_table(w: int):
    """2^w discrete logs, or None for w > 30 (galois.cpp:647-655)."""
    return _table(N.lib.ecgpu_galois_get_log_table(w), 1 << w) if 0 < w <= 30 else None


def galois_get_ilog_table(w: int):
    """The antilog table as the reference lays it out around its offset
    pointer: entry v of the reference is element v + (2^w - 1) here, for
    -(2^w - 1) <= v < 2(2^w - 1) (a Python negative index would wrap), or
    None for w > 30 (galois.cpp:657-665)."""
    nwm1 = (1 << w) - 1
    return _table(N.lib.ecgpu_galois_get_ilog_table(w), 3 * nwm1, offset=nwm1) if 0 < w <= 30 else None


def galois_w08_region_multiply(region, multby: int, nbytes: int, r2=None, add: int = 0) -> None:
    """r2 (^)= multby * region, or region *= multby in place when r2 is None (galois.cpp:415-467)."""
    N.check(N.lib.ecgpu_galois_w08_region_multiply(addr(region), multby, nbytes, addr(r2) or None, add),
            "galois_w08_region_multiply")


def galois_w16_region_multiply(region, multby: int, nbytes: int, r2=None, add: int = 0) -> None:
    """GF(2^16) over nbytes // 2 words (galois.cpp:469-542), on the MI355X."""
    N.check(N.lib.ecgpu_galois_w16_region_multiply(addr(region), multby, nbytes, addr(r2) or None, add),
            "galois_w16_region_multiply")


def galois_w32_region_multiply(region, multby: int, nbytes: int, r2=None, add: int = 0) -> None:
    """GF(2^32) over nbytes // 4 words (galois.cpp:666-727), on the MI355X; add applies in place too."""
    N.check(N.lib.ecgpu_galois_w32_region_multiply(addr(region), multby, nbytes, addr(r2) or None, add),
            "galois_w32_region_multiply")


def galois_region_xor(r1, r2, r3, nbytes: int) -> None:
    """r3 = r1 ^ r2 (galois.cpp:731-754)."""
    N.check(N.lib.ecgpu_galois_region_xor(addr(r1), addr(r2), addr(r3), nbytes), "galois_region_xor")
