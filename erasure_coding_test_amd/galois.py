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
