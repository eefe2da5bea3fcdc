"""galois.h surface (reference include/galois.h:41-95) over the C ABI.

Scalar field ops run on the host; the w=8 region ops run on the MI355X.
"""
from __future__ import annotations

from . import _native as N
from ._buffers import addr


def galois_single_multiply(a: int, b: int, w: int) -> int:
    return N.lib.ecgpu_galois_single_multiply(a, b, w)


def galois_single_divide(a: int, b: int, w: int) -> int:
    return N.lib.ecgpu_galois_single_divide(a, b, w)


def galois_inverse(a: int, w: int) -> int:
    return N.lib.ecgpu_galois_inverse(a, w)


def galois_log(value: int, w: int) -> int:
    return N.lib.ecgpu_galois_log(value, w)


def galois_ilog(value: int, w: int) -> int:
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
