"""reed_sol.h surface (reference include/reed_sol.h:33-42) over the C ABI.

Matrices come back as flat row-major Python int lists (m*k entries), or None
where the reference returns NULL.  Matrix construction runs on the host
(csrc/matrix_host.cpp); the region ops and the RAID-6 encode run on the
MI355X.
"""
from __future__ import annotations

from typing import List, Optional

from . import _native as N
from ._buffers import addr, addrs


def reed_sol_vandermonde_coding_matrix(k: int, m: int, w: int) -> Optional[List[int]]:
    """m x k coding matrix, first row and column all ones (reed_sol.cpp:63-88)."""
    return N.take_int_matrix(N.lib.ecgpu_reed_sol_vandermonde_coding_matrix(k, m, w), k * m)


def reed_sol_extended_vandermonde_matrix(rows: int, cols: int, w: int) -> Optional[List[int]]:
    """rows x cols extended Vandermonde matrix; None when w < 30 and rows or cols exceed 2^w (reed_sol.cpp:227-255)."""
    return N.take_int_matrix(N.lib.ecgpu_reed_sol_extended_vandermonde_matrix(rows, cols, w), rows * cols)


def reed_sol_big_vandermonde_distribution_matrix(rows: int, cols: int, w: int) -> Optional[List[int]]:
    """Systematic distribution matrix by column ops (reed_sol.cpp:257-349); None for cols >= rows."""
    return N.take_int_matrix(N.lib.ecgpu_reed_sol_big_vandermonde_distribution_matrix(rows, cols, w), rows * cols)


def reed_sol_r6_coding_matrix(k: int, w: int) -> Optional[List[int]]:
    """2 x k RAID-6 matrix: ones, then powers of 2 (reed_sol.cpp:43-61); None for w not in {8, 16, 32}."""
    return N.take_int_matrix(N.lib.ecgpu_reed_sol_r6_coding_matrix(k, w), 2 * k)


def reed_sol_r6_encode(k: int, w: int, data_ptrs, coding_ptrs, size: int) -> int:
    """RAID-6 P/Q encode (reed_sol.cpp:200-225): 1, or 0 for w not in {8, 16, 32}."""
    return N.check(N.lib.ecgpu_reed_sol_r6_encode(k, w, N.ptr_array(addrs(data_ptrs)),
                                                  N.ptr_array(addrs(coding_ptrs)), size), "reed_sol_r6_encode")


def reed_sol_galois_w08_region_multby_2(region, nbytes: int) -> None:
    """region *= 2 over GF(2^8) bytes, in place (reed_sol.cpp:112-156)."""
    N.check(N.lib.ecgpu_reed_sol_galois_w08_region_multby_2(addr(region), nbytes),
            "reed_sol_galois_w08_region_multby_2")


def reed_sol_galois_w16_region_multby_2(region, nbytes: int) -> None:
    """region *= 2 over GF(2^16) words, in place (reed_sol.cpp:158-198)."""
    N.check(N.lib.ecgpu_reed_sol_galois_w16_region_multby_2(addr(region), nbytes),
            "reed_sol_galois_w16_region_multby_2")


def reed_sol_galois_w32_region_multby_2(region, nbytes: int) -> None:
    """region *= 2 over GF(2^32) words, in place (reed_sol.cpp:90-110)."""
    N.check(N.lib.ecgpu_reed_sol_galois_w32_region_multby_2(addr(region), nbytes),
            "reed_sol_galois_w32_region_multby_2")
