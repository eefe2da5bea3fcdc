"""Deterministic synthetic shards shared by tests, golden generation and bench.

splitmix64 stream per shard, seeded as SURVEY.md §8d prescribes:
``seed = 0xEC00_0000 ^ (cfg << 32) ^ (stripe << 8) ^ shard``; bytes are the
little-endian 64-bit outputs in order.  Pure numpy (no oracle needed), and
bit-identical to ``orc_splitmix_fill`` in oracle/ec_oracle.c (checked by
tests/test_oracle.py).
"""
from __future__ import annotations

import numpy as np

GAMMA = np.uint64(0x9E3779B97F4A7C15)
M1 = np.uint64(0xBF58476D1CE4E5B9)
M2 = np.uint64(0x94D049BB133111EB)

# configs C1..C5 (BASELINE.json "configs", SURVEY.md §8 legend)
CONFIGS = {
    1: dict(k=4, m=2, size=64 << 10),
    2: dict(k=6, m=3, size=1 << 20),
    3: dict(k=10, m=4, size=4 << 20),
    4: dict(k=10, m=4, size=4 << 20),
    5: dict(k=12, m=4, size=16 << 20),
}


def shard_seed(cfg: int, stripe: int, shard: int) -> int:
    return (0xEC000000 ^ (cfg << 32) ^ (stripe << 8) ^ shard) & (2**64 - 1)


def splitmix_bytes(n: int, seed: int) -> np.ndarray:
    words = (n + 7) // 8
    with np.errstate(over="ignore"):
        z = np.uint64(seed & (2**64 - 1)) + GAMMA * np.arange(1, words + 1, dtype=np.uint64)
        z = (z ^ (z >> np.uint64(30))) * M1
        z = (z ^ (z >> np.uint64(27))) * M2
        z = z ^ (z >> np.uint64(31))
    return z.astype("<u8").view(np.uint8)[:n].copy()


def stripe_shards(cfg: int, stripe: int, count: int, size: int, first_shard: int = 0) -> list:
    return [splitmix_bytes(size, shard_seed(cfg, stripe, first_shard + s)) for s in range(count)]


def fnv1a64(buf) -> int:
    """FNV-1a 64 of a uint8 array (pure Python up to 64 KiB, oracle C loop above)."""
    b = np.ascontiguousarray(np.asarray(buf, dtype=np.uint8).ravel())
    if b.size > (64 << 10):
        return _fnv_large(b)
    h, mask = 0xCBF29CE484222325, (1 << 64) - 1
    for x in b.tobytes():
        h = ((h ^ x) * 0x100000001B3) & mask
    return h


def _fnv_large(b: np.ndarray) -> int:
    # FNV is sequential; large inputs use the checker's C loop (test-only helper).
    import ctypes
    import os

    so = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "libecoracle.so")
    L = ctypes.CDLL(so)
    L.orc_fnv1a64.argtypes = [ctypes.c_void_p, ctypes.c_long]
    L.orc_fnv1a64.restype = ctypes.c_uint64
    return int(L.orc_fnv1a64(b.ctypes.data, b.size))
