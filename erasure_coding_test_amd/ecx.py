"""ECX-style incremental parity accumulation with HBM-resident accumulators.

The reference's ECX datanode (ecx_datanode_main.cpp:667-735) receives the
k source blocks of a stripe one at a time and, for each, updates its m
parity accumulators with galois_region_xor / galois_w08_region_multiply and
per-accumulator first-touch flags (init[]).  ``ParityAccumulator`` keeps the
m accumulators on the GPU: each ``add`` is one fused launch (only the block
crosses PCIe when it is in host memory), and ``read`` copies a finished
parity block out once.  Same byte results as the reference loop.
``add(..., wait=False)`` only queues the block's update: a pinned block is read
in place by the update kernel over PCIe, and consecutive queued adds run back
to back on the accumulator's stream with no host round trip. ``sync()``, or
any read, reset or synchronous add, waits for the queued adds and releases
their blocks.
"""
from __future__ import annotations

from typing import Sequence

from . import _native as N
from ._buffers import addr


class ParityAccumulator:
    def __init__(self, m: int, size: int, device: int = -1):
        self.m, self.size = m, size
        self._keep = []  # blocks of queued asynchronous adds
        self._a = N.lib.ecgpu_accum_create(m, size, device)
        if not self._a:
            raise N.EcgpuError(f"ecgpu_accum_create failed: {N.last_error()}")

    def add(self, block, coefs: Sequence[int], wait: bool = True) -> None:
        """acc_i (+)= coefs[i] * block for every i (coefficient 0: untouched).
        wait=False queues the add and returns; keep `block` unchanged until sync()."""
        if len(coefs) != self.m:
            raise ValueError("one coefficient per accumulator")
        if wait:
            N.check(N.lib.ecgpu_accum_add(self._a, addr(block), N.int_array(coefs)), "ecgpu_accum_add")
            self._keep.clear()
        else:
            self._keep.append(block)  # referenced until the queued copy is done
            N.check(N.lib.ecgpu_accum_add_async(self._a, addr(block), N.int_array(coefs)), "ecgpu_accum_add_async")

    def sync(self) -> None:
        N.check(N.lib.ecgpu_accum_sync(self._a), "ecgpu_accum_sync")
        self._keep.clear()

    def read(self, i: int, out, nbytes: int = -1) -> bool:
        """Copy accumulator i into `out` (host or device); False if never touched."""
        n = self.size if nbytes < 0 else nbytes
        rc = N.check(N.lib.ecgpu_accum_read(self._a, i, addr(out), n), "ecgpu_accum_read")
        self._keep.clear()
        return rc == N.ECGPU_OK

    def device_ptr(self, i: int) -> int:
        return int(N.lib.ecgpu_accum_device_ptr(self._a, i) or 0)

    def reset(self) -> None:
        N.check(N.lib.ecgpu_accum_reset(self._a), "ecgpu_accum_reset")
        self._keep.clear()

    def close(self) -> None:
        if getattr(self, "_a", None):
            N.lib.ecgpu_accum_destroy(self._a)
            self._a = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
