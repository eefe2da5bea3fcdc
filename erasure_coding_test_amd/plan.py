"""Batched, device-resident stripe coding (ecgpu_plan_* in include/ecgpu.h).

A :class:`StripePlan` holds one rows x nsrc GF(2^8) coefficient matrix on
the GPU and a table of device pointers for many stripes; ``launch`` enqueues
the fused apply asynchronously on a HIP stream (torch's current stream by
default), so it composes with torch events and HIP graphs.  This is the
interface the bench and multi-stripe callers use; the jerasure-named
functions are the synchronous, one-stripe drop-in over the same kernels.
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch

from . import _native as N
from ._buffers import addr
from .jerasure import decode_plan as _decode_map


class StripePlan:
    def __init__(self, rows: int, nsrc: int, coefs: Sequence[int], device: int = -1):
        coefs = [int(c) for c in coefs]
        if len(coefs) != rows * nsrc:
            raise ValueError("coefs must hold rows * nsrc entries")
        self.rows, self.nsrc, self.coefs = rows, nsrc, coefs
        self.device = torch.cuda.current_device() if device < 0 else device
        self._p = N.lib.ecgpu_plan_create(rows, nsrc, N.int_array(coefs), self.device)
        if not self._p:
            raise N.EcgpuError(f"ecgpu_plan_create failed: {N.last_error()}")
        self.stripes, self.size = 0, 0

    def bind(self, srcs: Sequence[Sequence], dsts: Sequence[Sequence], size: int) -> "StripePlan":
        """srcs[s][j] / dsts[s][r]: device buffers (CUDA tensors or raw device addresses)."""
        if len(srcs) != len(dsts):
            raise ValueError("srcs and dsts must list the same number of stripes")
        flat_s = [addr(b) for row in srcs for b in row]
        flat_d = [addr(b) for row in dsts for b in row]
        if len(flat_s) != len(srcs) * self.nsrc or len(flat_d) != len(dsts) * self.rows:
            raise ValueError("every stripe needs nsrc sources and rows destinations")
        N.check(N.lib.ecgpu_plan_bind(self._p, len(srcs), N.ptr_array(flat_s), N.ptr_array(flat_d), size),
                "ecgpu_plan_bind")
        self.stripes, self.size = len(srcs), size
        return self

    def set_kernel(self, kind: int = N.KERNEL_PERM, nontemporal: bool = True) -> "StripePlan":
        N.check(N.lib.ecgpu_plan_set_kernel(self._p, kind, int(bool(nontemporal))), "ecgpu_plan_set_kernel")
        return self

    def launch(self, stream: Optional[int] = None) -> None:
        if stream is None:
            stream = torch.cuda.current_stream(self.device).cuda_stream
        N.check(N.lib.ecgpu_plan_launch(self._p, stream or None), "ecgpu_plan_launch")

    def close(self) -> None:
        if getattr(self, "_p", None):
            N.lib.ecgpu_plan_destroy(self._p)
            self._p = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def alloc_stripes(stripes: int, k: int, m: int, size: int, device=None):
    """One HBM slab for `stripes` stripes of k+m shards, laid out with the
    library's recommended shard stride for the scheme
    (ecgpu_recommended_shard_stride_km: a per-size skew so a column's k+m
    accesses do not share an HBM channel/bank; none for small shards).
    Returns (slab, shards) with shards[s][i] a `size`-byte uint8 view."""
    stride = int(N.lib.ecgpu_recommended_shard_stride_km(size, k, m))
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    slab = torch.empty((stripes, k + m, stride), dtype=torch.uint8, device=dev)
    shards = [[slab[s, i, :size] for i in range(k + m)] for s in range(stripes)]
    return slab, shards


def encode_plan(k: int, m: int, matrix: Sequence[int], device: int = -1) -> StripePlan:
    """Plan computing the m coding shards from the k data shards of each stripe."""
    return StripePlan(m, k, matrix, device)


class DecodePlan(StripePlan):
    """The fused map of jerasure_matrix_decode for one erasure pattern.

    ``out_ids`` are the shard ids it writes and ``src_ids`` the shard ids it
    reads; bind with :meth:`bind_stripes` from full per-stripe shard lists.
    """

    def __init__(self, k: int, m: int, matrix, erasures, row_k_ones: int = 0, device: int = -1):
        fused = _decode_map(k, m, matrix, erasures, row_k_ones)
        if fused is None:
            raise ValueError("unrecoverable erasure pattern (the reference decode returns -1)")
        self.out_ids, self.src_ids, rows = fused
        self.k, self.m = k, m
        flat = [c for r in rows for c in r]
        super().__init__(max(1, len(self.out_ids)), max(1, len(self.src_ids)), flat or [0], device)
        self.empty = not self.out_ids

    def bind_stripes(self, shards: Sequence[Sequence], size: int) -> "DecodePlan":
        """shards[s] = the k+m shard buffers of stripe s (ids 0..k+m-1)."""
        if self.empty:
            return self
        return self.bind([[st[i] for i in self.src_ids] for st in shards],
                         [[st[i] for i in self.out_ids] for st in shards], size)

    def launch(self, stream: Optional[int] = None) -> None:
        if not self.empty:
            super().launch(stream)
