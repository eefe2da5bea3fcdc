"""Host-memory stripe pipeline (client write path, client_main.cpp:1714-1815).

``HostPipeline`` encodes stripes whose shards live in host memory with the
H2D copy, the encode and the D2H copy of consecutive stripes overlapped on
three HIP streams (ecgpu_pipeline_* in include/ecgpu.h).  ``submit`` returns
a ticket immediately; the buffers must stay untouched until ``wait(ticket)``.
Pinned buffers (torch ``pin_memory()`` or :func:`host_register`) get
asynchronous DMA. Pageable ones are staged by HIP, whose pageable copies
block the thread that issues them. So the D2H into pageable outputs is issued
by the pipeline's own worker thread, overlapping the next stripe's H2D.

``HostPipeline.decoder`` is the read path (client_main.cpp:2055-2182, decode
after recv): the fused map of jerasure_matrix_decode for one erasure pattern;
``submit`` takes the full data[k] / coding[m] buffer lists like the reference
decode and writes the erased shards back in place.
"""
from __future__ import annotations

from typing import Sequence

from . import _native as N
from ._buffers import addr, addrs


class HostPipeline:
    def __init__(self, k: int, m: int, matrix: Sequence[int], size: int, depth: int = 3, device: int = -1,
                 _handle=None):
        self.k, self.m, self.size = k, m, size
        self._p = _handle if _handle is not None else N.lib.ecgpu_pipeline_create(
            k, m, N.int_array(matrix), size, depth, device)
        if not self._p:
            raise N.EcgpuError(f"ecgpu_pipeline_create failed: {N.last_error()}")
        self._keep = {}  # ticket -> buffers (kept alive until waited)

    @classmethod
    def decoder(cls, k: int, m: int, matrix: Sequence[int], erasures: Sequence[int], size: int,
                row_k_ones: int = 0, depth: int = 3, device: int = -1) -> "HostPipeline":
        """Raises EcgpuError where the reference decode would return -1."""
        er = list(erasures)
        if not er or er[-1] != -1:
            er.append(-1)
        h = N.lib.ecgpu_pipeline_create_decode(k, m, 8, N.int_array(matrix), row_k_ones, N.int_array(er), size,
                                               depth, device)
        if not h:
            raise N.EcgpuError(f"ecgpu_pipeline_create_decode failed: {N.last_error()}")
        return cls(k, m, matrix, size, depth, device, _handle=h)

    def submit(self, data_ptrs, coding_ptrs) -> int:
        if len(data_ptrs) != self.k or len(coding_ptrs) != self.m:
            raise ValueError("k data and m coding buffers required")
        for b in list(data_ptrs) + list(coding_ptrs):
            if getattr(b, "is_cuda", False):
                raise ValueError("HostPipeline takes host buffers; use encode_plan/DecodePlan for HBM shards")
        t = N.lib.ecgpu_pipeline_submit(self._p, N.ptr_array(addrs(data_ptrs)), N.ptr_array(addrs(coding_ptrs)))
        if t < 0:
            raise N.EcgpuError(f"ecgpu_pipeline_submit failed ({t}): {N.last_error()}")
        self._keep[t] = (data_ptrs, coding_ptrs)
        return t

    def wait(self, ticket: int) -> None:
        N.check(N.lib.ecgpu_pipeline_wait(self._p, ticket), "ecgpu_pipeline_wait")
        for t in [t for t in self._keep if t <= ticket]:
            del self._keep[t]

    def drain(self) -> None:
        N.check(N.lib.ecgpu_pipeline_drain(self._p), "ecgpu_pipeline_drain")
        self._keep.clear()

    def close(self) -> None:
        if getattr(self, "_p", None):
            N.lib.ecgpu_pipeline_destroy(self._p)
            self._p = None
            self._keep.clear()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class HostPipelineGroup:
    """Several GPUs from one process (ecgpu_pipeline_group_*): one
    single-device pipeline per entry of ``devices`` (repeats allowed), stripe
    ticket t on member t % len(devices), each member with its own submit
    thread bound to its device.  Stripes are independent, so there is no
    collective; the interface is HostPipeline's (submit may be called from
    several threads)."""

    def __init__(self, k: int, m: int, matrix: Sequence[int], size: int, devices: Sequence[int], depth: int = 3,
                 _handle=None):
        self.k, self.m, self.size = k, m, size
        self.devices = list(devices)
        self._g = _handle if _handle is not None else N.lib.ecgpu_pipeline_group_create(
            k, m, N.int_array(matrix), size, depth, len(self.devices), N.int_array(self.devices))
        if not self._g:
            raise N.EcgpuError(f"ecgpu_pipeline_group_create failed: {N.last_error()}")
        self._keep = {}

    @classmethod
    def decoder(cls, k: int, m: int, matrix: Sequence[int], erasures: Sequence[int], size: int,
                devices: Sequence[int], row_k_ones: int = 0, depth: int = 3) -> "HostPipelineGroup":
        """Raises EcgpuError where the reference decode would return -1."""
        er = list(erasures)
        if not er or er[-1] != -1:
            er.append(-1)
        devs = list(devices)
        h = N.lib.ecgpu_pipeline_group_create_decode(k, m, 8, N.int_array(matrix), row_k_ones, N.int_array(er), size,
                                                     depth, len(devs), N.int_array(devs))
        if not h:
            raise N.EcgpuError(f"ecgpu_pipeline_group_create_decode failed: {N.last_error()}")
        return cls(k, m, matrix, size, devs, depth, _handle=h)

    def submit(self, data_ptrs, coding_ptrs) -> int:
        if len(data_ptrs) != self.k or len(coding_ptrs) != self.m:
            raise ValueError("k data and m coding buffers required")
        for b in list(data_ptrs) + list(coding_ptrs):
            if getattr(b, "is_cuda", False):
                raise ValueError("HostPipelineGroup takes host buffers")
        t = N.lib.ecgpu_pipeline_group_submit(self._g, N.ptr_array(addrs(data_ptrs)), N.ptr_array(addrs(coding_ptrs)))
        if t < 0:
            raise N.EcgpuError(f"ecgpu_pipeline_group_submit failed ({t}): {N.last_error()}")
        self._keep[t] = (data_ptrs, coding_ptrs)
        return t

    def wait(self, ticket: int) -> None:
        N.check(N.lib.ecgpu_pipeline_group_wait(self._g, ticket), "ecgpu_pipeline_group_wait")
        # a member completes its tickets in order: every earlier ticket of the
        # same member is done too, so its buffers are released as well
        n = len(self.devices)
        for t in [t for t in self._keep if t <= ticket and t % n == ticket % n]:
            del self._keep[t]

    def drain(self) -> None:
        N.check(N.lib.ecgpu_pipeline_group_drain(self._g), "ecgpu_pipeline_group_drain")
        self._keep.clear()

    def close(self) -> None:
        if getattr(self, "_g", None):
            N.lib.ecgpu_pipeline_group_destroy(self._g)
            self._g = None
            self._keep.clear()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def host_register(buf, nbytes: int = -1) -> None:
    """Page-lock a host buffer (numpy array) for asynchronous DMA."""
    n = buf.nbytes if nbytes < 0 else nbytes
    N.check(N.lib.ecgpu_host_register(addr(buf), n), "ecgpu_host_register")


def host_unregister(buf) -> None:
    N.check(N.lib.ecgpu_host_unregister(addr(buf)), "ecgpu_host_unregister")
