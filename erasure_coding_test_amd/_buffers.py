"""Buffer address helpers: torch tensors (CUDA or CPU), numpy arrays, raw ints."""
from __future__ import annotations


def addr(buf) -> int:
    """Base address of a shard buffer.  CUDA tensors give device pointers
    (used in place by the library); CPU tensors / numpy arrays give host
    pointers (staged through HBM by the library)."""
    if buf is None:
        return 0
    if isinstance(buf, int):
        return buf
    if hasattr(buf, "data_ptr"):  # torch.Tensor
        if not buf.is_contiguous():
            raise ValueError("shard tensors must be contiguous")
        return int(buf.data_ptr())
    if hasattr(buf, "ctypes"):  # numpy.ndarray
        if not buf.flags["C_CONTIGUOUS"]:
            raise ValueError("shard arrays must be C-contiguous")
        return int(buf.ctypes.data)
    raise TypeError(f"unsupported shard buffer type {type(buf)!r}")


def addrs(bufs) -> list:
    return [addr(b) for b in bufs]
