"""ctypes binding of include/ecgpu.h (libecgpu.so).

Loaded strictly from the in-tree build (erasure_coding_test_amd/lib/).  There
is no substitute for a missing library: the import fails with instructions to
run the build.  The C library's CPU fallback on HIP errors and
its CPU executor for small host-memory calls are turned off for this package
(PACKAGE_KNOB_DEFAULTS below).  ``torch`` is imported first on purpose -- the PyTorch-ROCm
wheel ships its own HIP runtime (soname libamdhip64.so.7); loading it first
makes libecgpu bind to that same runtime, so device pointers and streams from
torch tensors are valid in our kernels.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch  # noqa: F401  (must precede the CDLL load, see module doc)

LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")
LIB_PATH = os.path.join(LIB_DIR, "libecgpu.so")
DROPIN_PATH = os.path.join(LIB_DIR, "libjerasure_amd.so")

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"{LIB_PATH} is missing: build the HIP extension first "
        "(python erasure_coding_test_amd/build.py, or __graft_entry__.build())")

lib = ctypes.CDLL(LIB_PATH)

c_int, c_int64, c_void_p, c_char_p = ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_char_p
c_int_p = ctypes.POINTER(ctypes.c_int)
c_void_pp = ctypes.POINTER(ctypes.c_void_p)
c_double_p = ctypes.POINTER(ctypes.c_double)

ECGPU_OK, ECGPU_ERR, ECGPU_ERR_ARG, ECGPU_ERR_HIP, ECGPU_ERR_NOMEM = 0, -1, -2, -3, -4
KERNEL_PERM, KERNEL_LDS = 0, 1

# name -> (restype, argtypes); kept in step with include/ecgpu.h (tests check
# that every declared symbol is exported).
SIGNATURES = {
    "ecgpu_version": (c_char_p, []),
    "ecgpu_build_id": (c_char_p, [c_int]),
    "ecgpu_last_error": (c_char_p, []),
    "ecgpu_set_knob": (c_int, [c_char_p, c_int]),
    "ecgpu_reset_knob": (c_int, [c_char_p]),
    "ecgpu_get_knob": (c_int, [c_char_p, c_int_p]),
    "ecgpu_free": (None, [c_void_p]),
    "ecgpu_fallback_count": (c_int64, []),
    "ecgpu_cpu_call_count": (c_int64, []),
    "ecgpu_min_offload_bytes": (c_int64, []),
    "ecgpu_device_lost": (c_int, [c_int]),
    "ecgpu_set_devices": (c_int, [c_int, c_int_p]),
    "ecgpu_get_devices": (c_int, [c_int_p, c_int]),
    "ecgpu_call_device": (c_int, []),
    "ecgpu_engine_launches": (c_int64, [c_int]),
    "ecgpu_galois_single_multiply": (c_int, [c_int, c_int, c_int]),
    "ecgpu_galois_single_divide": (c_int, [c_int, c_int, c_int]),
    "ecgpu_galois_inverse": (c_int, [c_int, c_int]),
    "ecgpu_galois_log": (c_int, [c_int, c_int]),
    "ecgpu_galois_ilog": (c_int, [c_int, c_int]),
    "ecgpu_galois_create_log_tables": (c_int, [c_int]),
    "ecgpu_galois_create_mult_tables": (c_int, [c_int]),
    "ecgpu_galois_get_mult_table": (c_int_p, [c_int]),
    "ecgpu_galois_get_div_table": (c_int_p, [c_int]),
    "ecgpu_galois_get_log_table": (c_int_p, [c_int]),
    "ecgpu_galois_get_ilog_table": (c_int_p, [c_int]),
    "ecgpu_galois_shift_multiply": (c_int, [c_int, c_int, c_int]),
    "ecgpu_galois_shift_inverse": (c_int, [c_int, c_int]),
    "ecgpu_galois_create_split_w8_tables": (c_int, []),
    "ecgpu_galois_split_w8_multiply": (c_int, [c_int, c_int]),
    "ecgpu_reed_sol_vandermonde_coding_matrix": (c_void_p, [c_int, c_int, c_int]),
    "ecgpu_reed_sol_extended_vandermonde_matrix": (c_void_p, [c_int, c_int, c_int]),
    "ecgpu_reed_sol_big_vandermonde_distribution_matrix": (c_void_p, [c_int, c_int, c_int]),
    "ecgpu_reed_sol_r6_coding_matrix": (c_void_p, [c_int, c_int]),
    "ecgpu_jerasure_invert_matrix": (c_int, [c_int_p, c_int_p, c_int, c_int]),
    "ecgpu_jerasure_invertible_matrix": (c_int, [c_int_p, c_int, c_int]),
    "ecgpu_jerasure_matrix_multiply": (c_void_p, [c_int_p, c_int_p, c_int, c_int, c_int, c_int, c_int]),
    "ecgpu_jerasure_erasures_to_erased": (c_void_p, [c_int, c_int, c_int_p]),
    "ecgpu_jerasure_make_decoding_matrix": (c_int, [c_int, c_int, c_int, c_int_p, c_int_p, c_int_p, c_int_p]),
    "ecgpu_jerasure_matrix_to_bitmatrix": (c_void_p, [c_int, c_int, c_int, c_int_p]),
    "ecgpu_jerasure_make_decoding_bitmatrix": (c_int, [c_int, c_int, c_int, c_int_p, c_int_p, c_int_p, c_int_p]),
    "ecgpu_jerasure_invert_bitmatrix": (c_int, [c_int_p, c_int_p, c_int]),
    "ecgpu_jerasure_invertible_bitmatrix": (c_int, [c_int_p, c_int]),
    "ecgpu_decode_plan": (c_int, [c_int, c_int, c_int, c_int_p, c_int, c_int_p, c_int_p, c_int_p, c_int_p,
                                  c_int_p, c_int_p]),
    "ecgpu_jerasure_matrix_encode": (c_int, [c_int, c_int, c_int, c_int_p, c_void_pp, c_void_pp, c_int]),
    "ecgpu_jerasure_matrix_decode": (c_int, [c_int, c_int, c_int, c_int_p, c_int, c_int_p, c_void_pp, c_void_pp,
                                             c_int]),
    "ecgpu_jerasure_matrix_dotprod": (c_int, [c_int, c_int, c_int_p, c_int_p, c_int, c_void_pp, c_void_pp, c_int]),
    "ecgpu_jerasure_do_parity": (c_int, [c_int, c_void_pp, c_void_p, c_int]),
    "ecgpu_galois_w08_region_multiply": (c_int, [c_void_p, c_int, c_int, c_void_p, c_int]),
    "ecgpu_galois_region_xor": (c_int, [c_void_p, c_void_p, c_void_p, c_int]),
    "ecgpu_reed_sol_r6_encode": (c_int, [c_int, c_int, c_void_pp, c_void_pp, c_int]),
    "ecgpu_reed_sol_galois_w08_region_multby_2": (c_int, [c_void_p, c_int]),
    "ecgpu_jerasure_bitmatrix_dotprod": (c_int, [c_int, c_int, c_int_p, c_int_p, c_int, c_void_pp, c_void_pp, c_int, c_int]),
    "ecgpu_jerasure_bitmatrix_encode": (c_int, [c_int, c_int, c_int, c_int_p, c_void_pp, c_void_pp, c_int, c_int]),
    "ecgpu_jerasure_bitmatrix_decode": (c_int, [c_int, c_int, c_int, c_int_p, c_int, c_int_p, c_void_pp, c_void_pp, c_int, c_int]),
    "ecgpu_jerasure_do_scheduled_operations": (c_int, [c_void_pp, c_void_p, c_int]),
    "ecgpu_jerasure_schedule_encode": (c_int, [c_int, c_int, c_int, c_void_p, c_void_pp, c_void_pp, c_int, c_int]),
    "ecgpu_schedule_run": (c_int, [c_int, c_void_pp, c_void_p, c_int, c_int, c_int]),
    "ecgpu_jerasure_dumb_bitmatrix_to_schedule": (c_void_p, [c_int, c_int, c_int, c_int_p]),
    "ecgpu_jerasure_smart_bitmatrix_to_schedule": (c_void_p, [c_int, c_int, c_int, c_int_p]),
    "ecgpu_jerasure_free_schedule": (None, [c_void_p]),
    "ecgpu_jerasure_generate_schedule_cache": (c_void_p, [c_int, c_int, c_int, c_int_p, c_int]),
    "ecgpu_jerasure_free_schedule_cache": (c_int, [c_int, c_int, c_void_p]),
    "ecgpu_jerasure_schedule_decode_lazy": (c_int, [c_int, c_int, c_int, c_int_p, c_int_p, c_void_pp, c_void_pp, c_int, c_int, c_int]),
    "ecgpu_jerasure_schedule_decode_cache": (c_int, [c_int, c_int, c_int, c_void_p, c_int_p, c_void_pp, c_void_pp, c_int, c_int]),
    "ecgpu_reed_sol_galois_w16_region_multby_2": (c_int, [c_void_p, c_int]),
    "ecgpu_reed_sol_galois_w32_region_multby_2": (c_int, [c_void_p, c_int]),
    "ecgpu_galois_w16_region_multiply": (c_int, [c_void_p, c_int, c_int, c_void_p, c_int]),
    "ecgpu_galois_w32_region_multiply": (c_int, [c_void_p, c_int, c_int, c_void_p, c_int]),
    "ecgpu_jerasure_get_stats": (c_int, [c_double_p]),
    "ecgpu_plan_create": (c_void_p, [c_int, c_int, c_int_p, c_int]),
    "ecgpu_plan_bind": (c_int, [c_void_p, c_int, c_void_pp, c_void_pp, c_int64]),
    "ecgpu_plan_check_buffers": (c_int, [c_int, c_int, c_int, c_void_pp, c_void_pp, c_int64]),
    "ecgpu_plan_set_kernel": (c_int, [c_void_p, c_int, c_int]),
    "ecgpu_plan_launch": (c_int, [c_void_p, c_void_p]),
    "ecgpu_plan_destroy": (None, [c_void_p]),
    "ecgpu_recommended_shard_stride": (c_int64, [c_int64]),
    "ecgpu_recommended_shard_stride_km": (c_int64, [c_int64, c_int, c_int]),
    "ecgpu_pipeline_create": (c_void_p, [c_int, c_int, c_int_p, c_int64, c_int, c_int]),
    "ecgpu_pipeline_create_decode": (c_void_p, [c_int, c_int, c_int, c_int_p, c_int, c_int_p, c_int64, c_int, c_int]),
    "ecgpu_pipeline_submit": (c_int64, [c_void_p, c_void_pp, c_void_pp]),
    "ecgpu_pipeline_wait": (c_int, [c_void_p, c_int64]),
    "ecgpu_pipeline_drain": (c_int, [c_void_p]),
    "ecgpu_pipeline_destroy": (None, [c_void_p]),
    "ecgpu_pipeline_group_create": (c_void_p, [c_int, c_int, c_int_p, c_int64, c_int, c_int, c_int_p]),
    "ecgpu_pipeline_group_create_decode": (c_void_p, [c_int, c_int, c_int, c_int_p, c_int, c_int_p, c_int64, c_int,
                                                      c_int, c_int_p]),
    "ecgpu_pipeline_group_submit": (c_int64, [c_void_p, c_void_pp, c_void_pp]),
    "ecgpu_pipeline_group_wait": (c_int, [c_void_p, c_int64]),
    "ecgpu_pipeline_group_drain": (c_int, [c_void_p]),
    "ecgpu_pipeline_group_size": (c_int, [c_void_p]),
    "ecgpu_pipeline_group_destroy": (None, [c_void_p]),
    "ecgpu_device_pci_bus_id": (c_int, [c_int, c_char_p, c_int]),
    "ecgpu_host_register": (c_int, [c_void_p, c_int64]),
    "ecgpu_host_unregister": (c_int, [c_void_p]),
    "ecgpu_accum_create": (c_void_p, [c_int, c_int64, c_int]),
    "ecgpu_accum_add": (c_int, [c_void_p, c_void_p, c_int_p]),
    "ecgpu_accum_add_async": (c_int, [c_void_p, c_void_p, c_int_p]),
    "ecgpu_accum_sync": (c_int, [c_void_p]),
    "ecgpu_accum_read": (c_int, [c_void_p, c_int, c_void_p, c_int64]),
    "ecgpu_accum_device_ptr": (c_void_p, [c_void_p, c_int]),
    "ecgpu_accum_reset": (c_int, [c_void_p]),
    "ecgpu_accum_destroy": (None, [c_void_p]),
    "ecgpu_encode_batch": (c_int, [c_int, c_int, c_int_p, c_int, c_void_pp, c_void_pp, c_int64, c_void_p]),
}

for _name, (_res, _args) in SIGNATURES.items():
    _f = getattr(lib, _name)
    _f.restype, _f.argtypes = _res, _args


class EcgpuError(RuntimeError):
    pass


# The package's own knob defaults, where they differ from the C library's.
# ECGPU_CPU_FALLBACK: libjerasure_amd.so completes a host-memory call on the
# CPU after a HIP error (cpu_fallback.hpp) so a deployed datanode
# keeps running; this package -- what the tests, smoke() and bench.py drive --
# fails loudly instead (EcgpuError), so no checked or measured result can come
# from the CPU.  An ECGPU_CPU_FALLBACK set in the environment wins.
#
# ECGPU_MIN_OFFLOAD_KIB / ECGPU_LINK_CALLS: the C library runs small
# host-memory calls, and large ones arriving while another holds the device's
# link, on its CPU executor; this package sends every call to
# the GPU, so each checked or measured result is the HIP path's.
PACKAGE_KNOB_DEFAULTS = {"ECGPU_CPU_FALLBACK": 0, "ECGPU_MIN_OFFLOAD_KIB": 0, "ECGPU_LINK_CALLS": 0}


def _apply_package_defaults(names=None) -> None:
    for env, value in PACKAGE_KNOB_DEFAULTS.items():
        if (names is None or env in names) and not os.environ.get(env):
            lib.ecgpu_set_knob(env.encode(), value)


_apply_package_defaults()


def set_knob(name: str, value: int) -> None:
    """Override a tuning knob for this process (ecgpu_set_knob; knobs.hpp)."""
    check(lib.ecgpu_set_knob(name.encode(), int(value)), "ecgpu_set_knob")


def reset_knob(name=None) -> None:
    """Back to the environment's value (None: every knob), or the package's
    default for knobs it sets (PACKAGE_KNOB_DEFAULTS)."""
    check(lib.ecgpu_reset_knob(None if name is None else name.encode()), "ecgpu_reset_knob")
    if name is None:
        _apply_package_defaults()
    else:
        _apply_package_defaults({n for n in PACKAGE_KNOB_DEFAULTS if name in (n, n[len("ECGPU_"):].lower())})


def set_devices(devices) -> None:
    """ECGPU_DEVICES for this process (ecgpu_set_devices); None or [] unsets."""
    devices = list(devices or [])
    check(lib.ecgpu_set_devices(len(devices), (c_int * max(1, len(devices)))(*devices)), "ecgpu_set_devices")


def get_devices() -> list:
    n = lib.ecgpu_get_devices(None, 0)
    buf = (c_int * max(1, n))()
    lib.ecgpu_get_devices(buf, n)
    return list(buf[:n])


def fallback_count() -> int:
    """Synchronous calls completed on the CPU after a HIP error (ecgpu_fallback_count)."""
    return int(lib.ecgpu_fallback_count())


def cpu_call_count() -> int:
    """Synchronous host-memory calls run on the CPU executor by choice
    (ECGPU_MIN_OFFLOAD_KIB / ECGPU_GPU=0; ecgpu_cpu_call_count)."""
    return int(lib.ecgpu_cpu_call_count())


def get_knob(name: str) -> int:
    v = c_int()
    check(lib.ecgpu_get_knob(name.encode(), ctypes.byref(v)), "ecgpu_get_knob")
    return v.value


def last_error() -> str:
    msg = lib.ecgpu_last_error()
    return msg.decode() if msg else ""


def check(rc: int, what: str) -> int:
    if rc < ECGPU_ERR:  # ECGPU_ERR (-1) is a reference-style result, not an exception
        raise EcgpuError(f"{what} failed ({rc}): {last_error()}")
    return rc


def int_array(values) -> ctypes.Array:
    """C int[] from ints (values wrap to 32 bits like a C int assignment:
    w = 32 coefficients >= 2^31 pass through).  Long inputs -- bit-matrices,
    k*m*w*w ints -- convert through numpy (2.5x faster at 2,560 entries)."""
    if not isinstance(values, np.ndarray) and not hasattr(values, "__len__"):
        values = list(values)  # generators and other unsized iterables
    if isinstance(values, np.ndarray) or len(values) >= 64:
        a = np.asarray(values)
        if a.dtype.kind not in "iu":
            a = np.array([int(v) for v in values], dtype=np.int64)
        a = a.reshape(-1).astype(np.int64, copy=False).astype(np.int32)
        if a.size == 0:
            a = np.zeros(1, np.int32)
        return (c_int * a.size).from_buffer_copy(a)
    vals = [int(v) for v in values]
    arr = (c_int * max(1, len(vals)))()
    for i, v in enumerate(vals):
        arr[i] = v
    return arr


def ptr_array(ptrs) -> ctypes.Array:
    ptrs = list(ptrs)
    arr = (c_void_p * max(1, len(ptrs)))()
    for i, p in enumerate(ptrs):
        arr[i] = p
    return arr


def take_int_matrix(addr: int, n: int) -> list:
    """Copy n ints out of a malloc'd C array and free it (NULL -> None)."""
    if not addr:
        return None
    out = list((c_int * n).from_address(addr))
    lib.ecgpu_free(addr)
    return out
