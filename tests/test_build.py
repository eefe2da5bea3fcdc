"""Build provenance: objects are rebuilt on
content, not mtime; the library reports content IDs of its sources; and
bench.py reports PMC traffic only for the kernel build it was measured on.
CPU only (the library is loaded, no GPU call is made)."""
import ctypes
import importlib.util
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
LIB = os.path.join(ROOT, "erasure_coding_test_amd", "lib", "libecgpu.so")


def _build_module():
    spec = importlib.util.spec_from_file_location("_ecgpu_build_t", os.path.join(ROOT, "erasure_coding_test_amd",
                                                                                  "build.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_library_is_built_from_these_sources():
    b = _build_module()
    lib = ctypes.CDLL(LIB)
    lib.ecgpu_build_id.restype = ctypes.c_char_p
    lib.ecgpu_build_id.argtypes = [ctypes.c_int]
    ids = b.build_ids()
    assert lib.ecgpu_build_id(0).decode() == ids["build"], "libecgpu.so is stale: rebuild"
    assert lib.ecgpu_build_id(1).decode() == ids["kernels"]
    assert len(ids["build"]) == 16 and ids["build"] != ids["kernels"]


def test_rebuild_decision_is_content_based(tmp_path):
    b = _build_module()
    src, obj = tmp_path / "a.cpp", tmp_path / "a.o"
    src.write_text("int x;\n")
    cmd = ["cc", "-c", str(src)]
    assert b._stale(str(obj), [str(src)], cmd)  # no object yet
    obj.write_text("obj")
    b._commit_keys()
    assert not b._stale(str(obj), [str(src)], cmd)
    os.utime(src, (1e10, 1e10))  # newer mtime, same bytes: not stale
    assert not b._stale(str(obj), [str(src)], cmd)
    assert b._stale(str(obj), [str(src)], cmd + ["-O3"])  # another command line
    b._pending_keys.clear()
    src.write_text("int y;\n")  # other bytes, older mtime: stale
    os.utime(src, (1, 1))
    assert b._stale(str(obj), [str(src)], cmd)
    b._pending_keys.clear()


def test_bench_traffic_only_for_the_measured_kernel_build(tmp_path):
    import bench
    rec = {"workload_key": "C3:96", "kernel": "gf_apply<10, 4, 3,", "hbm_bytes_per_launch": 123,
           "kernel_build_id": "aaaa", "from": "profiles/rXX_rocprof_summary.json"}
    (tmp_path / "pmc_encode.json").write_text(json.dumps(rec))
    v, note = bench.load_traffic("encode", "C3:96", "aaaa", str(tmp_path))
    assert v == 123 and "aaaa" in note
    v, note = bench.load_traffic("encode", "C3:96", "bbbb", str(tmp_path))
    assert v is None and "stale" in note
    v, note = bench.load_traffic("encode", "C5:8", "aaaa", str(tmp_path))
    assert v is None and "workload" in note
    v, note = bench.load_traffic("decode", "C3:96", "aaaa", str(tmp_path))
    assert v is None and "no PMC record" in note


def test_committed_pmc_records_carry_a_kernel_build_id():
    for name in ("encode", "decode"):
        with open(os.path.join(ROOT, "profiles", f"pmc_{name}.json")) as f:
            d = json.load(f)
        assert "kernel_build_id" in d, name
