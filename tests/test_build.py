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
    assert lib.ecgpu_build_id(2).decode() == ids["wide"]
    assert lib.ecgpu_build_id(3).decode() == ids["packets"]
    assert len(ids["build"]) == 16 and len({ids["build"], ids["kernels"], ids["wide"], ids["packets"]}) == 4


def _ids_with_edit(b, tmp_path, name, text=None):
    """build_ids() over a copy of csrc/ with one file appended to (or a knob
    row's default changed: text = (old, new))."""
    import shutil
    csrc = tmp_path / "csrc"
    if csrc.exists():
        shutil.rmtree(csrc)
    shutil.copytree(b.CSRC, csrc)
    f = csrc / name
    if isinstance(text, tuple):
        f.write_text(f.read_text().replace(*text))
    else:
        f.write_text(f.read_text() + "\n// edited\n")
    saved = b.CSRC
    b.CSRC = str(csrc)
    try:
        return b.build_ids()
    finally:
        b.CSRC = saved


def test_kernel_families_have_their_own_build_ids(tmp_path):
    """an edit to a w = 32, packet or lab kernel must not
    invalidate the w = 8 PMC records (keyed to ecgpu_build_id(1))."""
    b = _build_module()
    base = b.build_ids()
    for name in ("gf_kernels_wide.hpp", "gf_kernels_packets.hpp", "dispatch_wide.hip", "wide_spec.hip",
                 "packets.hip", "diag_kernels_w8.hpp", "diag_kernels.hip", "ecgpu_runtime.hip", "cpu_fallback.cpp"):
        ids = _ids_with_edit(b, tmp_path, name)
        assert ids["kernels"] == base["kernels"], name
        assert ids["build"] != base["build"] or name.startswith("diag_kernels"), name
    for name in ("gf_kernels_w8.hpp", "gf_spec.hip", "dispatch_w8.hip"):
        assert _ids_with_edit(b, tmp_path, name)["kernels"] != base["kernels"], name
    assert _ids_with_edit(b, tmp_path, "gf_kernels_wide.hpp")["wide"] != base["wide"]
    assert _ids_with_edit(b, tmp_path, "gf_kernels_packets.hpp")["packets"] != base["packets"]
    # the defaults of the knobs a family's dispatch reads are part of its ID, others are not
    cap = _ids_with_edit(b, tmp_path, "knobs.cpp", ('{"ECGPU_CAP", "cap", -1}', '{"ECGPU_CAP", "cap", 1}'))
    assert cap["kernels"] != base["kernels"] and cap["wide"] == base["wide"]
    pipe = _ids_with_edit(b, tmp_path, "knobs.cpp", ('{"ECGPU_WIDE_PIPE", "wide_pipe", 1}',
                                                     '{"ECGPU_WIDE_PIPE", "wide_pipe", 2}'))
    assert pipe["kernels"] == base["kernels"] and pipe["wide"] != base["wide"]


def test_lab_kernels_are_not_in_the_production_library():
    import shutil
    import subprocess
    if not shutil.which("nm"):
        pytest.skip("nm not installed")
    out = subprocess.run(["nm", "-C", LIB], capture_output=True, text=True, check=True).stdout
    for k in ("gf_apply_dma", "gf_apply_occ8", "gf_apply_perm_stream", "gf_apply_perm<", "diag_copy"):
        assert k not in out, k
    assert "gf_apply<10, 4, 3" in out


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
