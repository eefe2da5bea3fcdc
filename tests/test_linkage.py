"""The reference's own callers build and link, unchanged, against the drop-in.

Compiles src/client/client_main.cpp, src/eck_datanode/eck_datanode_main.cpp
and src/ecx_datanode/ecx_datanode_main.cpp from /root/reference (read as
compiler input only; outputs go to a temp dir) with (a) our drop-in headers
include/dropin/*.h and (b) the reference's own headers, then links them
against libjerasure_amd.so with no reference coding object.  `client -h`
runs.  Needs /root/reference (this container); skipped elsewhere.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
LIB = os.path.join(ROOT, "erasure_coding_test_amd", "lib")
APPS = {
    "client": "src/client/client_main.cpp",
    "eck": "src/eck_datanode/eck_datanode_main.cpp",
    "ecx": "src/ecx_datanode/ecx_datanode_main.cpp",
}

pytestmark = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "src")), reason="needs /root/reference")


@pytest.mark.parametrize("headers", ["dropin", "reference"])
@pytest.mark.parametrize("app", sorted(APPS))
def test_reference_app_links_against_dropin(tmp_path, app, headers):
    inc = [f"-I{os.path.join(ROOT, 'include', 'dropin')}"] if headers == "dropin" else []
    inc.append(f"-I{os.path.join(REF, 'include')}")  # ych_ec_test.h (and, for "reference", the coding headers)
    exe = tmp_path / app
    cmd = (["g++", "-O1", "-w", "-o", str(exe), os.path.join(REF, APPS[app])] + inc +
           [f"-L{LIB}", "-ljerasure_amd", f"-Wl,-rpath,{LIB}", "-lpthread"])
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    undefined = subprocess.run(["nm", "-u", "-C", str(exe)], capture_output=True, text=True).stdout
    used = sorted({l.strip()[2:].split("(")[0] for l in undefined.splitlines()
                   if l.strip().startswith("U ") and any(t in l for t in ("jerasure_", "galois_", "reed_sol_"))})
    expected = {"client": ["jerasure_matrix_decode", "jerasure_matrix_encode", "reed_sol_vandermonde_coding_matrix"],
                "ecx": ["galois_region_xor", "galois_w08_region_multiply", "reed_sol_vandermonde_coding_matrix"],
                "eck": []}[app]
    assert used == expected, used  # SURVEY.md §8b caller surface
    if app == "client":
        out = subprocess.run([str(exe), "-h"], capture_output=True, text=True, timeout=30)
        assert out.returncode == 0
