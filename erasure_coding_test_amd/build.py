"""In-tree build of the native libraries (gfx950 only).

    python -m erasure_coding_test_amd.build          # or __graft_entry__.build()

Produces, under erasure_coding_test_amd/lib/:
  libecgpu.so        -- the C ABI of include/ecgpu.h: HIP kernels (hipcc,
                        --offload-arch=gfx950) + host C++ (g++)
  libjerasure_amd.so -- drop-in: the reference's C++ coding surface
                        (galois.h / jerasure.h / reed_sol.h names) on top of
                        libecgpu.so (rpath $ORIGIN)
and the test-only checker under oracle/ (make -C oracle).

Objects are rebuilt only when a source is newer than its object.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "lib")
OBJ = os.path.join(PKG, "build", "obj")
INCLUDE = os.path.join(ROOT, "include")

ARCH = os.environ.get("ECGPU_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", shutil.which("hipcc") or "/opt/rocm/bin/hipcc")
CXX = os.environ.get("CXX", "g++")

HOST_SRCS = ["gf_host.cpp", "matrix_host.cpp", "planner.cpp", "schedule_host.cpp", "capi_host.cpp"]
# (source, object, extra flags): the specialised kernel table is split into
# one translation unit per output-row count so the four compile in parallel
HIP_UNITS = [(f, f + ".o", []) for f in ("ecgpu_runtime.hip", "accum.hip", "pipeline.hip", "packets.hip")] + [
    ("gf_spec.hip", f"gf_spec_r{r}.hip.o", [f"-DECGPU_SPEC_R={r}"]) for r in (1, 2, 3, 4)]
HDRS = ["gf_host.hpp", "host_sync.hpp", "matrix_host.hpp", "planner.hpp", "schedule_host.hpp", "gf_kernels.hpp", "gf_spec.hpp",
        "runtime.hpp"]
DROPIN_SRCS = ["jerasure_dropin.cpp", "jerasure_surface.cpp"]

CXXFLAGS = ["-O2", "-std=c++17", "-fPIC", "-Wall", "-Wextra", "-Wno-unused-parameter", f"-I{INCLUDE}", f"-I{CSRC}"]
HIPFLAGS = ["-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-Wall", "-Wextra", "-Wno-unused-parameter", f"--offload-arch={ARCH}", f"-I{INCLUDE}", f"-I{CSRC}",
            "-Wno-unused-result"]


def _run(cmd):
    print("  " + " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


def _run_parallel(cmds):
    """hipcc jobs in parallel (each is single-threaded); fails on the first error."""
    from concurrent.futures import ThreadPoolExecutor
    if not cmds:
        return
    workers = max(1, min(len(cmds), int(os.environ.get("MAX_JOBS", "0")) or (os.cpu_count() or 1), 8))
    with ThreadPoolExecutor(workers) as ex:
        for f in [ex.submit(_run, c) for c in cmds]:
            f.result()


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _headers():
    return [os.path.join(CSRC, h) for h in HDRS] + [os.path.join(INCLUDE, "ecgpu.h")]


def build_native(verbose: bool = True) -> dict:
    os.makedirs(LIB, exist_ok=True)
    os.makedirs(OBJ, exist_ok=True)
    hdrs = _headers()
    objs = []
    for src in HOST_SRCS:
        s, o = os.path.join(CSRC, src), os.path.join(OBJ, src + ".o")
        if _stale(o, [s] + hdrs):
            _run([CXX] + CXXFLAGS + ["-fvisibility=hidden", "-c", s, "-o", o])
        objs.append(o)
    jobs = []
    for src, obj, extra in HIP_UNITS:
        s, o = os.path.join(CSRC, src), os.path.join(OBJ, obj)
        if _stale(o, [s] + hdrs):
            jobs.append([HIPCC] + HIPFLAGS + extra + ["-c", s, "-o", o])
        objs.append(o)
    _run_parallel(jobs)
    ecgpu = os.path.join(LIB, "libecgpu.so")
    if _stale(ecgpu, objs):
        _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-Wl,-soname,libecgpu.so"] + objs + ["-o", ecgpu])

    dropin_objs = []
    for src in DROPIN_SRCS:
        s, o = os.path.join(CSRC, src), os.path.join(OBJ, src + ".o")
        if _stale(o, [s] + hdrs + [os.path.join(INCLUDE, "dropin", h) for h in ("galois.h", "jerasure.h", "reed_sol.h")]):
            _run([CXX] + CXXFLAGS + [f"-I{os.path.join(INCLUDE, 'dropin')}", "-fvisibility=hidden",
                                     "-fvisibility-inlines-hidden", "-c", s, "-o", o])
        dropin_objs.append(o)
    # the CPU-surface code reuses the host GF / matrix objects (hidden symbols)
    dropin_objs += [os.path.join(OBJ, s + ".o") for s in ("gf_host.cpp", "matrix_host.cpp", "schedule_host.cpp")]
    dropin = os.path.join(LIB, "libjerasure_amd.so")
    if _stale(dropin, dropin_objs + [ecgpu]):
        _run([CXX, "-shared", "-fPIC"] + dropin_objs +
             ["-o", dropin, f"-L{LIB}", "-lecgpu", "-Wl,-rpath,$ORIGIN"])
    out = {"libecgpu": ecgpu, "libjerasure_amd": dropin}
    if os.environ.get("ECGPU_BUILD_DIAG", "1") != "0":
        s, o = os.path.join(CSRC, "diag_kernels.hip"), os.path.join(OBJ, "diag_kernels.hip.o")
        diag = os.path.join(LIB, "libecgpu_diag.so")
        if _stale(o, [s] + hdrs):
            _run([HIPCC] + HIPFLAGS + ["-c", s, "-o", o])
        if _stale(diag, [o]):
            _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", o, "-o", diag])
        out["libecgpu_diag"] = diag
    return out


def build_oracle():
    _run(["make", "-s", "-C", os.path.join(ROOT, "oracle")])


def main():
    out = build_native()
    build_oracle()
    for k, v in out.items():
        print(f"built {k}: {v}")


if __name__ == "__main__":
    sys.exit(main())
