"""In-tree build of the native libraries (gfx950 only).

    python erasure_coding_test_amd/build.py          # or __graft_entry__.build()

Produces, under erasure_coding_test_amd/lib/:
  libecgpu.so        -- the C ABI of include/ecgpu.h: HIP kernels (hipcc,
                        --offload-arch=gfx950) + host C++ (g++)
  libjerasure_amd.so -- drop-in: the reference's C++ coding surface
                        (galois.h / jerasure.h / reed_sol.h names) on top of
                        libecgpu.so (rpath $ORIGIN)
and the test-only checker under oracle/ (make -C oracle).

An object is rebuilt when its key changes: a SHA-256 of its compiler command
line and the bytes of its source and every header (stored beside it as
<object>.key), so neither a touched-but-unchanged file nor a stale object with
a newer mtime decides.  The library carries content IDs (ecgpu_build_id):
  0  the whole library: every source and header under csrc/ + ecgpu.h + flags
     + both compilers' --version
  1  the w = 8 kernels and their dispatch (gf_kernels_w8.hpp, gf_spec.*,
     dispatch_w8.hip and the defaults of the knobs it reads) + HIP flags +
     hipcc --version -- the identity a rocprofv3 PMC record of the bench's
     launches is valid for (profiles/summarize.py writes it, bench.py checks it)
  2  the same for the w = 16 / 32 kernels, 3 for the GF(2) packet kernels.
"""
from __future__ import annotations

import hashlib
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

HOST_SRCS = ["gf_host.cpp", "matrix_host.cpp", "planner.cpp", "schedule_host.cpp", "capi_host.cpp", "contract_host.cpp", "knobs.cpp",
             "cpu_fallback.cpp", "cpu_exec.cpp"]
# (source, object, extra flags): the specialised kernel table is split into
# one translation unit per output-row count so the four compile in parallel
HIP_UNITS = [(f, f + ".o", []) for f in ("ecgpu_runtime.hip", "dispatch_w8.hip", "dispatch_wide.hip", "accum.hip",
                                           "pipeline.hip", "packets.hip")] + [
    (f"{t}.hip", f"{t}_r{r}.hip.o", [f"-DECGPU_SPEC_R={r}"]) for t in ("gf_spec", "wide_spec") for r in (1, 2, 3, 4)]
HDRS = ["buffer_contract.hpp", "cpu_fallback.hpp", "cpu_exec.hpp", "gf_host.hpp", "knobs.hpp", "shard_stride.hpp", "host_sync.hpp", "matrix_host.hpp", "planner.hpp", "schedule_host.hpp", "gf_kernels.hpp", "gf_kernels_w8.hpp", "gf_kernels_wide.hpp",
        "gf_kernels_packets.hpp", "gf_spec.hpp", "wide_spec.hpp", "diag_kernels_w8.hpp",
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


# One build ID per kernel family: the kernel code, its
# instantiation table and its dispatch (grid, residency, engine and cache
# policy), plus the default values of the knobs that dispatch reads -- so a
# w = 32 or packet edit leaves the w = 8 ID, which the bench's PMC traffic
# records are keyed to, unchanged.  The synchronous calls' staging
# (ecgpu_runtime.hip) and the measurement-only kernels (diag_kernels*) are in
# no family.
KERNEL_FAMILIES = {
    "kernels": (["gf_kernels_w8.hpp", "gf_spec.hip", "gf_spec.hpp", "dispatch_w8.hip"],
                ["ECGPU_CAP", "ECGPU_BLOCKS_PER_CU", "ECGPU_KERNEL", "ECGPU_NT"]),
    "wide": (["gf_kernels_w8.hpp", "gf_kernels_wide.hpp", "wide_spec.hip", "wide_spec.hpp", "dispatch_wide.hip"],
             ["ECGPU_WIDE", "ECGPU_NIB16", "ECGPU_WIDE_UNITS", "ECGPU_WIDE_PIPE", "ECGPU_WIDE16_BPCU",
              "ECGPU_WIDE16_UNITS"]),
    "packets": (["gf_kernels_w8.hpp", "gf_kernels_packets.hpp", "packets.hip"], ["ECGPU_PACKET"]),
}


def knob_rows(names) -> list:
    """The knobs.cpp table rows of these knobs (their defaults), in order."""
    with open(os.path.join(CSRC, "knobs.cpp")) as f:
        lines = f.read().splitlines()
    return [ln.strip() for n in names for ln in lines if ln.strip().startswith('{"%s",' % n)]


def _digest(parts, files) -> str:
    h = hashlib.sha256()
    for p in parts:
        h.update(p.encode())
        h.update(b"\0")
    for f in files:
        h.update(os.path.basename(f).encode())
        h.update(b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


_versions: dict = {}


def toolchain(compiler: str) -> str:
    """`<compiler> --version` (cached per process): part of every object key
    and build ID, so a compiler change rebuilds everything and invalidates PMC
    records taken on the old code."""
    if compiler not in _versions:
        try:
            r = subprocess.run([compiler, "--version"], capture_output=True, text=True, timeout=60)
            _versions[compiler] = r.stdout.strip() or f"{compiler}: no version output"
        except (OSError, subprocess.SubprocessError) as ex:
            _versions[compiler] = f"{compiler}: {type(ex).__name__}"
    return _versions[compiler]


def build_ids() -> dict:
    """{'build', 'kernels' (w = 8), 'wide', 'packets'}: 16-hex content IDs (see
    the module doc and KERNEL_FAMILIES)."""
    all_srcs = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC)
                      if f.endswith((".hip", ".cpp", ".hpp")) and not f.startswith("diag_kernels"))
    hip, cxx = toolchain(HIPCC), toolchain(CXX)
    ids = {"build": _digest([ARCH, hip, cxx] + CXXFLAGS + HIPFLAGS,
                            all_srcs + [os.path.join(INCLUDE, "ecgpu.h")])[:16]}
    for name, (files, knobs) in KERNEL_FAMILIES.items():
        ids[name] = _digest([ARCH, hip] + HIPFLAGS + knob_rows(knobs), [os.path.join(CSRC, f) for f in files])[:16]
    return ids


def _stale(target, deps, cmd=()):
    """True when `target` must be rebuilt; records the new key when so (the
    caller builds it next; a failed build raises before anything reads it)."""
    key = _digest(list(cmd) + ([toolchain(cmd[0])] if cmd else []), [d for d in deps if os.path.exists(d)])
    stamp = target + ".key"
    try:
        with open(stamp) as f:
            if os.path.exists(target) and f.read().strip() == key:
                return False
    except OSError:
        pass
    _pending_keys[stamp] = key
    return True


_pending_keys: dict = {}


def _commit_keys():
    for stamp, key in _pending_keys.items():
        with open(stamp, "w") as f:
            f.write(key + "\n")
    _pending_keys.clear()


def _headers():
    return [os.path.join(CSRC, h) for h in HDRS] + [os.path.join(INCLUDE, "ecgpu.h")]


def build_native(verbose: bool = True) -> dict:
    os.makedirs(LIB, exist_ok=True)
    os.makedirs(OBJ, exist_ok=True)
    hdrs = _headers()
    ids = build_ids()
    objs = []
    for src in HOST_SRCS:
        s, o = os.path.join(CSRC, src), os.path.join(OBJ, src + ".o")
        extra = ([f'-DECGPU_BUILD_ID="{ids["build"]}"', f'-DECGPU_KERNEL_ID="{ids["kernels"]}"',
                  f'-DECGPU_WIDE_ID="{ids["wide"]}"', f'-DECGPU_PACKETS_ID="{ids["packets"]}"']
                 if src == "capi_host.cpp" else [])
        cmd = [CXX] + CXXFLAGS + extra + ["-fvisibility=hidden", "-c", s, "-o", o]
        if _stale(o, [s] + hdrs, cmd):
            _run(cmd)
        objs.append(o)
    jobs = []
    for src, obj, extra in HIP_UNITS:
        s, o = os.path.join(CSRC, src), os.path.join(OBJ, obj)
        cmd = [HIPCC] + HIPFLAGS + extra + ["-c", s, "-o", o]
        if _stale(o, [s] + hdrs, cmd):
            jobs.append(cmd)
        objs.append(o)
    _run_parallel(jobs)
    _commit_keys()
    ecgpu = os.path.join(LIB, "libecgpu.so")
    cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-Wl,-soname,libecgpu.so"] + objs + ["-o", ecgpu]
    if _stale(ecgpu, objs, cmd):
        _run(cmd)
        _commit_keys()

    dropin_objs = []
    for src in DROPIN_SRCS:
        s, o = os.path.join(CSRC, src), os.path.join(OBJ, src + ".o")
        cmd = [CXX] + CXXFLAGS + [f"-I{os.path.join(INCLUDE, 'dropin')}", "-fvisibility=hidden",
                                  "-fvisibility-inlines-hidden", "-c", s, "-o", o]
        if _stale(o, [s] + hdrs + [os.path.join(INCLUDE, "dropin", h) for h in ("galois.h", "jerasure.h", "reed_sol.h")],
                  cmd):
            _run(cmd)
            _commit_keys()
        dropin_objs.append(o)
    # the CPU-surface code reuses the host GF / matrix objects (hidden symbols)
    dropin_objs += [os.path.join(OBJ, s + ".o") for s in ("gf_host.cpp", "matrix_host.cpp", "schedule_host.cpp")]
    dropin = os.path.join(LIB, "libjerasure_amd.so")
    cmd = [CXX, "-shared", "-fPIC"] + dropin_objs + ["-o", dropin, f"-L{LIB}", "-lecgpu", "-Wl,-rpath,$ORIGIN"]
    if _stale(dropin, dropin_objs + [ecgpu], cmd):
        _run(cmd)
        _commit_keys()
    out = {"libecgpu": ecgpu, "libjerasure_amd": dropin, "build_ids": ids}
    if os.environ.get("ECGPU_BUILD_DIAG", "1") != "0":
        s, o = os.path.join(CSRC, "diag_kernels.hip"), os.path.join(OBJ, "diag_kernels.hip.o")
        diag = os.path.join(LIB, "libecgpu_diag.so")
        cmd = [HIPCC] + HIPFLAGS + ["-c", s, "-o", o]
        if _stale(o, [s] + hdrs, cmd):
            _run(cmd)
            _commit_keys()
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", o, "-o", diag]
        if _stale(diag, [o], cmd):
            _run(cmd)
            _commit_keys()
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
