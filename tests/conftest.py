import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TESTS = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, TESTS):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN_DIR = os.path.join(TESTS, "golden")
REFERENCE_ROOT = "/root/reference"

# No test result may come from the library's CPU executor (csrc/cpu_exec.hpp):
# neither the fallback after a HIP error nor the small-call
# routing below ECGPU_MIN_OFFLOAD_KIB -- both off for this process and every
# process a test starts, unless the test sets them itself
# (tests/test_cpu_fallback.py, tests/test_cpu_exec.py).  ECGPU_TEST_INJECT_HIP
# is the drivers' own variable (the library never reads it; they set the
# test_inject_hip knob from it).
os.environ["ECGPU_CPU_FALLBACK"] = "0"
os.environ["ECGPU_MIN_OFFLOAD_KIB"] = "0"
os.environ.pop("ECGPU_GPU", None)
os.environ.pop("ECGPU_TEST_INJECT_HIP", None)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box with -m gpu)")
    import refcheck
    refcheck.configure(config)


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(GOLDEN_DIR, "golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def vectors():
    with np.load(os.path.join(GOLDEN_DIR, "vectors.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def restatement():
    from oracle.oracle import Restatement
    return Restatement()


@pytest.fixture(scope="session")
def reference():
    from oracle.oracle import Reference
    try:
        return Reference()
    except (FileNotFoundError, OSError):
        import refcheck
        refcheck.reference_missing("oracle/_ref/libjerasure_ref.so")


@pytest.fixture(scope="session")
def gpu():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X (run with -m gpu on the GPU box)"
    import erasure_coding_test_amd  # noqa: F401
    return torch.device("cuda:0")


@pytest.fixture
def knobs():
    """The library's tuning knobs (ecgpu_set_knob), restored after the test:
    the environment is read once per process, so in-process switches go
    through the setter."""
    from erasure_coding_test_amd import _native as N

    class Knobs:
        @staticmethod
        def set(name, value):
            N.set_knob(name, int(value))

        @staticmethod
        def reset(name):
            N.reset_knob(name)

    yield Knobs()
    N.reset_knob(None)


@pytest.fixture(autouse=True)
def _no_cpu_fallback():
    """Every test ends with ecgpu_fallback_count() == ecgpu_cpu_call_count() ==
    0 in this process: a GPU result that silently came from the CPU would void
    the parity claims."""
    yield
    N = sys.modules.get("erasure_coding_test_amd._native")
    if N is not None:
        assert N.fallback_count() == 0, "a synchronous call completed on the CPU fallback inside the test session"
        assert N.cpu_call_count() == 0, "a synchronous call ran on the CPU executor inside the test session"
