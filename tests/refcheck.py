"""Missing-reference policy shared by the test modules.

The reference-backed parity tests load oracle/_ref (the reference's own
src/erasure_coding compiled in this container and shipped with the tree).
Where that build is absent they skip -- except in a GPU run (-m gpu), where a
missing _ref would silently turn the parity suite into skips: there it fails.
"""
import pytest

_STATE = {"gpu_selected": False}


def configure(config) -> None:
    expr = (config.option.markexpr or "").replace(" ", "")
    _STATE["gpu_selected"] = "gpu" in expr and "notgpu" not in expr


def reference_missing(what: str):
    msg = f"{what} not built (make -C oracle where /root/reference exists; the tree ships it to the GPU box)"
    if _STATE["gpu_selected"]:
        pytest.fail(msg + " -- required by the -m gpu parity suite")
    pytest.skip(msg)
