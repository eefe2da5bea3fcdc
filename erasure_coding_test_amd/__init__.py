"""MI355X-native Reed-Solomon GF(2^8) erasure coding.

Drop-in for the coding hot path of canghaiyang/Erasure_Coding_Test (its
vendored Jerasure: galois.h / jerasure.h / reed_sol.h).  The native pieces
live in erasure_coding_test_amd/lib/ (built in-tree for gfx950):

* libecgpu.so        -- C ABI (include/ecgpu.h): HIP kernels + host planning
* libjerasure_amd.so -- the reference's C++ surface on top of it

Python mirrors the reference API by module (``galois``, ``reed_sol``,
``jerasure``) and adds the batched device-resident ``plan`` API.
"""
from . import _native  # noqa: F401  -- fails loudly if the HIP extension is missing
from . import ecx, formats, galois, jerasure, pipeline, plan, reed_sol  # noqa: F401
from .pipeline import HostPipeline, HostPipelineGroup  # noqa: F401
from .ecx import ParityAccumulator  # noqa: F401
from .plan import DecodePlan, StripePlan, alloc_stripes, encode_plan  # noqa: F401

__all__ = ["galois", "jerasure", "reed_sol", "formats", "plan", "StripePlan", "DecodePlan", "encode_plan", "alloc_stripes", "ecx",
           "ParityAccumulator", "pipeline", "HostPipeline", "HostPipelineGroup"]
