"""Fused ops for the MI355X training workload, each a hand-written HIP/CDNA4 kernel.

Every op is an ``autograd.Function`` whose forward/backward call ``dstack_amd.ops._C`` for ROCm
tensors and ``dstack_amd.ops.reference`` for CPU tensors (unit tests). See ``_ext`` for the
fail-loudly policy.
"""

from dstack_amd.ops.functional import (  # noqa: F401
    adamw_,
    add_rms_norm,
    attention,
    cross_entropy,
    embedding,
    linear,
    rms_norm,
    rope,
    swiglu,
    swiglu_mlp,
    weight_grad,
)
from dstack_amd.ops import _ext  # noqa: F401
