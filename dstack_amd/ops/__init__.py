"""Fused ops for the MI355X training workload, each a hand-written HIP/CDNA4 kernel.

Every op is an ``autograd.Function`` whose forward/backward call ``dstack_amd.ops._C`` for ROCm
tensors and ``dstack_amd.ops.reference`` for CPU tensors (unit tests). See ``_ext`` for the
fail-loudly policy.

The ops are resolved lazily (PEP 562): importing ``dstack_amd.ops.build`` -- the first command of
a training job (``python -m dstack_amd.ops.build``) -- does not import torch when the extension is
already current.
"""

_OPS = ("adamw_", "add_rms_norm", "attention", "cross_entropy", "embedding", "linear", "qkv_rope_attention",
        "rms_norm", "rope", "swiglu", "swiglu_mlp", "weight_grad")


def __getattr__(name):
    import importlib

    if name in _OPS:
        return getattr(importlib.import_module("dstack_amd.ops.functional"), name)
    if name in ("_ext", "functional", "reference", "gemm_tuning", "serving", "build"):
        return importlib.import_module(f"dstack_amd.ops.{name}")
    raise AttributeError(f"module 'dstack_amd.ops' has no attribute {name!r}")


def __dir__():
    return sorted(list(globals()) + list(_OPS) + ["_ext"])
