"""Loader for the in-tree HIP/CDNA4 extension ``dstack_amd/ops/_C*.so``.

The extension is built for gfx950 only (``python setup.py build_ext --inplace`` or
``__graft_entry__.build()``). On a ROCm device the HIP path is mandatory: if the ``.so`` is
missing we raise instead of silently falling back to PyTorch. ``DSTACK_AMD_OPS=torch`` is an
explicit, opt-in A/B switch that routes GPU tensors through ``ops.reference``.
"""

from __future__ import annotations

import os

import torch

_C = None
_IMPORT_ERROR: Exception | None = None

try:  # pragma: no cover - depends on a built extension
    from dstack_amd.ops import _C as _C  # type: ignore[attr-defined,no-redef]
except Exception as e:  # noqa: BLE001
    _IMPORT_ERROR = e


def available() -> bool:
    return _C is not None


def force_torch() -> bool:
    return os.environ.get("DSTACK_AMD_OPS", "hip").lower() == "torch"


def use_hip(t: torch.Tensor) -> bool:
    """True when ``t`` must go through the HIP kernels."""
    if not t.is_cuda or force_torch():
        return False
    require()
    return True


def require():
    if _C is None:
        raise RuntimeError(
            "dstack_amd HIP extension (_C) is not built/importable on a GPU run; run "
            "`python setup.py build_ext --inplace` (PYTORCH_ROCM_ARCH=gfx950). "
            f"Import error: {_IMPORT_ERROR!r}"
        )
    return _C
