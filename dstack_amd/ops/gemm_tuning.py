"""Offline GEMM algorithm selection for the plain library GEMMs (hipBLASLt / rocBLAS through
PyTorch TunableOp).

The Llama projections are a handful of fixed shapes (per model, seq_len and micro-batch), so the
best hipBLASLt solution per shape is found once on an MI355X (``mode="tune"``) and shipped as a
results CSV next to this file; training runs load it with tuning disabled (``mode="use"``), so no
step ever pays for tuning.  The CSV carries TunableOp's validators (ROCm, hipBLASLt, gfx arch);
on a mismatch PyTorch ignores it and falls back to the default heuristics.

``DSTACK_AMD_GEMM_TUNING`` = ``use`` (default when the file exists) | ``tune`` | ``off``.
"""

from __future__ import annotations

import os
from pathlib import Path
from typing import Optional

TUNED_DIR = Path(__file__).resolve().parent / "tuned"


def results_path(arch: str = "gfx950", kind: str = "train") -> Path:
    """``kind`` = ``train`` (Llama training projections) or ``serving`` (the decode GEMMs of the
    serving engine: M = every hipGraph batch bucket, N/K = the fused projections and LM head)."""
    override = os.environ.get("DSTACK_AMD_GEMM_TUNING_FILE")
    if override:
        return Path(override)
    return TUNED_DIR / (f"gemm_tunableop_{arch}.csv" if kind == "train" else f"gemm_tunableop_{kind}_{arch}.csv")


def setup(mode: Optional[str] = None, device_index: int = 0, kind: str = "train") -> str:
    """Configure TunableOp before the first GEMM.  Returns the effective mode."""
    import torch

    if not torch.cuda.is_available() or torch.version.hip is None:
        return "off"
    mode = (mode or os.environ.get("DSTACK_AMD_GEMM_TUNING") or "use").lower()
    arch = torch.cuda.get_device_properties(device_index).gcnArchName.split(":")[0]
    path = results_path(arch, kind)
    tunable = torch.cuda.tunable
    if mode == "off":
        tunable.enable(False)
        return "off"
    if mode == "tune":
        path.parent.mkdir(parents=True, exist_ok=True)
        tunable.enable(True)
        tunable.tuning_enable(True)
        tunable.set_max_tuning_duration(int(os.environ.get("DSTACK_AMD_GEMM_TUNE_MS", "200")))
        tunable.set_max_tuning_iterations(int(os.environ.get("DSTACK_AMD_GEMM_TUNE_ITERS", "50")))
        tunable.set_filename(str(path), insert_device_ordinal=False)
        if path.exists():
            tunable.read_file(str(path))
        return "tune"
    if not path.exists():
        tunable.enable(False)
        return "off"
    tunable.enable(True)
    tunable.tuning_enable(False)
    # never write back from a production run (all ranks share one read-only file)
    tunable.set_filename(os.path.join("/tmp", f"dstack_amd_tunableop_unused_{os.getpid()}.csv"),
                         insert_device_ordinal=False)
    tunable.read_file(str(path))
    return "use"


def flush():
    """Tune mode: TunableOp writes the results file when the process exits normally."""
    return None
