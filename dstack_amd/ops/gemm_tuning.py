"""Offline GEMM algorithm selection for the plain library GEMMs (hipBLASLt / rocBLAS through
PyTorch TunableOp).

The Llama projections are a handful of fixed shapes (per model, seq_len and micro-batch), so the
best hipBLASLt solution per shape is found once on an MI355X (``mode="tune"``) and shipped as a
results CSV next to this file; training runs load it with tuning disabled (``mode="use"``), so no
step ever pays for tuning.  The CSV carries TunableOp's validators (ROCm, hipBLASLt, gfx arch);
on a mismatch PyTorch ignores it and falls back to the default heuristics.

``DSTACK_AMD_GEMM_TUNING`` = ``use`` | ``tune`` | ``off``.  Default: ``off`` for training (since the
weight gradients moved to the in-tree GEMM, hipBLASLt's own heuristics run the remaining training
GEMMs as fast as the tuned selections -- 22.70/22.72k vs 22.67/22.65k tokens/s, same box,
profiles/gemm_tuning_ab_r8h.txt -- and skip TunableOp's ~1 s first-call set-up, which sat on every
job's start), ``use`` for serving (the tuned fp8 decode GEMMs are up to 2.8x faster).
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
    mode = (mode or os.environ.get("DSTACK_AMD_GEMM_TUNING") or ("off" if kind == "train" else "use")).lower()
    tunable = torch.cuda.tunable
    if mode == "off":
        # TunableOp is off unless PYTORCH_TUNABLEOP_ENABLED says otherwise; touching it (86-140 ms:
        # its context is created on first use) or the device properties (106-124 ms on first call)
        # sat on every job's start-up path (tools/diag/init_split.py, profiles/init_split_r9n.txt)
        if os.environ.get("PYTORCH_TUNABLEOP_ENABLED", "0") not in ("0", ""):
            tunable.enable(False)
        return "off"
    arch = torch.cuda.get_device_properties(device_index).gcnArchName.split(":")[0]
    path = results_path(arch, kind)
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


def llama_shapes(cfg, tokens: int):
    """(M, N, K) of every ``a @ b.t()`` library GEMM of a Llama training micro-batch that the
    in-tree GEMM does not run: the forward projections (qkv, o, down, LM head) and the input
    gradients through the cached W^T (qkv, o, gate/up, LM head)."""
    d, hd = cfg.dim, cfg.dim // cfg.n_heads
    qkv = (cfg.n_heads + 2 * cfg.n_kv_heads) * hd
    return [(tokens, qkv, d), (tokens, d, d), (tokens, d, cfg.ffn_dim), (tokens, cfg.vocab_size, d),
            (tokens, d, qkv), (tokens, d, 2 * cfg.ffn_dim), (tokens, d, cfg.vocab_size)]


def prewarm(shapes, device, extra=None):
    """Start a thread that runs one ``a @ b.t()`` per shape on a side stream, so the library's
    first-call work -- hipBLASLt's handle and heuristics (0.17 s on the first GEMM of a process), and
    with ``use`` TunableOp mapping its saved selections onto hipBLASLt's solution list (1.1 s,
    profiles/first_step_r8b.txt, tools/diag/gemm_first_call.py), plus loading each selected kernel --
    overlaps the model's initialisation instead of landing in the first forward.  Not while tuning.  ``extra`` (a
    callable) runs on the same thread afterwards: the first use of the data pipeline's kernels.  Returns the thread
    (join it before the first step) or None."""
    import threading

    import torch

    tunable = torch.cuda.tunable
    if device.type != "cuda" or (tunable.is_enabled() and tunable.tuning_is_enabled()):
        return None
    if os.environ.get("DSTACK_AMD_GEMM_PREWARM", "1") == "0" and not float(os.environ.get("DSTACK_AMD_ACT_POOL_GB", "0") or 0):
        return None

    def work():
        torch.cuda.set_device(device)
        st = torch.cuda.Stream(device=device)
        with torch.cuda.stream(st):
            for m, n, k in shapes:
                a = torch.empty(m, k, device=device, dtype=torch.bfloat16)
                b = torch.empty(n, k, device=device, dtype=torch.bfloat16)
                torch.mm(a.zero_(), b.zero_().t())
                del a, b
        st.synchronize()
        # the caching allocator ties freed blocks to the stream that allocated them: released here,
        # the side stream's operands (the LM-head pair alone is ~2 x 2 GiB at 8k tokens) would stay
        # reserved for the whole run, unusable by the default stream's training step
        torch.cuda.empty_cache()
        # DSTACK_AMD_ACT_POOL_GB: reserve the first step's activation memory here, beside model
        # init, as one default-stream segment the caching allocator then splits (the first forward
        # otherwise grows the pool with hipMalloc calls inside the timed-to-first-step path)
        gb = float(os.environ.get("DSTACK_AMD_ACT_POOL_GB", "0") or 0)
        if gb > 0:
            pool = torch.empty(int(gb * 2**30), dtype=torch.uint8, device=device)
            del pool
        if extra is not None:
            extra()
            torch.cuda.current_stream(device).synchronize()

    th = threading.Thread(target=work, name="gemm-prewarm", daemon=True)
    th.start()
    return th


def flush():
    """Tune mode: TunableOp writes the results file when the process exits normally."""
    return None
