"""The training workload trains at the bench shape: Llama-3-8B's layer (dim 4096, 32 heads of 128,
8 KV heads, FFN 14336, vocab 128256) in a 4-layer stack (Llama-3.2-1B itself has head_dim 64,
which the HIP flash-attention kernels do not take), seq 8192, one fixed batch, 30 optimizer steps
with LR warmup.
Under the HIP path the loss falls (memorising the batch) monotonically after warmup, and it
tracks the ``DSTACK_AMD_OPS=torch`` path (PyTorch-ROCm SDPA / library ops, fp32 reference
AdamW) step by step."""

import gc

import pytest
import torch

pytestmark = pytest.mark.gpu

STEPS, WARMUP = 30, 5


def _train(gpu, ops, monkeypatch):
    import dataclasses

    from dstack_amd.models.llama import CONFIGS
    from dstack_amd.workloads.train_llama import Trainer

    monkeypatch.setitem(CONFIGS, "llama-3-8b-4l", dataclasses.replace(CONFIGS["llama-3-8b"], name="llama-3-8b-4l",
                                                                      n_layers=4))
    monkeypatch.setenv("DSTACK_AMD_OPS", ops)
    tr = Trainer("llama-3-8b-4l", seq_len=8192, micro_batch=1, device=gpu, lr=3e-4, lr_warmup=WARMUP,
                 data="fixed", data_rows=1, bucket_numel=64 * 1024 * 1024)
    losses = [tr.step().item() for _ in range(STEPS)]
    del tr
    gc.collect()
    torch.cuda.empty_cache()
    return losses


def test_llama3_layers_seq8192_loss_falls_and_tracks_torch_path(gpu, monkeypatch):
    import math

    hip = _train(gpu, "hip", monkeypatch)
    ref = _train(gpu, "torch", monkeypatch)
    print("hip", [round(x, 6) for x in hip])
    print("torch", [round(x, 6) for x in ref])
    ln_v = math.log(128256)
    assert all(math.isfinite(x) for x in hip + ref)
    assert max(hip[2:]) < ln_v + 1.0  # no blow-up past the uniform-prediction loss
    for a, b in zip(hip[WARMUP:], hip[WARMUP + 1:]):
        assert b <= a * 1.02 + 0.02, hip  # monotone after warmup (2 % slack for bf16 noise)
    assert hip[-1] < 0.5 * hip[0]
    for i, (a, b) in enumerate(zip(hip, ref)):
        assert abs(a - b) <= 0.05 * abs(b) + 0.1, (i, hip, ref)


def test_grad_accum8_bf16_vs_fp32_accumulation(gpu, monkeypatch):
    """Gradient precision of the bench's step (8 micro-batches of 8192 tokens, 4 Llama-3-8B layers):
    the flat bf16 gradients with the default bf16 accumulation (one rounding per micro-batch in the
    weight-gradient GEMM's epilogue) and with the fp32 accumulator (DSTACK_AMD_GRAD_ACCUM_FP32: one
    rounding per step), per tensor, against the fp32-accumulated GEMM outputs.  Same parameters, same
    data, deterministic kernels: the three runs differ only in how the micro-batches are summed.
    Prints the per-tensor relative errors (docs/reference/performance.md quotes them)."""
    import dataclasses
    import statistics

    from dstack_amd.models.llama import CONFIGS
    from dstack_amd.workloads.train_llama import Trainer

    monkeypatch.setitem(CONFIGS, "llama-3-8b-4l", dataclasses.replace(CONFIGS["llama-3-8b"], name="llama-3-8b-4l",
                                                                      n_layers=4))
    n = 8
    tr = Trainer("llama-3-8b-4l", seq_len=8192, micro_batch=1, device=gpu, grad_accum=n,
                 bucket_numel=64 * 1024 * 1024)
    opt = tr.opt
    opt._side = None  # no optimizer-in-backward: the parameters stay fixed across the three runs
    batches = [tr.batch() for _ in range(n)]

    def run(fp32: bool):
        opt.grad_accum_fp32 = fp32
        opt.zero_grad()
        for i, (x, y) in enumerate(batches):
            opt.sync_grads = i == n - 1
            (tr.model.loss(x, y) / n).backward()
        torch.cuda.synchronize()
        return opt.flat_grad.float().clone()

    g16 = run(False)
    g32 = run(True)
    # reference: the weight gradients of the fp32 run before its final rounding = acc32 + the last
    # micro-batch's product; recomputed exactly by a fresh fp32 accumulation of all n micro-batches
    # through the same fp32 GEMM epilogue and read from the accumulator (mode 1 for the last one)
    opt.grad_accum_fp32 = True
    opt.zero_grad()
    for i, (x, y) in enumerate(batches):
        opt.sync_grads = False  # every micro-batch, the last included, stays in the fp32 accumulator
        (tr.model.loss(x, y) / n).backward()
    torch.cuda.synchronize()
    ref = opt.acc32
    errs16, errs32 = [], []
    for p in tr.model.parameters():
        if p.dim() != 2 or p is tr.model.embed:
            continue  # GEMM weight gradients only (norms and the embedding accumulate in bf16 in both)
        o, k = opt._offset[p], p.numel()
        r = ref[o : o + k]
        rn = r.norm().item()
        errs16.append(((g16[o : o + k] - r).norm().item() / rn))
        errs32.append(((g32[o : o + k] - r).norm().item() / rn))
    print(f"{len(errs16)} weight gradients; rel err bf16-accum median {statistics.median(errs16):.3e} "
          f"max {max(errs16):.3e}; fp32-accum median {statistics.median(errs32):.3e} max {max(errs32):.3e}")
    assert max(errs32) < 3e-3  # one bf16 rounding
    assert statistics.median(errs32) < statistics.median(errs16)
    assert max(errs16) < 2e-2
    del tr, opt
    gc.collect()
    torch.cuda.empty_cache()
