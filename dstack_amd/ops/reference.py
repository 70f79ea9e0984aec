"""Plain-PyTorch fp32 reference implementations of every fused op.

These are (a) the numerics oracle the HIP kernels are tested against and (b) the CPU path used by
the CPU-only unit tests. They are never used silently on a GPU: ``dstack_amd.ops`` raises if the
HIP extension is missing on a ROCm device (see ``_ext.require``), unless the user explicitly asks
for ``DSTACK_AMD_OPS=torch`` (A/B benchmarking).
"""

from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    r = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return (xf * r * w.float()).to(x.dtype)


def add_rms_norm(x: torch.Tensor, delta: torch.Tensor, w: torch.Tensor, eps: float):
    h = (x.float() + delta.float()).to(x.dtype)
    return h, rms_norm(h, w, eps)


def swiglu(gu: torch.Tensor) -> torch.Tensor:
    f = gu.shape[-1] // 2
    g, u = gu[..., :f].float(), gu[..., f:].float()
    return (F.silu(g) * u).to(gu.dtype)


def rope_cos_sin(seq_len: int, head_dim: int, theta: float, device=None):
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    t = torch.arange(seq_len, dtype=torch.float64)
    ang = torch.outer(t, inv)
    return ang.cos().float().to(device), ang.sin().float().to(device)


def apply_rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    """x: [B, S, H, D] (rotate-half convention, as Llama-3 / HF)."""
    d2 = x.shape[-1] // 2
    xf = x.float()
    x1, x2 = xf[..., :d2], xf[..., d2:]
    c = cos[: x.shape[1]].view(1, x.shape[1], 1, d2)
    s = sin[: x.shape[1]].view(1, x.shape[1], 1, d2)
    return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1).to(x.dtype)


def attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, causal: bool = True) -> torch.Tensor:
    """q: [B, S, H, D], k/v: [B, S, KV, D] → [B, S, H, D] (GQA by head repetition)."""
    b, s, h, d = q.shape
    kvh = k.shape[2]
    rep = h // kvh
    qf = q.float().transpose(1, 2)
    kf = k.float().transpose(1, 2).repeat_interleave(rep, dim=1)
    vf = v.float().transpose(1, 2).repeat_interleave(rep, dim=1)
    scores = qf @ kf.transpose(-1, -2) / math.sqrt(d)
    if causal:
        mask = torch.ones(s, kf.shape[2], dtype=torch.bool, device=q.device).triu(1)
        scores = scores.masked_fill(mask, float("-inf"))
    p = scores.softmax(-1)
    return (p @ vf).transpose(1, 2).to(q.dtype)


E4M3_MAX = 448.0


def quant_fp8_rows(x: torch.Tensor):
    """Per-row e4m3 quantization (csrc/fp8.hip ``quant_rows``): q [M, K] float8_e4m3fn, s [M] fp32
    with s = max|x_row| / 448, x ~= q * s."""
    xf = x.float()
    s = xf.abs().amax(dim=1).clamp_min(1e-12) / E4M3_MAX
    q = (xf / s[:, None]).clamp(-E4M3_MAX, E4M3_MAX).to(torch.float8_e4m3fn)
    return q, s


def fp8_linear(x: torch.Tensor, q: torch.Tensor, s: torch.Tensor) -> torch.Tensor:
    """x @ (q * s)^T with x quantized per row first: the math of the fp8 serving GEMMs, in fp32."""
    xq, xs = quant_fp8_rows(x)
    return ((xq.float() * xs[:, None]) @ (q.float() * s[:, None]).t()).to(x.dtype)


def cross_entropy(logits: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    return F.cross_entropy(logits.float(), target, reduction="mean")


def adamw_(
    param: torch.Tensor,
    grad: torch.Tensor,
    master: torch.Tensor,
    m: torch.Tensor,
    v: torch.Tensor,
    lr: float,
    beta1: float,
    beta2: float,
    eps: float,
    weight_decay: float,
    step: int,
    grad_scale: float = 1.0,
) -> None:
    """Decoupled-weight-decay Adam on an fp32 master copy; writes the bf16 param back."""
    g = grad.float() * grad_scale
    m.mul_(beta1).add_(g, alpha=1 - beta1)
    v.mul_(beta2).addcmul_(g, g, value=1 - beta2)
    bc1 = 1 - beta1**step
    bc2 = 1 - beta2**step
    master.mul_(1 - lr * weight_decay)
    denom = (v / bc2).sqrt_().add_(eps)
    master.addcdiv_(m, denom, value=-lr / bc1)
    param.copy_(master.to(param.dtype))
