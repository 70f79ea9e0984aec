"""Llama-3 family decoder (the workload the orchestrator's headline benchmark runs).

MI355X-first layout choices:

* fused projections — one ``Wqkv`` [(H + 2*KV)*D, dim] and one ``Wgu`` [2*F, dim] GEMM per layer, so
  hipBLASLt sees few, large GEMMs (M = tokens ≥ 8192) instead of 5 small ones;
* activations stay in [B, S, heads, D] — the HIP flash-attention kernel reads q/k/v as strided views
  of the fused qkv output, no transposes;
* every elementwise/normalisation step is a fused HIP kernel (``dstack_amd.ops``): residual-add is
  folded into the next RMSNorm, RoPE is one pass over qkv, SwiGLU forward/backward run in the
  epilogues of the in-tree gate/up and down-projection GEMMs (``ops.swiglu_mlp``), the loss never
  materialises fp32 logits.

Reference parity: the reference orchestrator ships no model code; its Llama workloads are user
containers (``examples/fine-tuning/pytorch-distributed/train.dstack.yml``,
``examples/fine-tuning/trl``). This module is the MI355X-native equivalent of that workload.
"""

from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn as nn

from dstack_amd import ops
from dstack_amd.ops import reference as ref


@dataclass
class LlamaConfig:
    name: str = "llama-3-8b"
    dim: int = 4096
    n_layers: int = 32
    n_heads: int = 32
    n_kv_heads: int = 8
    ffn_dim: int = 14336
    vocab_size: int = 128256
    rope_theta: float = 500000.0
    norm_eps: float = 1e-5
    max_seq_len: int = 8192

    @property
    def head_dim(self) -> int:
        return self.dim // self.n_heads

    def num_params(self) -> int:
        d, f, v, L = self.dim, self.ffn_dim, self.vocab_size, self.n_layers
        qkv = d * (self.n_heads + 2 * self.n_kv_heads) * self.head_dim
        per_layer = qkv + d * d + 3 * d * f + 2 * d
        return L * per_layer + 2 * v * d + d

    def flops_per_token(self, seq_len: int) -> float:
        """Training FLOPs/token: 6·N_matmul + causal attention (fwd 2·2·S·D·H/2, ×3 for bwd)."""
        n_mm = self.num_params() - self.vocab_size * self.dim - (2 * self.n_layers + 1) * self.dim
        attn = 3 * 2 * 2 * self.n_layers * self.n_heads * self.head_dim * seq_len / 2
        return 6 * n_mm + attn


CONFIGS = {
    "llama-3-8b": LlamaConfig(),
    "llama-3-70b": LlamaConfig(
        name="llama-3-70b", dim=8192, n_layers=80, n_heads=64, n_kv_heads=8, ffn_dim=28672
    ),
    "llama-3.2-1b": LlamaConfig(
        name="llama-3.2-1b", dim=2048, n_layers=16, n_heads=32, n_kv_heads=8, ffn_dim=8192
    ),
    # tiny config used by CPU unit tests and the GPU smoke test (head_dim 128: the flash kernel's tile)
    "llama-tiny": LlamaConfig(
        name="llama-tiny", dim=512, n_layers=2, n_heads=4, n_kv_heads=2, ffn_dim=1024, vocab_size=1024,
        max_seq_len=256,
    ),
}


class DecoderLayer(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.cfg = cfg
        hd = cfg.head_dim
        self.attn_norm = nn.Parameter(torch.ones(cfg.dim))
        self.wqkv = nn.Parameter(torch.empty((cfg.n_heads + 2 * cfg.n_kv_heads) * hd, cfg.dim))
        self.wo = nn.Parameter(torch.empty(cfg.dim, cfg.n_heads * hd))
        self.ffn_norm = nn.Parameter(torch.ones(cfg.dim))
        self.wgu = nn.Parameter(torch.empty(2 * cfg.ffn_dim, cfg.dim))
        self.wdown = nn.Parameter(torch.empty(cfg.dim, cfg.ffn_dim))

    def forward(self, x, delta, cos, sin):
        """``x`` is the residual stream, ``delta`` the previous block's output still to be added
        (fused into this layer's first RMSNorm).  Returns the new (x, delta)."""
        cfg = self.cfg
        b, s, _ = x.shape
        hd = cfg.head_dim
        if delta is None:
            h = ops.rms_norm(x, self.attn_norm, cfg.norm_eps)
        else:
            x, h = ops.add_rms_norm(x, delta, self.attn_norm, cfg.norm_eps)
        o = ops.qkv_rope_attention(h, self.wqkv, cos, sin, cfg.n_heads, cfg.n_kv_heads)
        attn_out = ops.linear(o, self.wo)
        x, h = ops.add_rms_norm(x, attn_out, self.ffn_norm, cfg.norm_eps)
        return x, ops.swiglu_mlp(h, self.wgu, self.wdown)


class Llama(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.cfg = cfg
        self.embed = nn.Parameter(torch.empty(cfg.vocab_size, cfg.dim))
        self.layers = nn.ModuleList([DecoderLayer(cfg) for _ in range(cfg.n_layers)])
        self.norm = nn.Parameter(torch.ones(cfg.dim))
        self.lm_head = nn.Parameter(torch.empty(cfg.vocab_size, cfg.dim))
        self._rope_cache: dict = {}
        # set by ZeroOptimizer.install_prefetch_hooks: blocks until the all-gather of the given
        # (updated) parameters has landed, so embedding/head wait only when they are used
        self.param_waiter = None

    @torch.no_grad()
    def init_weights(self, std: float = 0.02, seed: int = 0, lm_head_std: float | None = None):
        """Normal(0, std) weights, GPT-2 residual scaling (std / sqrt(2 L)) for the projections
        that write into the residual stream, unit norms.  ``lm_head_std`` overrides the output
        head's std (0 = zero-init: uniform logits, an initial loss of exactly ln(vocab))."""
        g = torch.Generator(device=self.embed.device).manual_seed(seed)
        out_std = std / math.sqrt(2 * self.cfg.n_layers)
        for name, p in self.named_parameters():
            if p.dim() == 1:
                p.fill_(1.0)
            elif name.endswith("wo") or name.endswith("wdown"):
                p.normal_(0.0, out_std, generator=g)
            else:
                p.normal_(0.0, std, generator=g)
        if lm_head_std is not None:
            if lm_head_std == 0:
                self.lm_head.zero_()
            else:
                self.lm_head.normal_(0.0, lm_head_std, generator=g)

    def rope_tables(self, seq_len: int, device):
        key = (seq_len, str(device))
        if key not in self._rope_cache:
            self._rope_cache[key] = ref.rope_cos_sin(seq_len, self.cfg.head_dim, self.cfg.rope_theta, device)
        return self._rope_cache[key]

    def forward(self, tokens: torch.Tensor) -> torch.Tensor:
        """Returns logits [B*S, V] (bf16 when the weights are bf16)."""
        b, s = tokens.shape
        cos, sin = self.rope_tables(s, tokens.device)
        if self.param_waiter is not None:
            self.param_waiter([self.embed])
        x = ops.embedding(tokens, self.embed)
        delta = None
        for layer in self.layers:
            x, delta = layer(x, delta, cos, sin)
        if self.param_waiter is not None:
            self.param_waiter([self.norm, self.lm_head])
        _, h = ops.add_rms_norm(x, delta, self.norm, self.cfg.norm_eps)
        return ops.linear(h.reshape(b * s, -1), self.lm_head)

    def loss(self, tokens: torch.Tensor, targets: torch.Tensor) -> torch.Tensor:
        logits = self.forward(tokens)
        return ops.cross_entropy(logits, targets.reshape(-1))
