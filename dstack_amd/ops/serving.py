"""Serving ops: paged KV cache writes, paged decode attention and sampling.

HIP kernels in ``csrc/paged_attn.hip`` for ROCm tensors; the PyTorch functions here are the CPU
path of the engine and the fp32 references the GPU tests compare against.

Cache layout (per layer): ``k_cache [pages, KVH, PAGE, 128]`` token-major and
``v_cache [pages, KVH, 128, PAGE]`` dim-major (see the kernel file for why), ``PAGE = 64``.
A token's cache slot is ``page * PAGE + offset``.
"""

from __future__ import annotations

import math

import torch

from dstack_amd.ops import _ext

PAGE = 64
HEAD_DIM = 128


def alloc_cache(num_pages: int, n_kv_heads: int, dtype=torch.bfloat16, device=None):
    """``dtype`` bf16 (or fp32 on the CPU) or ``torch.float8_e4m3fn`` (an fp8 cache holds
    k / k_scale and v / v_scale: half the bytes a decode step streams, twice the tokens)."""
    k = torch.zeros(num_pages, n_kv_heads, PAGE, HEAD_DIM, dtype=dtype, device=device)
    v = torch.zeros(num_pages, n_kv_heads, HEAD_DIM, PAGE, dtype=dtype, device=device)
    return k, v


def _is_fp8(cache: torch.Tensor) -> bool:
    return cache.dtype == torch.float8_e4m3fn


# ----------------------------------------------------------------------------------------------
# RoPE + cache write
# ----------------------------------------------------------------------------------------------
def rope_cache_write(qkv: torch.Tensor, positions: torch.Tensor, slots: torch.Tensor, cos: torch.Tensor,
                     sin: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, n_heads: int,
                     n_kv_heads: int, k_scale: float = 1.0, v_scale: float = 1.0, rs=None, cs=None) -> torch.Tensor:
    """Rotate q and k of ``qkv`` [T, (H + 2*KVH) * 128] in place (token t at ``positions[t]``) and
    store k/v of every token with ``slots[t] >= 0`` in the cache.  Returns ``qkv``.

    ``rs`` [T] / ``cs`` [(H + 2*KVH) * 128]: ``qkv`` is the raw product of a tensor-wise-scaled fp8
    GEMM; its row-wise scales are applied first, in place for every head."""
    if _ext.use_hip(qkv):
        _ext.require().rope_cache_write(qkv, positions, slots, cos, sin, k_cache, v_cache, n_heads, n_kv_heads,
                                        k_scale, v_scale, rs, cs)
        return qkv
    if rs is not None:
        qkv.copy_((qkv.float() * rs[:, None] * cs[None, :]).to(qkv.dtype))
    return rope_cache_write_ref(qkv, positions, slots, cos, sin, k_cache, v_cache, n_heads, n_kv_heads,
                                k_scale, v_scale)


def rope_cache_write_ref(qkv, positions, slots, cos, sin, k_cache, v_cache, n_heads, n_kv_heads,
                         k_scale: float = 1.0, v_scale: float = 1.0):
    T = positions.numel()
    x = qkv.view(T, n_heads + 2 * n_kv_heads, HEAD_DIM)
    rot = x[:, : n_heads + n_kv_heads].float()
    c = cos[positions.long()].unsqueeze(1)
    s = sin[positions.long()].unsqueeze(1)
    x1, x2 = rot[..., : HEAD_DIM // 2], rot[..., HEAD_DIM // 2 :]
    x[:, : n_heads + n_kv_heads] = torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1).to(qkv.dtype)
    keep = slots >= 0
    if keep.any():
        sl = slots[keep].long()
        page, off = sl // PAGE, sl % PAGE
        k = x[keep][:, n_heads : n_heads + n_kv_heads]  # [n, KVH, D]
        v = x[keep][:, n_heads + n_kv_heads :]
        if _is_fp8(k_cache):
            k = (k.float() / k_scale).clamp(-448, 448)
            v = (v.float() / v_scale).clamp(-448, 448)
        k_cache[page, :, off, :] = k.to(k_cache.dtype)
        v_cache[page, :, :, off] = v.to(v_cache.dtype)
    return qkv


# ----------------------------------------------------------------------------------------------
# Paged decode attention
# ----------------------------------------------------------------------------------------------
def split_plan(batch: int, n_kv_heads: int, table_width: int, target_waves: int = 2048):
    """(nsplit, pages_per_split): enough one-wave workgroups to fill 256 CUs at any context, a
    function of the batch bucket and the block-table width only (graph-capturable)."""
    want = max(1, math.ceil(target_waves / max(1, batch * n_kv_heads)))
    nsplit = max(1, min(want, table_width))
    pps = math.ceil(table_width / nsplit)
    return math.ceil(table_width / pps), pps


class DecodeWorkspace:
    """Preallocated split-KV partials for a batch bucket (hipGraph-safe: no allocation per step)."""

    def __init__(self, batch: int, n_heads: int, n_kv_heads: int, table_width: int, device,
                 target_waves: int = 2048):
        self.nsplit, self.pps = split_plan(batch, n_kv_heads, table_width, target_waves)
        n = batch * n_heads * self.nsplit if self.nsplit > 1 else 1
        self.o_part = torch.empty(n * HEAD_DIM, dtype=torch.float32, device=device)
        self.lse_part = torch.empty(n, dtype=torch.float32, device=device)


def paged_decode(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, block_tables: torch.Tensor,
                 ctx_lens: torch.Tensor, n_heads: int, n_kv_heads: int, out: torch.Tensor | None = None,
                 ws: DecodeWorkspace | None = None, k_scale: float = 1.0, v_scale: float = 1.0) -> torch.Tensor:
    """Attention of one new query token per sequence over its cached keys/values.

    ``q`` [B, >= H*128] (rows may be the fused qkv output: only the first H*128 columns are read),
    ``block_tables`` [B, W] int32 page ids, ``ctx_lens`` [B] int32.  Returns [B, H*128]."""
    B = q.shape[0]
    if out is None:
        out = torch.empty(B, n_heads * HEAD_DIM, dtype=q.dtype, device=q.device)
    if _ext.use_hip(q):
        if ws is None:
            ws = DecodeWorkspace(B, n_heads, n_kv_heads, block_tables.shape[1], q.device)
        _ext.require().paged_decode(q, k_cache, v_cache, block_tables, ctx_lens, out, ws.o_part, ws.lse_part,
                                    n_heads, n_kv_heads, ws.nsplit, ws.pps, 1.0 / math.sqrt(HEAD_DIM), k_scale,
                                    v_scale)
        return out
    out.copy_(paged_decode_ref(q, k_cache, v_cache, block_tables, ctx_lens, n_heads, n_kv_heads, k_scale,
                               v_scale).to(out.dtype))
    return out


def paged_decode_ref(q, k_cache, v_cache, block_tables, ctx_lens, n_heads, n_kv_heads, k_scale: float = 1.0,
                     v_scale: float = 1.0):
    """fp32 reference: gathers each sequence's pages and runs plain softmax attention."""
    B = q.shape[0]
    G = n_heads // n_kv_heads
    out = torch.empty(B, n_heads * HEAD_DIM, dtype=torch.float32, device=q.device)
    for b in range(B):
        n = int(ctx_lens[b])
        pages = block_tables[b, : (n + PAGE - 1) // PAGE].long()
        ks, vs = (k_scale, v_scale) if _is_fp8(k_cache) else (1.0, 1.0)
        k = k_cache[pages].float().permute(1, 0, 2, 3).reshape(n_kv_heads, -1, HEAD_DIM)[:, :n] * ks  # [KVH, n, D]
        v = v_cache[pages].float().permute(1, 0, 3, 2).reshape(n_kv_heads, -1, HEAD_DIM)[:, :n] * vs
        qb = q[b, : n_heads * HEAD_DIM].float().view(n_kv_heads, G, HEAD_DIM)
        s = torch.einsum("hgd,hnd->hgn", qb, k) / math.sqrt(HEAD_DIM)
        p = torch.softmax(s, dim=-1)
        out[b] = torch.einsum("hgn,hnd->hgd", p, v).reshape(-1)
    return out


# ----------------------------------------------------------------------------------------------
# Sampling
# ----------------------------------------------------------------------------------------------
def sample(logits: torch.Tensor, temps: torch.Tensor, seeds: torch.Tensor, steps: torch.Tensor,
           tokens: torch.Tensor | None = None, logprobs: torch.Tensor | None = None):
    """Per row: greedy argmax when ``temps[r] <= 0``, else an exact draw from softmax(logits/T)
    (Gumbel-max with a counter-based hash of (seed, step, token)).  Returns (tokens int32,
    logprobs fp32: log-probability of the chosen token under softmax(logits / T))."""
    R = logits.shape[0]
    if tokens is None:
        tokens = torch.empty(R, dtype=torch.int32, device=logits.device)
    if logprobs is None:
        logprobs = torch.empty(R, dtype=torch.float32, device=logits.device)
    if _ext.use_hip(logits):
        _ext.require().sample(logits, temps, seeds, steps, tokens, logprobs)
        return tokens, logprobs
    t, lp = sample_ref(logits, temps, seeds, steps)
    tokens.copy_(t)
    logprobs.copy_(lp)
    return tokens, logprobs


def sample_ref(logits, temps, seeds, steps):
    x = logits.float()
    t = temps.float().clamp_min(0)
    scale = torch.where(t > 0, 1.0 / torch.where(t > 0, t, torch.ones_like(t)), torch.ones_like(t))
    z = x * scale[:, None]
    lse = torch.logsumexp(z, dim=-1)
    score = z.clone()
    for r in range(x.shape[0]):
        if t[r] > 0:
            g = torch.Generator(device="cpu").manual_seed(int(seeds[r]) * 1000003 + int(steps[r]))
            u = torch.rand(x.shape[1], generator=g).clamp(1e-7, 1 - 1e-7).to(x.device)
            score[r] = z[r] - torch.log(-torch.log(u))
    tok = score.argmax(dim=-1)
    lp = z.gather(1, tok[:, None]).squeeze(1) - lse
    return tok.to(torch.int32), lp


# ----------------------------------------------------------------------------------------------
# Decode-GEMM weight layout
# ----------------------------------------------------------------------------------------------
def fp8_stream_shuffle(wq: torch.Tensor, group: int = 16) -> torch.Tensor:
    """The weight layout of ``fp8_stream_gemm(..., shuffled=1 | 2)`` (``csrc/fp8_gemm.hip``): for each
    block of 16 weight rows and each 128-byte K-step, the 2 KiB that one MFMA fragment of a wave
    reads, in lane order -- half h (16 bytes of 32) of lane ``r + 16 g`` (row r, bytes 32 g .. 32 g + 32)
    at ``h * 1024 + lane * 16``.  Every weight load of the kernel is then 1 KiB contiguous.
    ``group`` 16 (shuffled=1): a block's pieces run consecutively over K; the workgroup's rows
    (shuffled=2: 256, or 224 for the 7-wave form): per K-step the blocks of one workgroup sit side
    by side (group x 128 bytes contiguous per workgroup and step).  ``wq`` [N][K] 1-byte, N % group == 0, K % 128 == 0; returns a contiguous
    [N][K] tensor of the same dtype (done once, when the weights are loaded)."""
    N, K = wq.shape
    assert group % 16 == 0 and N % group == 0 and K % 128 == 0 and wq.element_size() == 1, (
        tuple(wq.shape), wq.dtype, group)
    nb = group // 16
    b = wq.view(torch.uint8).reshape(N // group, nb, 16, K // 128, 4, 2, 16)  # (grp, blk, r, t, g, h, byte)
    return b.permute(0, 3, 1, 5, 4, 2, 6).contiguous().view(N, K).view(wq.dtype)


def fp8_stream_unshuffle(ws: torch.Tensor, group: int = 16) -> torch.Tensor:
    """Inverse of :func:`fp8_stream_shuffle` (tests)."""
    N, K = ws.shape
    nb = group // 16
    b = ws.view(torch.uint8).reshape(N // group, K // 128, nb, 2, 4, 16, 16)  # (grp, t, blk, h, g, r, byte)
    return b.permute(0, 2, 5, 1, 4, 3, 6).contiguous().view(N, K).view(ws.dtype)


def _f8_swz(r: torch.Tensor) -> torch.Tensor:
    """The 16-byte-chunk XOR swizzle of the fp8 GEMMs' LDS tiles (csrc/fp8_gemm.hip f8_swz)."""
    return ((r >> 1) & 1) | (((r >> 3) & 1) << 2)


def fp8_rows_shuffle(wq: torch.Tensor) -> torch.Tensor:
    """The weight layout of ``fp8_rows_gemm(..., wimg=True)``: per 128-row tile and 128-byte K-step
    the 16 KiB image the kernel's LDS holds -- row r's 16-byte chunk c at ``r * 128 + c * 16`` is the
    row's chunk ``c ^ f8_swz(r % 16)`` -- so every weight DMA of the kernel reads 1 KiB contiguous and
    a tile's stream is sequential over K.  ``wq`` [N][K] 1-byte, N % 128 == 0, K % 128 == 0; returns a
    contiguous [N][K] tensor of the same dtype."""
    N, K = wq.shape
    assert N % 128 == 0 and K % 128 == 0 and wq.element_size() == 1, (tuple(wq.shape), wq.dtype)
    b = wq.view(torch.uint8).reshape(N // 128, 128, K // 128, 8, 16).permute(0, 2, 1, 3, 4)  # (nb, t, r, c, byte)
    r = torch.arange(128, device=wq.device)
    src = torch.arange(8, device=wq.device)[None, :] ^ _f8_swz(r % 16)[:, None]  # [r, c] -> source chunk
    idx = src.view(1, 1, 128, 8, 1).expand(N // 128, K // 128, 128, 8, 16)
    return torch.gather(b, 3, idx).contiguous().view(N, K).view(wq.dtype)
