"""Autograd wrappers around the HIP kernels (``_C``) with CPU reference fallbacks."""

from __future__ import annotations

import os
import warnings

import torch

from dstack_amd.ops import _ext
from dstack_amd.ops import reference as ref


def _2d(t: torch.Tensor) -> torch.Tensor:
    return t.reshape(-1, t.shape[-1])


# ----------------------------------------------------------------------------------------------
# RMSNorm (+ fused residual add)
# ----------------------------------------------------------------------------------------------
class _RMSNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, eps):
        C = _ext.require()
        y, rstd = C.rms_norm_fwd(_2d(x), w, eps)
        ctx.save_for_backward(x, w, rstd)
        return y.view_as(x)

    @staticmethod
    def backward(ctx, dy):
        C = _ext.require()
        x, w, rstd = ctx.saved_tensors
        dy2 = _2d(dy.contiguous())
        writer = getattr(w, "_dsa_grad_writer", None)
        if writer is not None and w.dtype == torch.bfloat16:
            out = {}
            writer(w, lambda dst, acc: out.setdefault("dx", C.rms_norm_bwd(dy2, _2d(x), w, rstd, None, dst, acc)[0]))
            return out["dx"].view_as(x), None, None
        dx, dw = C.rms_norm_bwd(dy2, _2d(x), w, rstd, None)
        return dx.view_as(x), dw.to(w.dtype), None


class _AddRMSNorm(torch.autograd.Function):
    """h = x + delta ; y = rmsnorm(h) * w.  Returns (h, y); one HBM pass instead of two."""

    @staticmethod
    def forward(ctx, x, delta, w, eps):
        C = _ext.require()
        # an unused residual output (the final norm) gets dh=None, not a materialised zero tensor
        ctx.set_materialize_grads(False)
        h, y, rstd = C.add_rms_norm_fwd(_2d(x), _2d(delta), w, eps)
        ctx.save_for_backward(h, w, rstd)
        return h.view_as(x), y.view_as(x)

    @staticmethod
    def backward(ctx, dh, dy):
        C = _ext.require()
        h, w, rstd = ctx.saved_tensors
        if dh is not None:
            dh = _2d(dh.contiguous())
        dy2 = _2d(dy.contiguous())
        writer = getattr(w, "_dsa_grad_writer", None)
        if writer is not None and w.dtype == torch.bfloat16:
            # the weight gradient is written by the kernel into the optimizer's flat buffer
            out = {}
            writer(w, lambda dst, acc: out.setdefault("dx", C.rms_norm_bwd(dy2, h, w, rstd, dh, dst, acc)[0]))
            dx = out["dx"].view(dy.shape)
            return dx, dx, None, None
        dx, dw = C.rms_norm_bwd(dy2, h, w, rstd, dh)
        dx = dx.view(dy.shape)
        return dx, dx, dw.to(w.dtype), None


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float = 1e-5) -> torch.Tensor:
    if _ext.use_hip(x):
        return _RMSNorm.apply(x.contiguous(), w, eps)
    return ref.rms_norm(x, w, eps)


def add_rms_norm(x: torch.Tensor, delta: torch.Tensor, w: torch.Tensor, eps: float = 1e-5):
    if _ext.use_hip(x):
        return _AddRMSNorm.apply(x.contiguous(), delta.contiguous(), w, eps)
    return ref.add_rms_norm(x, delta, w, eps)


# ----------------------------------------------------------------------------------------------
# SwiGLU on the fused [gate | up] projection output
# ----------------------------------------------------------------------------------------------
class _SwiGLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gu, with_t):
        C = _ext.require()
        ctx.save_for_backward(gu)
        # aT is non-differentiable: without this autograd zero-fills a [F, T] gradient for it in
        # every backward (a 235 MB fill per layer and micro-batch of Llama-3-8B, r2g trace)
        ctx.set_materialize_grads(False)
        ctx.with_t = with_t
        if with_t:
            a, aT = C.swiglu_fwd_t(gu)
            ctx.mark_non_differentiable(aT)
            return a, aT
        return C.swiglu_fwd(gu), None

    @staticmethod
    def backward(ctx, da, _daT):
        C = _ext.require()
        (gu,) = ctx.saved_tensors
        if ctx.with_t and os.environ.get("DSTACK_AMD_SWIGLU_BWD_T", "1") != "0":
            # also write dgu^T: the gate/up weight gradient then takes token-contiguous operands
            dgu, dguT = C.swiglu_bwd_t(da.contiguous(), gu)
            dgu._dsa_t = dguT
            return dgu, None
        return C.swiglu_bwd(da.contiguous(), gu), None


def swiglu(gu: torch.Tensor) -> torch.Tensor:
    """silu(gate) * up of the fused [gate | up] projection.  On the HIP path with token-contiguous
    weight gradients (``DSTACK_AMD_WGRAD=transpose``) the kernel also writes the transposed output,
    attached as ``a._dsa_t`` [F, T]: ``linear`` then saves only that copy for the down projection's
    weight gradient (memory-neutral) and backward skips the transpose of ``a``."""
    if _ext.use_hip(gu):
        gu = gu.contiguous()
        T = gu.numel() // gu.shape[-1]
        F = gu.shape[-1] // 2
        with_t = _wgrad_mode() == "transpose" and T % 128 == 0 and F % 64 == 0
        a, aT = _SwiGLU.apply(gu, with_t)
        if aT is not None:
            a._dsa_t = aT
        return a
    return ref.swiglu(gu)


# ----------------------------------------------------------------------------------------------
# The SwiGLU MLP with both SwiGLU passes fused into the in-tree GEMM (csrc/gemm_nt.hip)
# ----------------------------------------------------------------------------------------------
class _SwiGLUMLP(torch.autograd.Function):
    """y = (silu(h Wg^T) * (h Wu^T)) Wdown^T with W_gu = [Wg; Wu].

    Forward: one gfx950 GEMM writes gu = h W_gu^T and, from the same tile, a = silu(g) * u and
    a^T (``gemm_nt_swiglu``: no separate SwiGLU pass re-reading gu); y = a Wdown^T (library GEMM).
    Backward: the down projection's input gradient da = dy Wdown is computed by the in-tree GEMM
    with the SwiGLU backward in its epilogue (``gemm_nt_swiglu_bwd``: dgu and dgu^T from the tile,
    da never reaches HBM); dx = dgu W_gu and the weight gradients (written into the optimizer's
    flat buffer through ``_dsa_grad_sink``) as in ``_Linear``."""

    @staticmethod
    def forward(ctx, h, wgu, wdown):
        C = _ext.require()
        h2 = _2d(h)
        # KM weight gradients take a and dgu token-major: no transposed copies from the epilogues
        ctx.km = _wgrad_mode() == "km"
        gu, a, aT = C.gemm_nt_swiglu(h2, wgu, not ctx.km)
        y = _nt(a, wdown)
        ctx.save_for_backward(h2, gu, a if ctx.km else aT, wgu, wdown)
        ctx.hshape = h.shape
        return y.view(*h.shape[:-1], wdown.shape[0])

    @staticmethod
    def backward(ctx, dy):
        C = _ext.require()
        h2, gu, a_or_aT, wgu, wdown = ctx.saved_tensors
        dy2 = _2d(dy.contiguous())
        # down projection weight gradient dW = dy^T a  (a^T already written by the forward)
        gwd = None
        if ctx.km:
            a_op, b_op = wgrad_operands(dy2, a_or_aT)
        else:
            a_op, b_op = wgrad_operands(dy2, None, xT=a_or_aT)
        sink = getattr(wdown, "_dsa_grad_sink", None)
        if sink is not None:
            sink(wdown, a_op, b_op)
        else:
            gwd = mm_into(a_op, b_op)
        # da = dy Wdown with the SwiGLU backward fused: dgu, dgu^T
        wdT = _transposed_weight(wdown)
        if wdT is None:
            wdT = wdown.t().contiguous()
        dgu, dguT = C.gemm_nt_swiglu_bwd(dy2, wdT, gu, not ctx.km)
        # dx = dgu W_gu
        wguT = _transposed_weight(wgu)
        dx = _nt(dgu, wguT) if wguT is not None else dgu @ wgu
        # gate/up weight gradient dW_gu = dgu^T h  (dgu^T from the fused epilogue)
        ggu = None
        a_op, b_op = wgrad_operands(dgu, h2, gT=None if ctx.km else dguT)
        sink = getattr(wgu, "_dsa_grad_sink", None)
        if sink is not None:
            sink(wgu, a_op, b_op)
        else:
            ggu = mm_into(a_op, b_op)
        return dx.view(ctx.hshape), ggu, gwd


def _mlp_fused_ok(h: torch.Tensor, wgu: torch.Tensor, wdown: torch.Tensor) -> bool:
    if os.environ.get("DSTACK_AMD_MLP_FUSED", "1") == "0" or _wgrad_mode() not in ("transpose", "km"):
        return False
    if h.dtype != torch.bfloat16 or wgu.dtype != torch.bfloat16 or wdown.dtype != torch.bfloat16:
        return False
    C = _ext.require()
    T, D = h.numel() // h.shape[-1], h.shape[-1]
    F = wgu.shape[0] // 2
    return (tuple(wgu.shape) == (2 * F, D) and tuple(wdown.shape) == (D, F) and wgu.is_contiguous()
            and wdown.is_contiguous() and C.gemm_nt_swiglu_supported(T, F, D)
            and C.gemm_nt_swiglu_bwd_supported(T, F, D))


def swiglu_mlp(h: torch.Tensor, wgu: torch.Tensor, wdown: torch.Tensor) -> torch.Tensor:
    """The Llama MLP: ``linear(swiglu(linear(h, wgu)), wdown)``.  On the HIP path both SwiGLU
    passes live in the epilogues of the in-tree GEMM (``_SwiGLUMLP``); ``DSTACK_AMD_MLP_FUSED=0``
    (or an untiled shape) keeps the separate kernels."""
    if _ext.use_hip(h) and _mlp_fused_ok(h, wgu, wdown):
        return _SwiGLUMLP.apply(h.contiguous(), wgu, wdown)
    return linear(swiglu(linear(h, wgu)), wdown)


# ----------------------------------------------------------------------------------------------
# RoPE applied to the q and k heads of a fused qkv activation [B, S, (H + 2*KV) * D]
# ----------------------------------------------------------------------------------------------
class _RopeQKV(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, cos, sin, n_rot_heads, head_dim):
        C = _ext.require()
        ctx.save_for_backward(cos, sin)
        ctx.meta = (n_rot_heads, head_dim)
        return C.rope_qkv(qkv, cos, sin, n_rot_heads, head_dim, False)

    @staticmethod
    def backward(ctx, dout):
        C = _ext.require()
        cos, sin = ctx.saved_tensors
        n_rot_heads, head_dim = ctx.meta
        return C.rope_qkv(dout.contiguous(), cos, sin, n_rot_heads, head_dim, True), None, None, None, None


def rope(qkv: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, n_rot_heads: int, head_dim: int):
    """Rotate the first ``n_rot_heads`` heads (q and k) of ``qkv`` [B, S, NH*D]; v passes through."""
    if _ext.use_hip(qkv):
        return _RopeQKV.apply(qkv.contiguous(), cos, sin, n_rot_heads, head_dim)
    b, s, _ = qkv.shape
    x = qkv.view(b, s, -1, head_dim)
    rot = ref.apply_rope(x[:, :, :n_rot_heads], cos, sin)
    return torch.cat([rot, x[:, :, n_rot_heads:]], dim=2).reshape(b, s, -1)


# ----------------------------------------------------------------------------------------------
# Token embedding whose backward scatter-sums straight into the optimizer's flat gradient buffer
# ----------------------------------------------------------------------------------------------
class _Embedding(torch.autograd.Function):
    @staticmethod
    def forward(ctx, tokens, w):
        ctx.save_for_backward(tokens, w)
        return torch.nn.functional.embedding(tokens, w)

    @staticmethod
    def backward(ctx, dy):
        C = _ext.require()
        tokens, w = ctx.saved_tensors
        dy2 = _2d(dy.contiguous())
        sorted_tok, order = torch.sort(tokens.reshape(-1), stable=True)
        writer = getattr(w, "_dsa_grad_writer", None)
        if writer is not None:
            writer(w, lambda dst, acc: C.embedding_bwd(dy2, sorted_tok, order, dst, acc))
            return None, None
        dw = torch.empty_like(w)
        C.embedding_bwd(dy2, sorted_tok, order, dw, False)
        return None, dw


def embedding(tokens: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """``w[tokens]``; the HIP backward sums repeated ids in fp32 in a fixed order (deterministic) and
    touches only the rows of the batch's ids (csrc/elementwise.hip ``embed_bwd_kernel``)."""
    if _ext.use_hip(w) and w.dtype == torch.bfloat16 and w.shape[1] % 8 == 0:
        return _Embedding.apply(tokens, w)
    return torch.nn.functional.embedding(tokens, w)


# ----------------------------------------------------------------------------------------------
# Attention (causal, GQA) straight from the fused qkv activation [B, S, (H + 2*KV) * D]
# ----------------------------------------------------------------------------------------------
class _FlashAttnQKV(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, n_heads, n_kv_heads, causal):
        C = _ext.require()
        o, lse = C.flash_attn_fwd(qkv, n_heads, n_kv_heads, causal)
        ctx.save_for_backward(qkv, o, lse)
        ctx.meta = (n_heads, n_kv_heads, causal)
        return o

    @staticmethod
    def backward(ctx, do):
        C = _ext.require()
        qkv, o, lse = ctx.saved_tensors
        n_heads, n_kv_heads, causal = ctx.meta
        dqkv = C.flash_attn_bwd(do.contiguous(), qkv, o, lse, n_heads, n_kv_heads, causal)
        return dqkv, None, None, None


class _QKVRopeAttn(torch.autograd.Function):
    """o = attention(rope(h Wqkv^T)) with both RoPE passes fused away: the forward rotates q and k
    in the in-tree qkv GEMM's epilogue (``gemm_nt_rope``, fp32 accumulators rotated before the one
    bf16 rounding), the backward hands the tables to the flash-attention backward, whose dQ epilogue
    and dK reduction write the gradient w.r.t. the unrotated projection.  No ``rope_qkv_kernel``
    pass (a full read + write of qkv) in either direction.  Weight and input gradients as in
    ``_Linear`` (the weight gradient through ``_dsa_grad_sink``)."""

    @staticmethod
    def forward(ctx, h, wqkv, cos, sin, n_heads, n_kv_heads):
        C = _ext.require()
        b, s, _ = h.shape
        h2 = _2d(h)
        qkv = C.gemm_nt_rope(h2, wqkv, cos, sin, s, (n_heads + n_kv_heads) * 128).view(b, s, -1)
        o, lse = C.flash_attn_fwd(qkv, n_heads, n_kv_heads, True)
        ctx.save_for_backward(h2, wqkv, qkv, o, lse, cos, sin)
        ctx.meta = (n_heads, n_kv_heads, h.shape)
        return o

    @staticmethod
    def backward(ctx, do):
        C = _ext.require()
        h2, wqkv, qkv, o, lse, cos, sin = ctx.saved_tensors
        n_heads, n_kv_heads, hshape = ctx.meta
        dqkv = C.flash_attn_bwd(do.contiguous(), qkv, o, lse, n_heads, n_kv_heads, True, cos, sin)
        g2 = dqkv.view(-1, dqkv.shape[-1])
        wt = _transposed_weight(wqkv)
        dh = _nt(g2, wt) if wt is not None else g2 @ wqkv
        a, b = wgrad_operands(g2, h2)
        sink = getattr(wqkv, "_dsa_grad_sink", None)
        gw = None
        if sink is None:
            gw = mm_into(a, b)
        else:
            sink(wqkv, a, b)
        return dh.view(hshape), gw, None, None, None, None


def _qkv_rope_ok(h: torch.Tensor, wqkv: torch.Tensor, cos: torch.Tensor, n_heads: int, n_kv_heads: int) -> bool:
    if os.environ.get("DSTACK_AMD_QKV_ROPE", "1") == "0" or _attn_impl() != "hip":
        return False
    if h.dtype != torch.bfloat16 or wqkv.dtype != torch.bfloat16 or not (h.is_contiguous() and wqkv.is_contiguous()):
        return False
    if h.dim() != 3 or wqkv.shape[0] != (n_heads + 2 * n_kv_heads) * 128 or cos.dtype != torch.float32:
        return False
    C = _ext.require()
    b, s, d = h.shape
    return s % 256 == 0 and C.gemm_nt_rope_supported(b * s, wqkv.shape[0], d, s, (n_heads + n_kv_heads) * 128)


def qkv_rope_attention(h: torch.Tensor, wqkv: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, n_heads: int,
                       n_kv_heads: int) -> torch.Tensor:
    """Causal GQA attention of the Llama block: ``attention(rope(linear(h, wqkv)))``, [B, S, H*D].
    On the HIP path with head_dim 128 and S % 256 == 0 the RoPE passes are fused into the qkv GEMM
    and the attention backward (``_QKVRopeAttn``; ``DSTACK_AMD_QKV_ROPE=0`` keeps the separate
    kernels)."""
    if _ext.use_hip(h) and _qkv_rope_ok(h, wqkv, cos, n_heads, n_kv_heads):
        return _QKVRopeAttn.apply(h, wqkv, cos.contiguous(), sin.contiguous(), n_heads, n_kv_heads)
    hd = wqkv.shape[0] // (n_heads + 2 * n_kv_heads)
    qkv = rope(linear(h, wqkv), cos, sin, n_heads + n_kv_heads, hd)
    return attention(qkv, n_heads, n_kv_heads, causal=True)


def _attn_impl() -> str:
    return os.environ.get("DSTACK_AMD_ATTN", "hip").lower()


def split_qkv(qkv: torch.Tensor, n_heads: int, n_kv_heads: int):
    b, s, _ = qkv.shape
    x = qkv.view(b, s, n_heads + 2 * n_kv_heads, -1)
    return x[:, :, :n_heads], x[:, :, n_heads : n_heads + n_kv_heads], x[:, :, n_heads + n_kv_heads :]


_ATTN_FALLBACK_WARNED: set = set()


def attention(qkv: torch.Tensor, n_heads: int, n_kv_heads: int, causal: bool = True) -> torch.Tensor:
    """Causal GQA attention on the fused projection output; returns [B, S, H*D]."""
    b, s, _ = qkv.shape
    if _ext.use_hip(qkv) and _attn_impl() == "hip":
        d = qkv.shape[-1] // (n_heads + 2 * n_kv_heads)
        if d == 128 and s % 128 == 0:
            return _FlashAttnQKV.apply(qkv.contiguous(), n_heads, n_kv_heads, causal)
        # the HIP kernels are tiled for head_dim 128 (Llama-3 8B/70B, Qwen2, Mistral); other shapes
        # (Llama-3.2 1B/3B: head_dim 64) run PyTorch's SDPA, said once per shape
        key = (d, s % 128 == 0)
        if key not in _ATTN_FALLBACK_WARNED:
            _ATTN_FALLBACK_WARNED.add(key)
            warnings.warn(f"HIP flash attention is tiled for head_dim 128 and seq_len % 128 == 0 (got head_dim {d}, "
                          f"seq_len {s}): using PyTorch SDPA for this shape", RuntimeWarning, stacklevel=2)
    q, k, v = split_qkv(qkv, n_heads, n_kv_heads)
    if q.is_cuda:
        # library attention (PyTorch-ROCm SDPA): shapes the HIP kernels do not tile, or the
        # DSTACK_AMD_ATTN=sdpa A/B baseline
        o = torch.nn.functional.scaled_dot_product_attention(
            q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), is_causal=causal, enable_gqa=True
        ).transpose(1, 2)
    else:
        o = ref.attention(q, k, v, causal)
    return o.reshape(b, s, -1)


# ----------------------------------------------------------------------------------------------
# Fused softmax cross-entropy over the vocab (never materialises fp32 logits)
# ----------------------------------------------------------------------------------------------
class _Linear(torch.autograd.Function):
    """``y = x @ w.T`` whose weight gradient is written by the GEMM itself into the optimizer's
    flat gradient buffer (``w._dsa_grad_sink``): the first micro-batch uses beta=0 (no memset of
    the buffer), later ones accumulate with beta=1 in the hipBLASLt epilogue — no separate
    AccumulateGrad add kernel, no zero-fill, one pass over the gradient instead of three.
    The dW GEMM's operands are re-laid out token-contiguous first (``wgrad_operands``); when the
    producer of ``x`` already wrote ``x^T`` (``x._dsa_t``, e.g. SwiGLU) only that copy is saved."""

    @staticmethod
    def forward(ctx, x, w):
        xT = getattr(x, "_dsa_t", None)
        ctx.x_is_t = xT is not None
        ctx.save_for_backward(xT if ctx.x_is_t else x, w)
        return _nt(x, w)

    @staticmethod
    def backward(ctx, g):
        xs, w = ctx.saved_tensors
        gx = None
        if ctx.needs_input_grad[0]:
            wt = _transposed_weight(w)
            gx = _nt(g, wt) if wt is not None else g @ w
        if not ctx.needs_input_grad[1]:
            return gx, None
        g2 = g.reshape(-1, g.shape[-1])
        gT = getattr(g, "_dsa_t", None)
        if ctx.x_is_t:
            a, b = wgrad_operands(g2, None, xT=xs, gT=gT)
        else:
            a, b = wgrad_operands(g2, xs.reshape(-1, xs.shape[-1]), gT=gT)
        sink = getattr(w, "_dsa_grad_sink", None)
        if sink is None:
            return gx, mm_into(a, b)
        sink(w, a, b)
        return gx, None


def _nt(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """``a @ b.t()`` for a [.., K] activation and a [N, K] weight.  ``DSTACK_AMD_LINEAR_NT=1`` runs it
    on the in-tree gfx950 GEMM (csrc/gemm_nt.hip) where the shape is tiled; otherwise (and by default:
    hipBLASLt measured at parity on these shapes) the library GEMM."""
    if (os.environ.get("DSTACK_AMD_LINEAR_NT") == "1" and _ext.use_hip(a) and a.dtype == torch.bfloat16
            and b.dtype == torch.bfloat16):
        a2 = a.reshape(-1, a.shape[-1])
        C = _ext.require()
        if (C.gemm_nt_supported(a2.shape[0], b.shape[0], a2.shape[1]) and a2.stride(1) == 1 and b.stride(1) == 1
                and a2.stride(0) % 8 == 0 and b.stride(0) % 8 == 0
                and a2.data_ptr() % 16 == 0 and b.data_ptr() % 16 == 0):
            out = torch.empty(a2.shape[0], b.shape[0], device=a.device, dtype=a.dtype)
            C.gemm_nt(a2, b, out, False)
            return out.view(*a.shape[:-1], b.shape[0])
    return a @ b.t()


def _transposed_weight(w: torch.Tensor):
    """W^T [K, N] of a weight W [N, K] whose optimizer publishes a weight generation
    (``w._dsa_wgen()``, bumped whenever the weights change: ZeroOptimizer.step / load_state).

    The input gradient g @ W reduces over N, which is W's strided dimension: hipBLASLt runs that
    "NN" GEMM at 1.22-1.40 PFLOP/s in the Llama-3-8B step, against 1.55-1.60 for the forward's
    layout, where the reduction dimension is contiguous in both operands.  g @ (W^T)^T is that
    layout.  The transpose is made once per weight generation, in the first micro-batch's
    backward (~225 us per layer, HIP transpose kernel) and reused by every later micro-batch;
    ``DSTACK_AMD_DGRAD_WT=0`` keeps the NN GEMM."""
    gen = getattr(w, "_dsa_wgen", None)
    if gen is None or w.dim() != 2 or not _ext.use_hip(w) or os.environ.get("DSTACK_AMD_DGRAD_WT", "1") == "0":
        return None
    C = _ext.require()
    if not (w.is_contiguous() and C.transpose2d_supported(w.shape[0], w.shape[1])):
        return None
    cur = gen()
    cached = getattr(w, "_dsa_wt", None)
    if cached is None or cached[0] != cur:
        w._dsa_wt = None  # drop the stale copy before allocating the new one
        w._dsa_wt = (cur, C.transpose2d(w.detach()))
    return w._dsa_wt[1]


def _wgrad_mode() -> str:
    """How weight gradients dW = g^T x get their operands: ``km`` (default: both operands left
    token-major, the in-tree GEMM's KM form, no transposes at all; +1.0 % tokens/s against
    ``transpose`` in a same-box A/B, profiles/wgrad_km_ab_r8a.txt), ``transpose`` (``auto``, the
    previous default: token-contiguous copies made by the HIP transpose kernel or written by the
    producer, hipBLASLt), ``strided`` (token-major, hipBLASLt)."""
    m = os.environ.get("DSTACK_AMD_WGRAD", "km").lower()
    return "transpose" if m == "auto" else m


def mm_into(a: torch.Tensor, b: torch.Tensor, out=None, accumulate: bool = False) -> torch.Tensor:
    """``out (+)= a @ b`` for a weight gradient's operands (``wgrad_operands``).  When ``a`` is the
    transposed view of a token-major [T, P] gradient and ``b`` a token-major [T, Q] input, the
    in-tree KM-form GEMM runs it (csrc/gemm_nt.hip, ``gemm_km``); other layouts go to the library."""
    if out is None:
        out = torch.empty(a.shape[0], b.shape[1], device=a.device, dtype=torch.result_type(a, b))
    if (a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16 and out.dtype == torch.bfloat16
            and _ext.use_hip(a) and a.stride(0) == 1 and b.stride(1) == 1 and out.stride(1) == 1
            and a.shape[1] == b.shape[0]):
        C = _ext.require()
        g = a.t()
        if (C.gemm_km_supported(a.shape[0], b.shape[1], a.shape[1]) and g.stride(0) % 8 == 0
                and b.stride(0) % 8 == 0 and out.stride(0) % 8 == 0
                and all(t.data_ptr() % 16 == 0 for t in (g, b, out))):
            C.gemm_km(g, b, out, 1 if accumulate else 0)
            return out
    if accumulate:
        return out.addmm_(a, b)
    return torch.mm(a, b, out=out)


def mm_into_f32(a: torch.Tensor, b: torch.Tensor, acc: torch.Tensor, out: torch.Tensor, mode: int) -> None:
    """Weight gradient ``a @ b`` with an fp32 accumulator ``acc``: mode 0 ``acc = a @ b``, 1
    ``acc += a @ b``, 2 ``out (bf16) = acc + a @ b`` (the last micro-batch: one rounding).  The
    in-tree KM GEMM does it in its epilogue (``gemm_km_f32``); other layouts/devices in fp32 torch."""
    if (a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16 and _ext.use_hip(a) and a.stride(0) == 1
            and b.stride(1) == 1 and acc.stride(1) == 1 and a.shape[1] == b.shape[0]):
        C = _ext.require()
        g = a.t()
        if (C.gemm_km_supported(a.shape[0], b.shape[1], a.shape[1]) and g.stride(0) % 8 == 0
                and b.stride(0) % 8 == 0 and acc.stride(0) % 4 == 0 and out.stride(0) % 8 == 0
                and all(t.data_ptr() % 16 == 0 for t in (g, b, acc, out))):
            C.gemm_km_f32(g, b, acc, out if mode == 2 else None, mode)
            return
    prod = torch.mm(a.float(), b.float())
    if mode == 0:
        acc.copy_(prod)
    elif mode == 1:
        acc.add_(prod)
    else:
        out.copy_(acc + prod)


def wgrad_operands(g2: torch.Tensor, x2, xT=None, gT=None):
    """Operands (a [P, T], b [T, Q]) with dW = a @ b for g2 [T, P] and x2 [T, Q] (or its transpose
    ``xT`` [Q, T] when the producer already wrote it; likewise ``gT`` [P, T] for g2).

    hipBLASLt runs dW = g^T x at ~1.0-1.1 PFLOP/s on MI355X when both operands are token-major
    (the reduction dimension is the strided one for both) and at 1.3-1.56 PFLOP/s when they are
    token-contiguous (tools/bench_wgrad_layouts.py, profiles/wgrad_layouts_r1.txt).  So x is
    transposed by the HIP transpose kernel (T x Q, a few % of the GEMM's time) and g too when it
    is no larger than x (down/o projections).  A larger g (the gate_up gradient, 3.5x its input)
    is used transposed only when its producer already wrote g^T (``gT``: SwiGLU backward);
    the lm_head gradient (31x) stays token-major.  ``DSTACK_AMD_WGRAD=strided`` keeps the old
    layout."""
    T, P = g2.shape
    Q = xT.shape[0] if xT is not None else x2.shape[1]
    a = g2.t()
    b = xT.t() if xT is not None else x2
    if not (_ext.use_hip(g2) and _wgrad_mode() == "transpose"):
        return a, b  # "km" (mm_into's in-tree KM GEMM) and "strided" take the token-major views
    C = _ext.require()
    if xT is None and x2.is_contiguous() and C.transpose2d_supported(T, Q):
        b = C.transpose2d(x2).t()
    if gT is not None and tuple(gT.shape) == (P, T):
        a = gT
    elif P <= Q and g2.is_contiguous() and C.transpose2d_supported(T, P):
        a = C.transpose2d(g2)
    return a, b


def linear(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    return _Linear.apply(x, w)


def weight_grad(g: torch.Tensor, x: torch.Tensor, out: torch.Tensor, accumulate: bool = False) -> torch.Tensor:
    """``out (+)= g^T x`` for g [T, P], x [T, Q] (dW of a linear layer) with the HIP gemm_tn kernel
    (csrc/gemm.hip) when the shape is tiled by it, else torch.  At parity with hipBLASLt on the
    Llama shapes (profiles/gemm_wgrad_r1.txt), so the training path keeps the library GEMM."""
    if _ext.use_hip(g):
        C = _ext.require()
        if C.gemm_tn_supported(g.shape[1], x.shape[1], g.shape[0]) and g.stride(1) == 1 and x.stride(1) == 1:
            C.gemm_tn(g, x, out, accumulate)
            return out
    if accumulate:
        return out.addmm_(g.t(), x)
    return torch.mm(g.t(), x, out=out)


class _CrossEntropy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target):
        C = _ext.require()
        loss_rows, lse = C.cross_entropy_fwd(logits, target)
        ctx.save_for_backward(logits, target, lse)
        return loss_rows.mean()

    @staticmethod
    def backward(ctx, dloss):
        C = _ext.require()
        logits, target, lse = ctx.saved_tensors
        scale = dloss / logits.shape[0]
        # gradient is written in place over the logits buffer (logits are dead after this)
        dlogits = C.cross_entropy_bwd(logits, target, lse, scale.float().reshape(1), True)
        return dlogits, None


def cross_entropy(logits: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """Mean token cross-entropy; ``logits`` [T, V] bf16, ``target`` [T] int64."""
    if _ext.use_hip(logits):
        return _CrossEntropy.apply(logits.contiguous(), target.contiguous())
    return ref.cross_entropy(logits, target)


# ----------------------------------------------------------------------------------------------
# Fused AdamW over flat buffers (bf16 param/grad, fp32 master/m/v)
# ----------------------------------------------------------------------------------------------
def adamw_(param, grad, master, m, v, *, lr, beta1, beta2, eps, weight_decay, step, grad_scale=1.0,
           max_blocks=0):
    """``max_blocks`` > 0 caps the HIP kernel's (grid-stride) grid, e.g. to leave most CUs to the
    compute stream when the update runs beside backward."""
    if _ext.use_hip(param):
        C = _ext.require()
        bc1 = 1.0 - beta1**step
        bc2 = 1.0 - beta2**step
        C.adamw(param, grad, master, m, v, lr, beta1, beta2, eps, weight_decay, bc1, bc2, grad_scale, max_blocks)
        return
    ref.adamw_(param, grad, master, m, v, lr, beta1, beta2, eps, weight_decay, step, grad_scale)
