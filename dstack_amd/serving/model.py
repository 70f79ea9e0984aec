"""Llama-family inference model for the serving engine: paged KV cache, prefill + decode.

MI355X-first layout (contrast: the reference runs vLLM/TGI containers for services,
``examples/deployment/vllm/.dstack.yml``):

* one GPU holds the whole model whenever it fits — Llama-3-70B bf16 is 141 GB of the 288 GB HBM3E,
  leaving ~110 GB of KV cache (≈340k tokens) — so a replica is one process on one GPU (no tensor
  parallel all-reduces on the decode path); services scale by replicas;
* fused projections (``wqkv``, ``wgu``) as in the training model, so a decode step is 4 GEMMs per
  layer (hipBLASLt; skinny M = batch) plus HIP kernels for everything else: fused add+RMSNorm,
  RoPE fused with the paged-cache scatter, MFMA paged decode attention reading q straight from the
  qkv projection output, SwiGLU, and a fused sampler;
* prefill runs the training flash-attention forward kernel on each prompt (padded to 128 rows;
  causal masking makes the padding inert) and computes the LM head only for the last token;
* ``decode`` takes only static-shape tensors, so the engine captures it in one hipGraph per batch
  bucket (launch-bound small batches);
* models that do not fit one GPU (Llama-3.1-405B: 810 GB bf16 = 102 GB per GPU at TP 8) run
  tensor-parallel over RCCL/xGMI (``tp_group``): attention heads (q and kv), the FFN and the vocab
  are sharded Megatron-style, so a layer costs two all-reduces of [tokens, dim] (after ``wo`` and
  ``wdown``) and the logits one all-gather; each rank holds the KV cache of its own KV heads.
"""

from __future__ import annotations

import json
import logging
import math
import os
import zlib
from dataclasses import dataclass

import torch
import torch.distributed as dist
import torch.nn.functional as F

from dstack_amd.models.llama import CONFIGS, LlamaConfig
from dstack_amd.ops import _ext
from dstack_amd.ops import reference as ref
from dstack_amd.ops import serving as sops

logger = logging.getLogger(__name__)


class Fp8Weight:
    """A linear weight stored as e4m3 bytes ``q`` [N, K] (uint8 storage, float8_e4m3fn values) with
    one fp32 scale per output row ``s`` [N]: W ~= q * s[:, None].  ``qs``: the same bytes in the
    weight-streaming decode GEMM's layout (``ops.serving.fp8_stream_shuffle``), or None."""

    __slots__ = ("q", "s", "qs")

    def __init__(self, q: torch.Tensor, s: torch.Tensor, qs: torch.Tensor | None = None):
        self.q, self.s, self.qs = q, s, qs

    @property
    def shape(self):
        return self.q.shape

    def nbytes(self) -> int:
        return self.q.numel() + self.s.numel() * 4 + (self.qs.numel() if self.qs is not None else 0)


class Fp8Act:
    """Activations already in e4m3 with per-row scales (``q`` uint8 [M, K], ``s`` fp32 [M]),
    produced by the fused add+RMSNorm->fp8 kernel for the next fp8 GEMM."""

    __slots__ = ("q", "s")

    def __init__(self, q: torch.Tensor, s: torch.Tensor):
        self.q, self.s = q, s


class RawScaled:
    """The raw product of a tensor-wise-scaled fp8 GEMM (``raw`` bf16 [M, N]) still owing its
    row-wise scales: per-token ``rs`` [M] and per-output-channel ``cs`` [N].  The consumer applies
    them (the fused add + RMSNorm -> e4m3 kernel, or ``materialize``)."""

    __slots__ = ("raw", "rs", "cs")

    def __init__(self, raw: torch.Tensor, rs: torch.Tensor, cs: torch.Tensor):
        self.raw, self.rs, self.cs = raw, rs, cs

    @property
    def shape(self):
        return self.raw.shape

    def rows(self, idx: torch.Tensor) -> "RawScaled":
        return RawScaled(self.raw[idx], self.rs[idx].contiguous(), self.cs)

    def materialize(self) -> torch.Tensor:
        return _ext.require().scale_rows_cols_(self.raw, self.rs, self.cs)


@dataclass
class RopeScaling:
    """Llama-3.1 "llama3" RoPE frequency scaling (HF ``rope_scaling``)."""

    factor: float = 8.0
    low_freq_factor: float = 1.0
    high_freq_factor: float = 4.0
    original_max_position_embeddings: int = 8192


def rope_tables(max_pos: int, head_dim: int, theta: float, scaling: RopeScaling | None, device):
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    if scaling is not None:
        low_wl = scaling.original_max_position_embeddings / scaling.low_freq_factor
        high_wl = scaling.original_max_position_embeddings / scaling.high_freq_factor
        wl = 2 * math.pi / inv
        smooth = (scaling.original_max_position_embeddings / wl - scaling.low_freq_factor) / (
            scaling.high_freq_factor - scaling.low_freq_factor)
        scaled = torch.where(wl > low_wl, inv / scaling.factor, inv)
        mid = (wl <= low_wl) & (wl >= high_wl)
        inv = torch.where(mid, (1 - smooth) * inv / scaling.factor + smooth * inv, scaled)
    ang = torch.outer(torch.arange(max_pos, dtype=torch.float64), inv)
    return ang.cos().float().contiguous().to(device), ang.sin().float().contiguous().to(device)


@dataclass
class ModelSpec:
    cfg: LlamaConfig
    rope_scaling: RopeScaling | None = None
    tie_embeddings: bool = False
    bos_token_id: int | None = None
    eos_token_ids: tuple = ()
    path: str | None = None  # HF checkpoint directory (None: random init)
    family: str = "llama"  # llama | mistral | qwen2 (same block; qwen2 adds q/k/v biases)
    qkv_bias: bool = False


def load_spec(model: str) -> ModelSpec:
    """``model`` is a built-in config name (``llama-3-8b``, ``llama-3-70b``, …: random weights) or an
    HF checkpoint directory (``config.json`` + ``*.safetensors``) of the Llama block family: Llama
    2/3/3.x, Mistral (sliding-window models are served up to their window) and Qwen2 / Qwen2.5
    (q/k/v projection biases)."""
    if model in CONFIGS:
        return ModelSpec(CONFIGS[model], eos_token_ids=())
    cfg_path = os.path.join(model, "config.json")
    if not os.path.exists(cfg_path):
        raise ValueError(f"unknown model {model!r}: neither a built-in config ({', '.join(CONFIGS)}) "
                         "nor a directory with config.json")
    with open(cfg_path) as f:
        hf = json.load(f)
    arch = (hf.get("architectures") or ["LlamaForCausalLM"])[0]
    family = hf.get("model_type", "llama")
    if family not in SUPPORTED_FAMILIES:
        raise ValueError(f"unsupported architecture {arch} (Llama family only: {', '.join(SUPPORTED_FAMILIES)})")
    heads = hf["num_attention_heads"]
    dim = hf["hidden_size"]
    head_dim = hf.get("head_dim") or dim // heads
    if head_dim != 128 or dim != heads * head_dim:
        raise ValueError(f"head_dim must be 128 with hidden_size = heads * head_dim (got {head_dim})")
    # rope: ``rope_theta`` + ``rope_scaling`` (transformers 4.x) or ``rope_parameters`` (5.x)
    rp = hf.get("rope_parameters") or {}
    theta = hf.get("rope_theta", rp.get("rope_theta", 10000.0))
    max_len = int(hf.get("max_position_embeddings", 8192))
    # sliding-window attention (Mistral v0.1, Qwen2 with use_sliding_window): up to the window it is
    # full causal attention, so such a model is served with max_model_len <= window
    window = hf.get("sliding_window")
    if window and (family == "mistral" or hf.get("use_sliding_window")):
        max_len = min(max_len, int(window))
    if hf.get("hidden_act", "silu") != "silu":
        raise ValueError(f"unsupported activation {hf.get('hidden_act')} (SwiGLU / silu only)")
    cfg = LlamaConfig(
        name=os.path.basename(os.path.normpath(model)), dim=dim, n_layers=hf["num_hidden_layers"], n_heads=heads,
        n_kv_heads=hf.get("num_key_value_heads", heads), ffn_dim=hf["intermediate_size"],
        vocab_size=hf["vocab_size"], rope_theta=float(theta),
        norm_eps=float(hf.get("rms_norm_eps", 1e-5)), max_seq_len=max_len,
    )
    rs = hf.get("rope_scaling") or (rp if rp.get("rope_type", "default") != "default" else None)
    scaling = None
    if rs and (rs.get("rope_type") or rs.get("type")) == "default":
        rs = None
    if rs and (rs.get("rope_type") or rs.get("type")) == "llama3":
        scaling = RopeScaling(float(rs["factor"]), float(rs.get("low_freq_factor", 1.0)),
                              float(rs.get("high_freq_factor", 4.0)),
                              int(rs.get("original_max_position_embeddings", 8192)))
    elif rs:
        raise ValueError(f"unsupported rope_scaling {rs}")
    eos = hf.get("eos_token_id")
    eos_ids = tuple(eos) if isinstance(eos, list) else ((eos,) if eos is not None else ())
    return ModelSpec(cfg, scaling, bool(hf.get("tie_word_embeddings", False)), hf.get("bos_token_id"), eos_ids,
                     path=model, family=family, qkv_bias=family == "qwen2")


SUPPORTED_FAMILIES = ("llama", "mistral", "qwen2")


class ServingLlama:
    """Weights + paged KV cache of one Llama model on one device (or of one tensor-parallel shard:
    ``H``/``KVH``/``F``/``V`` below are then this rank's local head / FFN / vocab counts)."""

    def __init__(self, spec: ModelSpec, device, dtype=None, max_model_len: int | None = None, tp_group=None,
                 quantization: str | None = None, kv_cache_dtype: str = "auto"):
        if quantization not in (None, "fp8"):
            raise ValueError(f"unsupported quantization {quantization!r} (supported: fp8)")
        if kv_cache_dtype not in ("auto", "fp8"):
            raise ValueError(f"unsupported kv_cache_dtype {kv_cache_dtype!r} (supported: auto, fp8)")
        self.quantization = quantization
        self.kv_cache_dtype = kv_cache_dtype
        # fp8 cache: e4m3 bytes of k / k_scale, v / v_scale (1.0: K and V of Llama layers stay far
        # inside e4m3's +-448 range)
        self.k_scale = self.v_scale = 1.0
        self.spec = spec
        self.cfg = cfg = spec.cfg
        self.device = torch.device(device)
        self.dtype = dtype or (torch.bfloat16 if self.device.type == "cuda" else torch.float32)
        if cfg.head_dim != sops.HEAD_DIM:
            raise ValueError("serving kernels need head_dim 128")
        self.max_model_len = max_model_len or cfg.max_seq_len
        self.tp_group = tp_group
        self.tp = dist.get_world_size(tp_group) if tp_group is not None else 1
        self.tp_rank = dist.get_rank(tp_group) if tp_group is not None else 0
        tp = self.tp
        if cfg.n_heads % tp or cfg.n_kv_heads % tp or cfg.ffn_dim % tp or cfg.vocab_size % tp:
            raise ValueError(f"tensor parallel {tp} must divide heads {cfg.n_heads}, kv heads {cfg.n_kv_heads}, "
                             f"ffn {cfg.ffn_dim} and vocab {cfg.vocab_size}")
        self.H, self.KVH, self.D = cfg.n_heads // tp, cfg.n_kv_heads // tp, cfg.head_dim
        self.F, self.V = cfg.ffn_dim // tp, cfg.vocab_size // tp
        self.NH = self.H + 2 * self.KVH
        self.hip = self.device.type == "cuda" and not _ext.force_torch()
        if self.hip:
            _ext.require()
        # DSTACK_AMD_GEMV=0: small decode batches on hipBLASLt too (A/B switch)
        self.gemv = os.environ.get("DSTACK_AMD_GEMV", "1") != "0"
        # decode-batch fp8 projections (5..256 rows) on the in-tree fp8 GEMM (csrc/fp8_gemm.hip)
        # instead of hipBLASLt; "lib" keeps hipBLASLt
        self.fp8_gemm = os.environ.get("DSTACK_AMD_FP8_GEMM", "hip").lower()
        # DSTACK_AMD_FP8_SWIGLU_GEMM=1: fp8 gate/up for batches of a multiple of 256 rows on the
        # in-tree 256x256 GEMM with the SwiGLU and the row-wise scales in its epilogue
        # (csrc/gemm_nt.hip EPI_SWIGLU_F8) and a one-pass row quantizer after it -- bit-identical
        # output, but 0.99x (16384 rows) / 0.95x (256 rows) the hipBLASLt + SwiGLU-quant pair
        # (profiles/fp8_swiglu_gemm_r7c.txt), so off by default
        self.fp8_swiglu_gemm = os.environ.get("DSTACK_AMD_FP8_SWIGLU_GEMM", "0") == "1"
        # fp8: norms feeding an fp8 GEMM write e4m3 directly (DSTACK_AMD_FP8_FUSE_NORM=0: separate quant)
        self.fuse_norm_quant = os.environ.get("DSTACK_AMD_FP8_FUSE_NORM", "1") != "0"
        # decode batches of 129..256 rows multiply the largest fp8 weights
        # (gate/up N >= 32768, down K >= 16384: the Llama-3-70B MLP on one GPU) on the weight-streaming
        # GEMM (csrc/fp8_gemm.hip fp8_stream_gemm) from a pre-shuffled second copy of those weights
        # (+0.7 GB per 70B layer): decode 6.86-6.88k -> 7.17-7.21k tok/s on the 70B fp8 bench, same box
        # (profiles/fp8_stream_shuffle_r9u.txt).  DSTACK_AMD_FP8_STREAM=0: hipBLASLt, no second copy
        self.fp8_stream = os.environ.get("DSTACK_AMD_FP8_STREAM", "1") != "0"
        self.fp8_stream_layout = int(os.environ.get("DSTACK_AMD_FP8_STREAM_LAYOUT", "2"))  # 1 | 2 (fp8_stream_shuffle)
        # fp8 GEMMs of at least this many rows (prefill) run hipBLASLt with scalar scales on the raw
        # e4m3 operands and apply the row-wise scales afterwards: in the gate/up output's SwiGLU-quant
        # kernel, or in one in-place pass for o / down (profiles/fp8_scaling_modes_r8z.txt: 12-25 %
        # faster GEMMs).  DSTACK_AMD_FP8_DEFER_SCALE=0 keeps hipBLASLt's row-wise scaling everywhere.
        self.fp8_defer_rows = int(os.environ.get("DSTACK_AMD_FP8_DEFER_ROWS", "1024"))
        if os.environ.get("DSTACK_AMD_FP8_DEFER_SCALE", "1") == "0":
            self.fp8_defer_rows = 1 << 62
        self._one = torch.ones((), device=self.device, dtype=torch.float32)
        self.cos, self.sin = rope_tables(self.max_model_len + sops.PAGE, self.D, cfg.rope_theta, spec.rope_scaling,
                                         self.device)
        self.layers: list[dict] = []
        self.k_cache: list[torch.Tensor] = []
        self.v_cache: list[torch.Tensor] = []
        self.num_pages = 0

    # ------------------------------------------------------------------------------------------
    # weights
    # ------------------------------------------------------------------------------------------
    def _empty(self, *shape):
        return torch.empty(*shape, dtype=self.dtype, device=self.device)

    def allocate_weights(self):
        cfg = self.cfg
        d, hd = cfg.dim, cfg.head_dim
        self.embed = self._empty(cfg.vocab_size, d)  # replicated (an index lookup)
        self.norm = self._empty(d)
        if self.spec.tie_embeddings:
            self.lm_head = self.embed[self.tp_rank * self.V : (self.tp_rank + 1) * self.V]
        else:
            self.lm_head = self._empty(self.V, d)
        self.layers = [
            dict(attn_norm=self._empty(d), wqkv=self._empty(self.NH * hd, d), wo=self._empty(d, self.H * hd),
                 ffn_norm=self._empty(d), wgu=self._empty(2 * self.F, d), wdown=self._empty(d, self.F))
            for _ in range(cfg.n_layers)
        ]
        if self.spec.qkv_bias:
            for L in self.layers:
                L["bqkv"] = self._empty(self.NH * hd)

    # ---- tensor-parallel sharding of full (unsharded) tensors ----
    def _shard(self, kind: str, t: torch.Tensor) -> torch.Tensor:
        """This rank's slice of a full weight: ``q``/``k``/``v`` rows by head, ``wo``/``wdown`` columns,
        ``gate``/``up`` rows by FFN unit, ``vocab`` rows (LM head)."""
        if self.tp == 1:
            return t
        r, hd = self.tp_rank, self.D
        rows = {"q": self.H * hd, "k": self.KVH * hd, "v": self.KVH * hd, "gate": self.F, "up": self.F,
                "vocab": self.V}
        if kind in rows:
            n = rows[kind]
            return t[r * n : (r + 1) * n]
        n = self.H * hd if kind == "wo" else self.F
        return t[:, r * n : (r + 1) * n]

    @torch.no_grad()
    def init_random(self, seed: int = 0, std: float = 0.02):
        """Random-init weights of the architecture (benchmarks: no network, no checkpoints).  Every
        full tensor is drawn from its own generator (seed, name) and then sharded, so a
        tensor-parallel model holds exactly the slices of the single-GPU one."""
        self.allocate_weights()
        cfg = self.cfg
        out_std = std / math.sqrt(2 * cfg.n_layers)
        hd = cfg.head_dim

        def draw(name, shape, sd):
            g = torch.Generator(device=self.device).manual_seed(zlib.crc32(f"{seed}:{name}".encode()))
            return torch.empty(*shape, dtype=self.dtype, device=self.device).normal_(0.0, sd, generator=g)

        self.embed.copy_(draw("embed", self.embed.shape, std))
        if not self.spec.tie_embeddings:
            self.lm_head.copy_(self._shard("vocab", draw("lm_head", (cfg.vocab_size, cfg.dim), std)))
        self.norm.fill_(1.0)
        for i, L in enumerate(self.layers):
            L["attn_norm"].fill_(1.0)
            L["ffn_norm"].fill_(1.0)
            full = draw(f"{i}.wqkv", ((cfg.n_heads + 2 * cfg.n_kv_heads) * hd, cfg.dim), std)
            q, k, v = full.split([cfg.n_heads * hd, cfg.n_kv_heads * hd, cfg.n_kv_heads * hd])
            L["wqkv"].copy_(torch.cat([self._shard("q", q), self._shard("k", k), self._shard("v", v)]))
            full = draw(f"{i}.wgu", (2 * cfg.ffn_dim, cfg.dim), std)
            L["wgu"].copy_(torch.cat([self._shard("gate", full[: cfg.ffn_dim]), self._shard("up", full[cfg.ffn_dim :])]))
            L["wo"].copy_(self._shard("wo", draw(f"{i}.wo", (cfg.dim, cfg.n_heads * hd), out_std)))
            L["wdown"].copy_(self._shard("wdown", draw(f"{i}.wdown", (cfg.dim, cfg.ffn_dim), out_std)))
            if self.spec.qkv_bias:
                b = draw(f"{i}.bqkv", ((cfg.n_heads + 2 * cfg.n_kv_heads) * hd,), std)
                bq, bk, bv = b.split([cfg.n_heads * hd, cfg.n_kv_heads * hd, cfg.n_kv_heads * hd])
                L["bqkv"].copy_(torch.cat([self._shard("q", bq), self._shard("k", bk), self._shard("v", bv)]))
            del full, q, k, v
        return self

    @torch.no_grad()
    def load_hf(self, path: str | None = None):
        """Load an HF Llama safetensors checkpoint (q/k/v and gate/up fused on load)."""
        from safetensors import safe_open

        path = path or self.spec.path
        self.allocate_weights()
        files = sorted(f for f in os.listdir(path) if f.endswith(".safetensors"))
        if not files:
            raise FileNotFoundError(f"no *.safetensors in {path}")
        H, KVH, hd, f = self.H, self.KVH, self.D, self.F  # local (per tensor-parallel rank)
        seen = set()

        def put(dst, src, kind=None):
            if kind is not None:
                src = self._shard(kind, src)
            dst.copy_(src.to(self.device, self.dtype))

        for fn in files:
            with safe_open(os.path.join(path, fn), framework="pt") as st:
                for name in st.keys():
                    t = st.get_tensor(name)
                    seen.add(name)
                    if name == "model.embed_tokens.weight":
                        put(self.embed, t)
                    elif name == "model.norm.weight":
                        put(self.norm, t)
                    elif name == "lm_head.weight":
                        if not self.spec.tie_embeddings:
                            put(self.lm_head, t, "vocab")
                    elif name.startswith("model.layers."):
                        parts = name.split(".")
                        L = self.layers[int(parts[2])]
                        key = ".".join(parts[3:])
                        if key == "input_layernorm.weight":
                            put(L["attn_norm"], t)
                        elif key == "post_attention_layernorm.weight":
                            put(L["ffn_norm"], t)
                        elif key == "self_attn.q_proj.weight":
                            put(L["wqkv"][: H * hd], t, "q")
                        elif key == "self_attn.k_proj.weight":
                            put(L["wqkv"][H * hd : (H + KVH) * hd], t, "k")
                        elif key == "self_attn.v_proj.weight":
                            put(L["wqkv"][(H + KVH) * hd :], t, "v")
                        elif key == "self_attn.o_proj.weight":
                            put(L["wo"], t, "wo")
                        elif key in ("self_attn.q_proj.bias", "self_attn.k_proj.bias", "self_attn.v_proj.bias") \
                                and self.spec.qkv_bias:
                            kind = key.split(".")[1][0]
                            lo = {"q": 0, "k": H * hd, "v": (H + KVH) * hd}[kind]
                            put(L["bqkv"][lo : lo + (H if kind == "q" else KVH) * hd], t, kind)
                        elif key == "mlp.gate_proj.weight":
                            put(L["wgu"][:f], t, "gate")
                        elif key == "mlp.up_proj.weight":
                            put(L["wgu"][f:], t, "up")
                        elif key == "mlp.down_proj.weight":
                            put(L["wdown"], t, "wdown")
                        elif "rotary_emb" not in key:
                            raise ValueError(f"unexpected tensor {name}")
                    else:
                        raise ValueError(f"unexpected tensor {name}")
        expected = {"model.embed_tokens.weight", "model.norm.weight"}
        if not self.spec.tie_embeddings:
            expected.add("lm_head.weight")
        for i in range(self.cfg.n_layers):
            expected |= {f"model.layers.{i}.{k}.weight" for k in (
                "input_layernorm", "post_attention_layernorm", "self_attn.q_proj", "self_attn.k_proj",
                "self_attn.v_proj", "self_attn.o_proj", "mlp.gate_proj", "mlp.up_proj", "mlp.down_proj")}
            if self.spec.qkv_bias:
                expected |= {f"model.layers.{i}.self_attn.{p}_proj.bias" for p in "qkv"}
        missing = expected - seen
        if missing:
            raise ValueError(f"checkpoint {path} is missing {len(missing)} tensors, e.g. {sorted(missing)[:3]}")
        return self

    # projections that fp8 quantization converts (the LM head, embedding and norms stay bf16)
    FP8_KEYS = ("wqkv", "wo", "wgu", "wdown")

    @torch.no_grad()
    def quantize_fp8(self):
        """Convert every layer's projections to e4m3 with per-output-row scales (dynamic per-token
        activation scales at run time), freeing the bf16 copies: halves the weight bytes a decode
        step streams and runs the larger GEMMs on the fp8 MFMA rate."""
        for L in self.layers:
            for k in self.FP8_KEYS:
                w = L[k]
                if isinstance(w, Fp8Weight):
                    continue
                if self.hip:
                    q, sc = _ext.require().quant_fp8_rows(w)
                else:
                    q8, sc = ref.quant_fp8_rows(w)
                    q = q8.view(torch.uint8)
                L[k] = Fp8Weight(q, sc)
                del w
        if self.device.type == "cuda":
            torch.cuda.empty_cache()
        self._add_stream_copies()
        return self

    def _add_stream_copies(self, reserve_bytes: int = 32 << 30):
        """The pre-shuffled second copies of the weights the streaming decode GEMM takes
        (``_stream_cfg``), when they fit with ``reserve_bytes`` of HBM left for the KV cache and
        workspaces; otherwise none (logged) and those GEMMs stay on hipBLASLt."""
        todo = [(L, k) for L in self.layers for k in ("wgu", "wdown")
                if isinstance(L.get(k), Fp8Weight) and L[k].qs is None and self._stream_cfg(*L[k].q.shape)]
        if not todo:
            return
        need = sum(L[k].q.numel() for L, k in todo)
        free, _ = torch.cuda.mem_get_info(self.device)
        if free - need < reserve_bytes:
            logger.warning("fp8 streaming decode GEMM off: its weight copies (%.1f GB) would leave %.1f GB of HBM",
                           need / 1e9, (free - need) / 1e9)
            return
        for L, k in todo:
            L[k].qs = self._stream_copy(k, L[k].q)

    def _stream_cfg(self, N: int, K: int) -> tuple[int, int] | None:
        """(weight rows per wave, K split) the weight-streaming decode GEMM runs an [N, K] fp8 weight
        with, or None where hipBLASLt stays faster (profiles/fp8_stream_shuffle_r9u.txt: gate/up
        N = 57344 and down K = 28672 at 256 rows win; qkv / o lose).  The 8-wave form (32 rows per
        wave, 256 per workgroup): the 7-wave one, whose 224-row workgroups cover all 256 CUs at the
        70B gate/up, measured no faster (117.5 vs 116.2 us, profiles/fp8_stream_shuffle_r9x.txt)."""
        if not (self.hip and self.fp8_stream and self.tp == 1) or not (N >= 32768 or K >= 16384):
            return None
        split = K // 4096 if K > 8192 else 1
        return (32, split) if _ext.require().fp8_stream_gemm_supported(256, N, K, 32, split) else None

    @staticmethod
    def _stream_min_rows(split: int) -> int:
        """Fewest rows the streaming GEMM is used for (its time barely depends on the rows; hipBLASLt's
        does): the unsplit gate/up wins from 160 rows on (111 vs 123 us), the split-K down projection
        only from 224 (71 vs 77 us; at 192, 68 vs 67), profiles/fp8_stream_rows_r9z.txt."""
        return 129 if split == 1 else 224

    def _stream_copy(self, key: str, q: torch.Tensor):
        cfg = self._stream_cfg(*q.shape) if key in ("wgu", "wdown") else None
        if cfg is None:
            return None
        group = 16 if self.fp8_stream_layout == 1 else (224 if cfg[0] == 28 else 256)
        return sops.fp8_stream_shuffle(q, group)

    def weight_bytes(self) -> int:
        ts = [self.embed, self.norm] + ([] if self.spec.tie_embeddings else [self.lm_head])
        n = sum(t.numel() * t.element_size() for t in ts)
        for L in self.layers:
            for t in L.values():
                n += t.nbytes() if isinstance(t, Fp8Weight) else t.numel() * t.element_size()
        return n

    # ------------------------------------------------------------------------------------------
    # KV cache
    # ------------------------------------------------------------------------------------------
    @property
    def cache_dtype(self):
        return torch.float8_e4m3fn if self.kv_cache_dtype == "fp8" else self.dtype

    def kv_bytes_per_page(self) -> int:
        esize = torch.empty(0, dtype=self.cache_dtype).element_size()
        return 2 * self.cfg.n_layers * self.KVH * sops.PAGE * self.D * esize

    def allocate_kv(self, num_pages: int | None = None, gpu_memory_utilization: float = 0.90,
                    reserve_bytes: int = 8 << 30):
        """``num_pages`` pages of every layer's cache; by default as many as fit in
        ``gpu_memory_utilization`` of HBM after the weights and a workspace reserve."""
        if num_pages is None:
            if self.device.type != "cuda":
                num_pages = max(4, (self.max_model_len // sops.PAGE + 1) * 4)
            else:
                free, total = torch.cuda.mem_get_info(self.device)
                used = total - free
                budget = total * gpu_memory_utilization - used - reserve_bytes
                num_pages = int(budget // self.kv_bytes_per_page())
            if self.tp > 1:  # every rank must hold the pages the leader's scheduler hands out
                t = torch.tensor([num_pages], dtype=torch.int64, device=self.device)
                dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.tp_group)
                num_pages = int(t.item())
            if self.device.type == "cuda" and num_pages < self.max_model_len // sops.PAGE + 1:
                raise RuntimeError(f"not enough HBM for the KV cache of one {self.max_model_len}-token sequence")
        self.num_pages = num_pages
        self.k_cache, self.v_cache = [], []
        for _ in range(self.cfg.n_layers):
            k, v = sops.alloc_cache(num_pages, self.KVH, self.cache_dtype, self.device)
            self.k_cache.append(k)
            self.v_cache.append(v)
        return num_pages

    # ------------------------------------------------------------------------------------------
    # fused ops (HIP on the GPU, fp32 references on the CPU)
    # ------------------------------------------------------------------------------------------
    def _fuse_fp8(self, x, w) -> bool:
        """Whether the norm feeding ``w`` should emit e4m3 directly: an fp8 weight multiplied by
        hipBLASLt (more than the GEMV's 4 rows) and a row count the fused kernel covers."""
        return (self.hip and isinstance(w, Fp8Weight) and x.shape[0] > 4 and self.fuse_norm_quant
                and _ext.require().rms_norm_fp8_supported(x.shape[0], x.shape[1]))

    def _rms(self, x, w, next_w=None):
        if self.hip:
            if next_w is not None and self._fuse_fp8(x, next_w):
                _, q, s = _ext.require().rms_norm_fp8(x, None, w, self.cfg.norm_eps)
                return Fp8Act(q, s)
            return _ext.require().rms_norm_fwd(x, w, self.cfg.norm_eps)[0]
        return ref.rms_norm(x, w, self.cfg.norm_eps)

    def _add_rms(self, x, delta, w, next_w=None):
        if self.hip:
            if next_w is not None and self._fuse_fp8(x, next_w):
                if isinstance(delta, RawScaled):  # the delta's fp8 GEMM scales applied in the norm
                    h, q, s = _ext.require().rms_norm_fp8(x, delta.raw, w, self.cfg.norm_eps, delta.rs, delta.cs)
                else:
                    h, q, s = _ext.require().rms_norm_fp8(x, delta, w, self.cfg.norm_eps)
                return h, Fp8Act(q, s)
            if isinstance(delta, RawScaled):
                delta = delta.materialize()
            h, y, _ = _ext.require().add_rms_norm_fwd(x, delta, w, self.cfg.norm_eps)
            return h, y
        return ref.add_rms_norm(x, delta, w, self.cfg.norm_eps)

    def _swiglu(self, gu):
        if self.hip:
            return _ext.require().swiglu_fwd(gu)
        return ref.swiglu(gu)

    def _mm(self, x, w):
        """``x @ w.T``: a batch-1 decode step streams the weights through the HIP GEMV kernel
        (``csrc/gemv.hip``: 6.1-6.8 TB/s on the 70B projections vs hipBLASLt's 5.5-6.2, where it
        wins; at 2-4 rows hipBLASLt is faster, profiles/bench_gemv_r2o.log); larger batches and
        prefill use hipBLASLt."""
        if isinstance(w, Fp8Weight) or isinstance(x, Fp8Act):
            return self._mm_fp8(x, w)
        if self.hip and self.gemv and x.shape[0] == 1:
            C = _ext.require()
            if C.gemv_supported(x.shape[0], x.shape[1]) and x.stride(-1) == 1:
                return C.gemv(x, w)
        return x @ w.t()

    def _mm_fp8(self, x, w: Fp8Weight, defer: str | None = None):
        """``x @ (q * s)^T``: up to 4 rows on the fp8 HIP GEMV (half the weight bytes of the bf16
        one); more rows are quantized per token (HIP) and multiplied by hipBLASLt's fp8 GEMM with
        row-wise scales (``torch._scaled_mm``).

        ``defer`` (prefill-sized batches, ``fp8_defer_rows``): ``"pass"`` runs the GEMM with scalar
        scales and applies the row-wise ones in one in-place pass; ``"raw"`` returns
        ``(raw product, row scales, column scales)`` for a consumer that applies them itself."""
        if isinstance(x, Fp8Act):  # quantized by the fused norm
            xq, xs = x.q, x.s
            M = xq.shape[0]
        else:
            if not self.hip:
                return ref.fp8_linear(x, w.q.view(torch.float8_e4m3fn), w.s)
            C = _ext.require()
            x = x if x.stride(-1) == 1 and x.stride(0) % 8 == 0 else x.contiguous()
            M = x.shape[0]
            if self.gemv and C.gemv_fp8_supported(M, x.shape[1]):
                return C.gemv_fp8(x, w.q, w.s)
            xq, xs = C.quant_fp8_rows(x)
        if w.qs is not None and M <= 256 and xq.stride(0) % 16 == 0:
            rw, split = self._stream_cfg(*w.q.shape)
            if M >= self._stream_min_rows(split):
                return _ext.require().fp8_stream_gemm(xq.view(torch.uint8), xs, w.qs, w.s, rw, split,
                                                      self.fp8_stream_layout)
        if self.hip and self.fp8_gemm == "hip" and M > 4:
            y = self._fp8_rows(xq, xs, w)
            if y is not None:
                return y
        if defer is not None and self.hip and M >= self.fp8_defer_rows and M % 16 == 0:
            raw = torch._scaled_mm(xq.view(torch.float8_e4m3fn), w.q.view(torch.float8_e4m3fn).t(),
                                   scale_a=self._one, scale_b=self._one, out_dtype=self.dtype)
            xs1 = xs.reshape(-1).contiguous()
            if defer == "raw":
                return RawScaled(raw, xs1, w.s)
            return _ext.require().scale_rows_cols_(raw, xs1, w.s)
        pad = -M % 16  # hipBLASLt's fp8 GEMM wants every dimension a multiple of 16
        if pad:  # zero rows (e4m3 0x00 = 0.0) with unit scales
            xq = torch.nn.functional.pad(xq, (0, 0, 0, pad))
            xs = torch.nn.functional.pad(xs, (0, pad), value=1.0)
        y = torch._scaled_mm(xq.view(torch.float8_e4m3fn), w.q.view(torch.float8_e4m3fn).t(),
                             scale_a=xs.view(-1, 1), scale_b=w.s.view(1, -1), out_dtype=self.dtype)
        return y[:M] if pad else y

    def _fp8_rows(self, xq, xs, w: Fp8Weight):
        """The in-tree decode fp8 GEMM (64-row batch blocks x 128 weight rows per workgroup) where it
        beats hipBLASLt (profiles/fp8_decode_gemm_r8j.txt, Llama-3-70B shapes): K <= 8192 and at most
        256 workgroups, i.e. the qkv and o projections up to 128 rows (1.16-1.19x) and o at 256
        (1.04x); the gate/up (many column blocks) and the K = 28672 down projection (64 column
        blocks: hipBLASLt splits K) stay on hipBLASLt."""
        C = _ext.require()
        M, K = xq.shape
        N = w.q.shape[0]
        if M > 256 or K > 8192 or (N // 128) * ((M + 63) // 64) > 256:
            return None
        if xq.stride(0) % 16 or w.q.stride(0) % 16 or not C.fp8_rows_gemm_supported(M, N, K, 64, 1):
            return None
        return C.fp8_rows_gemm(xq.view(torch.uint8), xs, w.q.view(torch.uint8), w.s)

    def _reduce(self, t):
        """Sum the row-parallel partial outputs of the tensor-parallel ranks (RCCL all-reduce)."""
        if self.tp > 1:
            dist.all_reduce(t, group=self.tp_group)
        return t

    def _logits(self, h):
        logits = self._mm(h, self.lm_head)
        if self.tp == 1:
            return logits
        parts = [torch.empty_like(logits) for _ in range(self.tp)]
        dist.all_gather(parts, logits.contiguous(), group=self.tp_group)
        return torch.cat(parts, dim=-1)

    def _mlp_and_attn_out(self, L, x, o):
        """(x + o @ wo^T) -> norm -> SwiGLU MLP; returns (new residual, mlp output)."""
        wo = L["wo"]
        # one rank: the o / down GEMMs' row-wise scales travel with the raw product into the next
        # fused add + RMSNorm; tensor parallel: applied before the all-reduce of the partial sums
        mode = "raw" if self.tp == 1 else "pass"
        ao = self._mm_fp8(o, wo, defer=mode) if isinstance(wo, Fp8Weight) else self._mm(o, wo)
        x, h = self._add_rms(x, self._reduce(ao), L["ffn_norm"], next_w=L["wgu"])
        wgu, wd = L["wgu"], L["wdown"]
        if self.hip and isinstance(wd, Fp8Weight) and isinstance(wgu, Fp8Weight) and not (
                self.gemv and self._rows(h) <= 4):
            # fp8 down projection past the GEMV's rows: SwiGLU and the per-token e4m3 quantization
            # in one kernel (no bf16 product written and re-read); for prefill-sized batches the
            # gate/up GEMM's row-wise scales are applied inside that kernel too
            C = _ext.require()
            fused = self._swiglu_gemm_fp8(h, wgu)
            if fused is not None:
                return x, self._reduce(self._mm_fp8(fused, wd, defer=mode))
            r = self._mm_fp8(h, wgu, defer="raw")
            if isinstance(r, RawScaled):
                q, sc = C.swiglu_quant_fp8_rows(r.raw, r.rs, r.cs)
            else:
                q, sc = C.swiglu_quant_fp8_rows(r if r.stride(-1) == 1 else r.contiguous())
            return x, self._reduce(self._mm_fp8(Fp8Act(q, sc), wd, defer=mode))
        gu = self._mm(h, wgu)
        return x, self._reduce(self._mm(self._swiglu(gu), wd))

    def _swiglu_gemm_fp8(self, h, wgu: Fp8Weight):
        """SwiGLU(h @ Wgu^T) quantized per token to e4m3 (an ``Fp8Act`` for the down projection) by
        the in-tree fp8 GEMM with the SwiGLU in its epilogue, or None where it does not apply
        (rows not a multiple of 256, untiled shapes, ``DSTACK_AMD_FP8_SWIGLU_GEMM=0``)."""
        if not (self.hip and self.fp8_swiglu_gemm):
            return None
        C = _ext.require()
        rows, K = (h.q.shape if isinstance(h, Fp8Act) else h.shape)
        F = wgu.q.shape[0] // 2
        if rows % 256 or not C.gemm_nt_f8_swiglu_supported(rows, F, K) or wgu.q.stride(0) % 16:
            return None
        if isinstance(h, Fp8Act):
            xq, xs = h.q, h.s
        else:
            xq, xs = C.quant_fp8_rows(h if h.stride(-1) == 1 and h.stride(0) % 8 == 0 else h.contiguous())
        if xq.stride(-1) != 1 or xq.stride(0) % 16:
            return None
        q, sc, _ = C.gemm_nt_f8_swiglu_quant(xq.view(torch.uint8), wgu.q.view(torch.uint8),
                                              xs.reshape(-1).contiguous(), wgu.s.reshape(-1).contiguous())
        return Fp8Act(q, sc)

    @staticmethod
    def _rows(h) -> int:
        return h.q.shape[0] if isinstance(h, Fp8Act) else h.shape[0]

    # ------------------------------------------------------------------------------------------
    # forward passes
    # ------------------------------------------------------------------------------------------
    @torch.no_grad()
    def prefill(self, tokens: torch.Tensor, positions: torch.Tensor, slots: torch.Tensor, offsets, lens):
        """Prompts packed into 128-row-aligned segments of one token buffer (``offsets[i]`` is the
        first row of prompt i, ``lens[i]`` its length; padding rows have slot -1).  Writes every
        prompt token's K/V into the cache and returns the logits of each prompt's last token
        [n, vocab]."""
        H, KVH = self.H, self.KVH
        rows = tokens.numel()
        x = F.embedding(tokens, self.embed)
        delta = None
        bounds = []
        for i in range(len(lens)):
            nxt = offsets[i + 1] if i + 1 < len(lens) else rows
            bounds.append((int(offsets[i]), int(nxt) - int(offsets[i])))
        # consecutive segments of one length attend as one batch (one kernel launch instead of one
        # per prompt: a 1024-token prompt alone fills 256 workgroups of a 70B layer)
        groups: list[list[int]] = []
        for off, n in bounds:
            g = groups[-1] if groups else None
            if g is not None and g[1] == n and g[0] + g[1] * g[2] == off:
                g[2] += 1
            else:
                groups.append([off, n, 1])
        for li, L in enumerate(self.layers):
            if delta is None:
                h = self._rms(x, L["attn_norm"], next_w=L["wqkv"])
            else:
                x, h = self._add_rms(x, delta, L["attn_norm"], next_w=L["wqkv"])
            wq = L["wqkv"]
            if isinstance(wq, Fp8Weight) and "bqkv" not in L:
                # prefill-sized: the GEMM's row-wise scales are applied by the RoPE / cache-write kernel
                r = self._mm_fp8(h, wq, defer="raw")
            else:
                r = self._mm(h, wq) if isinstance(wq, Fp8Weight) else h @ wq.t()
            if isinstance(r, RawScaled):
                qkv = r.raw
                sops.rope_cache_write(qkv, positions, slots, self.cos, self.sin, self.k_cache[li], self.v_cache[li],
                                      H, KVH, self.k_scale, self.v_scale, rs=r.rs, cs=r.cs)
            else:
                qkv = r
                if "bqkv" in L:
                    qkv = qkv + L["bqkv"]
                sops.rope_cache_write(qkv, positions, slots, self.cos, self.sin, self.k_cache[li], self.v_cache[li],
                                      H, KVH, self.k_scale, self.v_scale)
            o = torch.empty(rows, H * self.D, dtype=x.dtype, device=x.device)
            for off, n, cnt in groups:
                seg = qkv[off : off + n * cnt].view(cnt, n, -1)
                if self.hip:
                    o[off : off + n * cnt] = _ext.require().flash_attn_fwd(seg, H, KVH, True)[0].view(n * cnt, -1)
                else:
                    q, k, v = seg.view(cnt, n, self.NH, self.D).split([H, KVH, KVH], dim=2)
                    o[off : off + n * cnt] = ref.attention(q, k, v, causal=True).reshape(n * cnt, -1)
            x, delta = self._mlp_and_attn_out(L, x, o)
        last = torch.tensor([int(offsets[i]) + int(lens[i]) - 1 for i in range(len(lens))], device=x.device)
        x, h = self._add_rms(x[last], delta.rows(last) if isinstance(delta, RawScaled) else delta[last], self.norm)
        return self._logits(h)

    @torch.no_grad()
    def decode(self, tokens, positions, slots, block_tables, ctx_lens, ws=None):
        """One new token per sequence (all inputs [B] / [B, W] device tensors, static shapes):
        returns logits [B, vocab].  Rows with ``ctx_lens == 0`` (graph padding) are inert."""
        H, KVH = self.H, self.KVH
        x = F.embedding(tokens, self.embed)
        delta = None
        for li, L in enumerate(self.layers):
            if delta is None:
                h = self._rms(x, L["attn_norm"], next_w=L["wqkv"])
            else:
                x, h = self._add_rms(x, delta, L["attn_norm"], next_w=L["wqkv"])
            qkv = self._mm(h, L["wqkv"])
            if "bqkv" in L:
                qkv = qkv + L["bqkv"]
            sops.rope_cache_write(qkv, positions, slots, self.cos, self.sin, self.k_cache[li], self.v_cache[li], H, KVH,
                                  self.k_scale, self.v_scale)
            o = sops.paged_decode(qkv, self.k_cache[li], self.v_cache[li], block_tables, ctx_lens, H, KVH, ws=ws,
                                  k_scale=self.k_scale, v_scale=self.v_scale)
            x, delta = self._mlp_and_attn_out(L, x, o)
        _, h = self._add_rms(x, delta, self.norm)
        return self._logits(h)
