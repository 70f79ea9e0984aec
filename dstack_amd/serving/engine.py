"""Continuous-batching inference engine (one process, one GPU, one model replica).

Step loop: the native scheduler (``_sched.Scheduler``, C++) plans a PREFILL step (newly admitted
prompts, packed) or a DECODE step (one token for every running sequence); the model runs it; the
fused sampler picks tokens; finished sequences release their KV pages.  Decode steps run from
hipGraphs captured once per batch bucket (padding rows are inert), so a small-batch step costs one
graph launch instead of ~10 kernel launches per layer.

Offline use::

    eng = LLMEngine.from_model("llama-3-8b")
    outs = eng.generate([[1, 2, 3]], SamplingParams(max_tokens=32))

Online use: ``start()`` runs the loop in a background thread; ``add_request`` takes an ``on_event``
callback that receives ``(request, token_id, finished)`` from that thread (the HTTP server turns it
into an asyncio queue).

Tensor parallel (``ServingLlama(tp_group=...)``, one process per GPU under torchrun): rank 0 is the
leader — scheduler, requests, sampling, HTTP — and broadcasts every step's inputs (one packed int64
tensor) to the followers, which run ``follow()``: the same model step on their shard, joining the
step's all-reduces and the logits all-gather.
"""

from __future__ import annotations

import itertools
import threading
import time
from dataclasses import dataclass, field

import numpy as np
import torch
import torch.distributed as dist

from dstack_amd.ops import serving as sops
from dstack_amd.serving.model import ServingLlama, load_spec


@dataclass
class SamplingParams:
    max_tokens: int = 16
    temperature: float = 1.0
    top_p: float = 1.0
    top_k: int = 0
    seed: int | None = None
    ignore_eos: bool = False
    stop_token_ids: tuple = ()


@dataclass
class Request:
    id: int
    prompt_ids: list
    params: SamplingParams
    output_ids: list = field(default_factory=list)
    logprobs: list = field(default_factory=list)
    finished: bool = False
    finish_reason: str | None = None
    arrival: float = field(default_factory=time.perf_counter)
    first_token_at: float | None = None
    finished_at: float | None = None
    on_event: object = None
    seed: int = 0

    @property
    def all_ids(self):
        return self.prompt_ids + self.output_ids


def _buckets(max_batch: int):
    out, b = [], 1
    while b < max_batch:
        out.append(b)
        b = b * 2 if b < 32 else b + 32
    out.append(max_batch)
    return sorted(set(out))


class LLMEngine:
    def __init__(self, model: ServingLlama, max_batch: int = 256, max_prefill_tokens: int = 16384,
                 num_pages: int | None = None, use_graphs: bool | None = None, gpu_memory_utilization: float = 0.90,
                 eos_token_ids=()):
        from dstack_amd.serving import _native

        self.model = model
        self.device = model.device
        self.tp, self.tp_group = model.tp, model.tp_group
        self.leader = model.tp_rank == 0
        if self.tp > 1:
            self._src = dist.get_global_rank(self.tp_group, 0)
        if self.device.type == "cuda":
            from dstack_amd.ops import gemm_tuning

            # hipBLASLt solutions tuned offline for the decode GEMMs (tools/tune_serving_gemms.py)
            self.gemm_tuning = gemm_tuning.setup(device_index=self.device.index or 0, kind="serving")
        if not model.k_cache:
            model.allocate_kv(num_pages, gpu_memory_utilization=gpu_memory_utilization)
        self.max_batch = max_batch
        self.sched = _native.Scheduler(num_pages=model.num_pages, page_size=sops.PAGE, max_batch=max_batch,
                                       max_prefill_tokens=max(max_prefill_tokens, model.max_model_len),
                                       max_model_len=model.max_model_len, pad_to=128)
        self.width = self.sched.table_width
        self.eos_token_ids = tuple(eos_token_ids)
        self.requests: dict[int, Request] = {}
        self._ids = itertools.count()
        self._lock = threading.Lock()
        self._pending: list[Request] = []
        self._wake = threading.Event()
        self._thread = None
        self._stop = False
        # (tensor parallel: eager steps, so every rank issues the same RCCL collectives in order)
        self.use_graphs = (self.device.type == "cuda" and self.tp == 1) if use_graphs is None else use_graphs
        self.buckets = _buckets(max_batch)
        self._graphs: dict[int, torch.cuda.CUDAGraph] = {}
        self._alloc_static()
        self.stats = dict(prefill_tokens=0, decode_tokens=0, steps=0, preemptions=0, prefill_s=0.0, decode_s=0.0)

    @classmethod
    def from_model(cls, model: str, device=None, max_model_len: int | None = None, seed: int = 0, tp_group=None,
                   quantization: str | None = None, kv_cache_dtype: str = "auto", **kw):
        spec = load_spec(model)
        device = device or ("cuda" if torch.cuda.is_available() else "cpu")
        m = ServingLlama(spec, device, max_model_len=max_model_len, tp_group=tp_group, quantization=quantization,
                         kv_cache_dtype=kv_cache_dtype)
        if spec.path:
            m.load_hf()
        else:
            m.init_random(seed)
        if quantization == "fp8":
            m.quantize_fp8()  # before the KV cache is sized: the freed bf16 bytes become KV pages
        return cls(m, eos_token_ids=spec.eos_token_ids, **kw)

    # ------------------------------------------------------------------------------------------
    def _alloc_static(self):
        dev, B, W = self.device, self.max_batch, self.width
        i32 = dict(dtype=torch.int32, device=dev)
        self.s_tokens = torch.zeros(B, dtype=torch.int64, device=dev)
        self.s_pos = torch.zeros(B, **i32)
        self.s_slots = torch.full((B,), -1, **i32)
        self.s_tables = torch.zeros(B, W, **i32)
        self.s_ctx = torch.zeros(B, **i32)
        self.s_temps = torch.zeros(B, dtype=torch.float32, device=dev)
        self.s_seeds = torch.zeros(B, dtype=torch.int64, device=dev)
        self.s_steps = torch.zeros(B, **i32)
        self.s_out_tok = torch.zeros(B, **i32)
        self.s_out_lp = torch.zeros(B, dtype=torch.float32, device=dev)
        self._ws = {b: sops.DecodeWorkspace(b, self.model.H, self.model.KVH, W, dev) for b in self.buckets}
        self.s_logits = None  # last decode logits (graph output) for top-k/top-p re-sampling

    def _decode_body(self, b: int):
        logits = self.model.decode(self.s_tokens[:b], self.s_pos[:b], self.s_slots[:b], self.s_tables[:b],
                                   self.s_ctx[:b], ws=self._ws[b])
        sops.sample(logits, self.s_temps[:b], self.s_seeds[:b], self.s_steps[:b], self.s_out_tok[:b],
                    self.s_out_lp[:b])
        return logits

    def capture_graphs(self):
        """One hipGraph per batch bucket (largest first, sharing one memory pool)."""
        if not self.use_graphs or self._graphs:
            return
        self.s_slots.fill_(-1)
        self.s_ctx.zero_()
        self.s_temps.zero_()
        torch.cuda.synchronize(self.device)
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            # warm-up of every bucket: each row count may take a different GEMM path (HIP GEMV up to
            # 4 rows, the in-tree fp8 GEMM, hipBLASLt) and hipBLASLt may not set up a kernel inside
            # a capture ('operation not permitted when stream is capturing')
            for b in self.buckets:
                self._decode_body(b)
        torch.cuda.current_stream(self.device).wait_stream(s)
        pool = torch.cuda.graph_pool_handle()
        self._graph_logits = {}
        for b in reversed(self.buckets):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=pool):
                self._graph_logits[b] = self._decode_body(b)
            self._graphs[b] = g
        torch.cuda.synchronize(self.device)

    # ------------------------------------------------------------------------------------------
    def add_request(self, prompt_ids, params: SamplingParams | None = None, on_event=None) -> Request:
        params = params or SamplingParams()
        if not prompt_ids:
            raise ValueError("empty prompt")
        if len(prompt_ids) >= self.model.max_model_len:
            raise ValueError(f"prompt of {len(prompt_ids)} tokens does not fit max_model_len {self.model.max_model_len}")
        vocab = self.model.cfg.vocab_size
        if min(prompt_ids) < 0 or max(prompt_ids) >= vocab:
            raise ValueError(f"token ids must be in [0, {vocab})")
        rid = next(self._ids)
        seed = params.seed if params.seed is not None else (rid * 7919 + 17)
        req = Request(rid, list(prompt_ids), params, on_event=on_event, seed=int(seed))
        with self._lock:
            self.requests[rid] = req
            self._pending.append(req)
        self._wake.set()
        return req

    def abort(self, rid: int):
        with self._lock:
            req = self.requests.get(rid)
            if req is not None and not req.finished:
                req.finished, req.finish_reason = True, "abort"
                req.finished_at = time.perf_counter()
                self._aborted = getattr(self, "_aborted", set()) | {rid}
        self._wake.set()

    def has_work(self) -> bool:
        return bool(self._pending) or self.sched.num_running > 0 or self.sched.num_waiting > 0

    # ------------------------------------------------------------------------------------------
    def _admit_pending(self):
        with self._lock:
            pending, self._pending = self._pending, []
            aborted, self._aborted = getattr(self, "_aborted", set()), set()
        for req in pending:
            if req.finished:
                continue
            self.sched.add(req.id, len(req.prompt_ids), len(req.prompt_ids) + req.params.max_tokens)
        for rid in aborted:
            self.sched.finish(rid)
            self._emit(self.requests.pop(rid, None), None, True)

    def _emit(self, req, token, finished):
        if req is not None and req.on_event is not None:
            req.on_event(req, token, finished)

    def step(self) -> int:
        """Run one scheduled step; returns the number of tokens produced."""
        self._admit_pending()
        plan = self.sched.schedule(False)
        for rid in plan["preempted"]:
            self.stats["preemptions"] += 1
        kind = plan["kind"]
        if kind == "idle":
            return 0
        ids = list(plan["seq_ids"])
        reqs = [self.requests[i] for i in ids]
        t0 = time.perf_counter()
        if kind == "prefill":
            toks = np.zeros(plan["rows"], dtype=np.int64)
            for r, off, n in zip(reqs, plan["offsets"], plan["lens"]):
                toks[off : off + n] = r.all_ids[:n]
            if self.tp > 1:
                self._bcast_prefill(toks, plan["positions"], plan["slots"], plan["offsets"], plan["lens"])
            dev = self.device
            logits = self.model.prefill(torch.from_numpy(toks).to(dev), torch.from_numpy(plan["positions"]).to(dev),
                                        torch.from_numpy(plan["slots"]).to(dev), plan["offsets"], plan["lens"])
            tokens, lps = self._sample(logits, reqs)
            self.stats["prefill_tokens"] += int(sum(plan["lens"]))
            self.stats["prefill_s"] += time.perf_counter() - t0
        else:
            tokens, lps = self._decode(plan, reqs)
            self.stats["decode_tokens"] += len(reqs)
            self.stats["decode_s"] += time.perf_counter() - t0
        self.stats["steps"] += 1
        now = time.perf_counter()
        for req, tok, lp in zip(reqs, tokens, lps):
            self.sched.mark_computed(req.id)
            if req.finished:  # aborted while the step ran
                continue
            tok = int(tok)
            req.output_ids.append(tok)
            req.logprobs.append(float(lp))
            if req.first_token_at is None:
                req.first_token_at = now
            self.sched.append(req.id)
            reason = None
            if len(req.output_ids) >= req.params.max_tokens:
                reason = "length"
            elif not req.params.ignore_eos and (tok in self.eos_token_ids or tok in req.params.stop_token_ids):
                reason = "stop"
            elif len(req.all_ids) >= self.model.max_model_len:
                reason = "length"
            if reason:
                req.finished, req.finish_reason, req.finished_at = True, reason, now
                self.sched.finish(req.id)
            self._emit(req, tok, req.finished)
            if req.finished:
                self.requests.pop(req.id, None)
        return len(reqs)

    def _seed_rows(self, reqs):
        temps = torch.tensor([r.params.temperature for r in reqs], dtype=torch.float32)
        seeds = torch.tensor([r.seed for r in reqs], dtype=torch.int64)
        steps = torch.tensor([len(r.output_ids) for r in reqs], dtype=torch.int32)
        return temps, seeds, steps

    def _sample(self, logits, reqs):
        temps, seeds, steps = (t.to(self.device) for t in self._seed_rows(reqs))
        logits = _filter_top_k_top_p(logits, reqs)
        tok, lp = sops.sample(logits, temps, seeds, steps)
        return tok.tolist(), lp.tolist()

    def _decode(self, plan, reqs):
        n = len(reqs)
        b = next(x for x in self.buckets if x >= n)
        temps, seeds, steps = self._seed_rows(reqs)
        last = torch.tensor([r.all_ids[-1] for r in reqs], dtype=torch.int64)
        nb = torch.from_numpy
        with torch.no_grad():
            # stage the step's inputs into the static buffers (padding rows: inert)
            self.s_tokens[:n].copy_(last, non_blocking=True)
            self.s_pos[:n].copy_(nb(plan["positions"]), non_blocking=True)
            self.s_slots[:n].copy_(nb(plan["slots"]), non_blocking=True)
            self.s_tables[:n].copy_(nb(plan["block_tables"]), non_blocking=True)
            self.s_ctx[:n].copy_(nb(plan["ctx_lens"]), non_blocking=True)
            self.s_temps[:n].copy_(temps, non_blocking=True)
            self.s_seeds[:n].copy_(seeds, non_blocking=True)
            self.s_steps[:n].copy_(steps, non_blocking=True)
            if b > n:
                self.s_slots[n:b].fill_(-1)
                self.s_ctx[n:b].zero_()
                self.s_temps[n:b].zero_()
            filtered = any(r.params.top_p < 1.0 or r.params.top_k > 0 for r in reqs)
            if self.tp > 1:
                self._bcast_decode(b)
            if self._graphs and b in self._graphs:
                self._graphs[b].replay()
                logits = self._graph_logits[b]
            else:
                logits = self._decode_body(b)
            if filtered:
                logits = _filter_top_k_top_p(logits[:n], reqs)
                sops.sample(logits, self.s_temps[:n], self.s_seeds[:n], self.s_steps[:n], self.s_out_tok[:n],
                            self.s_out_lp[:n])
            return self.s_out_tok[:n].tolist(), self.s_out_lp[:n].tolist()

    # ------------------------------------------------------------------------------------------
    # tensor parallel: the leader broadcasts each step's inputs, followers replay them
    # ------------------------------------------------------------------------------------------
    _STOP, _PREFILL, _DECODE = 0, 1, 2

    def _bcast(self, header, payload=None):
        hdr = torch.tensor(header + [0] * (4 - len(header)), dtype=torch.int64, device=self.device)
        dist.broadcast(hdr, src=self._src, group=self.tp_group)
        if payload is not None:
            dist.broadcast(payload, src=self._src, group=self.tp_group)

    def _bcast_prefill(self, toks, positions, slots, offsets, lens):
        parts = [np.asarray(a, dtype=np.int64) for a in (toks, positions, slots, offsets, lens)]
        payload = torch.from_numpy(np.concatenate(parts)).to(self.device)
        self._bcast([self._PREFILL, len(lens), len(toks)], payload)

    def _bcast_decode(self, b: int):
        payload = torch.cat([self.s_tokens[:b], self.s_pos[:b].long(), self.s_slots[:b].long(), self.s_ctx[:b].long(),
                             self.s_tables[:b].long().flatten()])
        self._bcast([self._DECODE, b, b, self.width], payload)

    @torch.no_grad()
    def follow(self):
        """Follower rank loop: run the leader's steps on this rank's shard until it stops."""
        assert self.tp > 1 and not self.leader
        dev = self.device
        while True:
            hdr = torch.empty(4, dtype=torch.int64, device=dev)
            dist.broadcast(hdr, src=self._src, group=self.tp_group)
            kind, n, rows, width = hdr.tolist()
            if kind == self._STOP:
                return
            if kind == self._PREFILL:
                payload = torch.empty(3 * rows + 2 * n, dtype=torch.int64, device=dev)
                dist.broadcast(payload, src=self._src, group=self.tp_group)
                toks, pos, slots, offsets, lens = payload.split([rows, rows, rows, n, n])
                self.model.prefill(toks, pos.int(), slots.int(), offsets.tolist(), lens.tolist())
            else:
                b = n
                payload = torch.empty(4 * b + b * width, dtype=torch.int64, device=dev)
                dist.broadcast(payload, src=self._src, group=self.tp_group)
                toks, pos, slots, ctx, tables = payload.split([b, b, b, b, b * width])
                self.s_tokens[:b].copy_(toks)
                self.s_pos[:b].copy_(pos)
                self.s_slots[:b].copy_(slots)
                self.s_ctx[:b].copy_(ctx)
                self.s_tables[:b].copy_(tables.view(b, width))
                self.model.decode(self.s_tokens[:b], self.s_pos[:b], self.s_slots[:b], self.s_tables[:b],
                                  self.s_ctx[:b], ws=self._ws[b])

    def shutdown(self):
        """Leader: release the followers (tensor parallel) and stop the loop thread."""
        self.stop()
        if self.tp > 1 and self.leader and not getattr(self, "_released", False):
            self._released = True
            self._bcast([self._STOP])

    # ------------------------------------------------------------------------------------------
    def generate(self, prompts, params: SamplingParams | list | None = None) -> list[Request]:
        """Offline batch generation: returns the finished requests in prompt order."""
        ps = params if isinstance(params, list) else [params or SamplingParams()] * len(prompts)
        reqs = [self.add_request(p, sp) for p, sp in zip(prompts, ps)]
        while any(not r.finished for r in reqs):
            self.step()
        return reqs

    # ------------------------------------------------------------------------------------------
    def start(self):
        if self._thread is not None:
            return
        self._stop = False
        self._thread = threading.Thread(target=self._loop, name="dstack-amd-engine", daemon=True)
        self._thread.start()

    def stop(self):
        self._stop = True
        self._wake.set()
        if self._thread is not None:
            self._thread.join(timeout=30)
            self._thread = None

    def _loop(self):
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        while not self._stop:
            if not self.has_work():
                self._wake.wait(timeout=0.5)
                self._wake.clear()
                continue
            try:
                self.step()
            except Exception as e:  # noqa: BLE001 - fail every in-flight request, keep serving
                import logging

                logging.getLogger(__name__).exception("engine step failed")
                with self._lock:
                    victims = list(self.requests.values())
                    self.requests.clear()
                    self._pending.clear()
                for r in victims:
                    self.sched.finish(r.id)
                    r.finished, r.finish_reason = True, f"error: {e}"
                    self._emit(r, None, True)

    def metrics(self) -> dict:
        return dict(self.stats, running=self.sched.num_running, waiting=self.sched.num_waiting + len(self._pending),
                    kv_pages_free=self.sched.free_pages, kv_pages_total=self.sched.num_pages,
                    kv_usage=1.0 - self.sched.free_pages / max(1, self.sched.num_pages))


def _filter_top_k_top_p(logits: torch.Tensor, reqs) -> torch.Tensor:
    """Mask logits outside each row's top-k / nucleus (top-p) set to -inf (rows that ask for it)."""
    if not any(r.params.top_p < 1.0 or r.params.top_k > 0 for r in reqs):
        return logits
    out = logits.clone()
    for i, r in enumerate(reqs):
        k, p = r.params.top_k, r.params.top_p
        if k <= 0 and p >= 1.0:
            continue
        row = out[i].float()
        if r.params.temperature > 0:
            row = row / r.params.temperature
        if k > 0:
            kth = torch.topk(row, min(k, row.numel())).values[-1]
            out[i][row < kth] = float("-inf")
            row = row.masked_fill(row < kth, float("-inf"))
        if p < 1.0:
            srt, idx = torch.sort(row, descending=True)
            cum = torch.softmax(srt, dim=-1).cumsum(-1)
            drop = cum - torch.softmax(srt, dim=-1) > p  # keep the smallest prefix reaching p
            out[i][idx[drop]] = float("-inf")
    return out
