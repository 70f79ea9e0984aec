"""ZeRO-1 data parallelism over RCCL with flat, bucketed parameter/gradient storage.

Design (MI355X-first, not a DDP translation):

* **One flat bf16 parameter buffer and one flat bf16 gradient buffer.** Every ``nn.Parameter`` is a
  view into them, laid out in *reverse* registration order so that the parameters whose gradients
  are produced first in backward are contiguous. A bucket is a contiguous slice of both buffers,
  padded to a multiple of ``world_size * 64`` elements, so reduce-scatter/all-gather run on
  buffers in place with no packing copies.
* **Gradient reduce-scatter overlapped with backward.** A post-accumulate-grad hook counts down the
  parameters of each bucket; when a bucket is complete it is reduce-scattered
  asynchronously on RCCL's stream while autograd keeps computing earlier layers (SUM; the
  1/world of the average is folded into the AdamW kernel's grad scale).
* **Sharded fp32 optimizer state.** Rank r owns shard r of every bucket: fp32 master weights, Adam
  m and v (12 B/param / world_size). With 288 GB HBM3E per GPU, a single GPU holds the full 8B
  model state (≈128 GB); with 8 GPUs the optimizer state shrinks to ≈12 GB per GPU.
* **Fused AdamW** (``ops.adamw_``, one HIP kernel per bucket shard) then an all-gather of the
  updated bf16 shards back into the flat parameter buffer.
* Bucket size defaults to 256 Mi elements (512 MB bf16): xGMI rings are per-link bound (≈153 GB/s
  per link), so few large collectives amortise RCCL launch latency; backward of one Llama-3-8B
  layer produces ≈436 MB of gradients, so a bucket completes roughly every layer.
"""

from __future__ import annotations

import math

from dataclasses import dataclass, field

import torch
import torch.distributed as dist
import torch.nn as nn

from dstack_amd import ops

ALIGN = 64


@dataclass
class Bucket:
    index: int
    start: int  # offset in the flat buffers
    numel: int  # padded
    params: list = field(default_factory=list)
    pending: int = 0
    work: object = None
    ag_work: object = None
    updated: bool = False  # AdamW already ran for this step (optimizer-in-backward)

    def shard_range(self, rank: int, world: int):
        n = self.numel // world
        return self.start + rank * n, n


class ZeroOptimizer:
    def __init__(
        self,
        model: nn.Module,
        lr: float = 3e-4,
        betas=(0.9, 0.95),
        eps: float = 1e-8,
        weight_decay: float = 0.1,
        bucket_numel: int = 256 * 1024 * 1024,
        group: dist.ProcessGroup | None = None,
        overlap: bool = True,
        overlap_update: bool = True,
        force_collectives: bool | None = None,
        clip_grad_norm: float = 0.0,
        grad_accum_fp32: bool | None = None,
    ):
        self.model = model
        self.lr = lr
        # global gradient-norm clipping (0 = off).  The norm of the whole (averaged) gradient is
        # known only after backward, so with clipping AdamW runs in step() over every bucket --
        # the reduce-scatters still overlap backward and the all-gathers the next forward; only
        # the AdamW update itself leaves the backward's shadow.
        self.clip_grad_norm = float(clip_grad_norm)
        self.skipped_steps = 0  # optimizer steps skipped for a non-finite gradient norm (clipping on)
        self.last_grad_norm: float | None = None
        self.beta1, self.beta2 = betas
        self.eps = eps
        self.weight_decay = weight_decay
        self.group = group
        self.distributed = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if self.distributed else 1
        self.rank = dist.get_rank(group) if self.distributed else 0
        import os

        # debug/validation switch: issue the real reduce-scatter / all-gather even in a 1-rank
        # group (a valid 1-rank RCCL communicator), so the exact collective code path of an
        # 8-GPU job -- in-place RS/AG on RCCL's stream, joined from the side stream and the
        # prefetch hooks -- can run and be checked on a single-GPU box
        if force_collectives is None:
            force_collectives = os.environ.get("DSTACK_AMD_ZERO_FORCE_COLLECTIVES", "0") not in ("0", "", "false")
        self.collectives = self.distributed and (self.world > 1 or force_collectives)
        self.overlap = overlap and self.collectives
        self.step_count = 0
        # optimizer-in-backward: a bucket whose final gradients are complete is reduce-scattered,
        # updated (AdamW on its shard) and all-gathered on a side stream while backward keeps
        # computing earlier layers (HBM-bound AdamW beside MFMA-bound GEMMs)
        self.sync_grads = True  # False while accumulating non-final micro-batches

        params = [p for p in model.parameters() if p.requires_grad]
        device = params[0].device
        dtype = params[0].dtype
        # ---- bucket layout (reverse registration order ≈ gradient production order) ----
        self.buckets: list[Bucket] = []
        pad_to = self.world * ALIGN
        cur = Bucket(0, 0, 0)
        off = 0
        layout = []
        for p in reversed(params):
            n = p.numel()
            if cur.params and cur.numel + n > bucket_numel:
                cur.numel = _round_up(cur.numel, pad_to)
                off = cur.start + cur.numel
                self.buckets.append(cur)
                cur = Bucket(len(self.buckets), off, 0)
            layout.append((p, cur.start + cur.numel))
            cur.params.append(p)
            cur.numel += n
        cur.numel = _round_up(cur.numel, pad_to)
        self.buckets.append(cur)
        self.total_numel = cur.start + cur.numel

        self.flat_param = torch.zeros(self.total_numel, dtype=dtype, device=device)
        self.flat_grad = torch.zeros(self.total_numel, dtype=dtype, device=device)
        # fp32 accumulation of the GEMM weight gradients over micro-batches (DSTACK_AMD_GRAD_ACCUM_FP32
        # or ``grad_accum_fp32``): micro-batches 1..n-1 are summed in an fp32 buffer by the weight-
        # gradient GEMM's epilogue and the last one writes bf16(fp32 sum + its own tile) into
        # flat_grad -- one rounding per optimizer step instead of one per micro-batch.  The buffer
        # (4 bytes per parameter) is allocated at the first non-final micro-batch, so runs without
        # gradient accumulation never hold it.  Norm weights and the embedding accumulate in bf16.
        if grad_accum_fp32 is None:
            grad_accum_fp32 = os.environ.get("DSTACK_AMD_GRAD_ACCUM_FP32", "0") not in ("0", "", "false")
        self.grad_accum_fp32 = bool(grad_accum_fp32) and dtype == torch.bfloat16
        self.acc32 = None
        self._offset = {}
        self._bucket_of = {}
        for p, o in layout:
            n = p.numel()
            self.flat_param[o : o + n].copy_(p.detach().reshape(-1))
            p.data = self.flat_param[o : o + n].view_as(p)
            p.grad = self.flat_grad[o : o + n].view_as(p)
            self._offset[p] = o
        for b in self.buckets:
            for p in b.params:
                self._bucket_of[p] = b

        # ---- sharded fp32 state ----
        self.master, self.exp_avg, self.exp_avg_sq = [], [], []
        for b in self.buckets:
            s, n = b.shard_range(self.rank, self.world)
            self.master.append(self.flat_param[s : s + n].float())
            self.exp_avg.append(torch.zeros(n, dtype=torch.float32, device=device))
            self.exp_avg_sq.append(torch.zeros(n, dtype=torch.float32, device=device))

        # padding between buckets' real params is never written by backward: zero it once per step
        self._pads = []
        for b in self.buckets:
            used = sum(p.numel() for p in b.params)
            if used < b.numel:
                self._pads.append((b.start + used, b.numel - used))
        self._side = None
        if os.environ.get("DSTACK_AMD_OPT_OVERLAP") is not None:
            overlap_update = os.environ["DSTACK_AMD_OPT_OVERLAP"] not in ("0", "false", "")
        if overlap_update and device.type == "cuda":
            self._side = torch.cuda.Stream(device=device)
        # AdamW beside backward runs on a capped grid (persistent workgroups on a few CUs) so the
        # compute kernels keep the rest of the chip; 0 = full grid
        self._side_blocks = int(os.environ.get("DSTACK_AMD_ADAMW_SIDE_BLOCKS", "0"))
        self._hooks_on = self.overlap or self._side is not None
        self._hooks = []
        for p in params:
            if p.dim() == 2:
                # GEMM-produced weight gradients are written straight into flat_grad (ops.linear)
                p._dsa_grad_sink = self._direct_grad
                p._dsa_fresh = True
                # weight generation: ops.linear caches W^T for the input-gradient GEMM per generation
                p._dsa_wgen = self._weight_generation
            # norm weights (RMSNorm backward's column-sum kernel) and the token embedding (sorted,
            # fp32 segment-sum scatter kernel) write their gradients into flat_grad themselves too
            # (ops.functional); a 2-D weight used by ops.linear only ever uses the sink above
            p._dsa_grad_writer = self._direct_write
            p._dsa_fresh = True
            if self._hooks_on:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad_ready))
        self._direct_ok = set()
        self._prefetch = False
        self._wgen = 0
        self._arm()

    def _weight_generation(self) -> int:
        """Changes whenever the parameters are rewritten (optimizer step, checkpoint load)."""
        return self._wgen

    # ------------------------------------------------------------------------------------------
    def _arm(self):
        for b in self.buckets:
            b.pending = len(b.params)
            b.work = None
            b.updated = False
        # parameters already counted down in this step's synchronising backward (see _on_grad_ready)
        self._reported = set()

    def _acc32_view(self, p: torch.Tensor) -> torch.Tensor:
        if self.acc32 is None:
            self.acc32 = torch.zeros(self.total_numel, dtype=torch.float32, device=self.flat_grad.device)
        o = self._offset[p]
        return self.acc32[o : o + p.numel()].view(p.shape)

    def _direct_grad(self, p: torch.Tensor, a: torch.Tensor, b: torch.Tensor):
        """Weight gradient sink for ``ops.linear``: dW = a @ b (a = g^T [P, T], b = x [T, Q], as
        views in whichever layout ``ops.functional.wgrad_operands`` chose) into the flat buffer."""
        if self.grad_accum_fp32 and not (p._dsa_fresh and self.sync_grads):
            # 0: first of several micro-batches -> fp32; 1: a middle one, fp32 += ; 2: the last one,
            # bf16(fp32 + this) into flat_grad
            mode = 2 if self.sync_grads else (0 if p._dsa_fresh else 1)
            ops.functional.mm_into_f32(a, b, self._acc32_view(p), p.grad, mode)
        else:
            ops.functional.mm_into(a, b, p.grad, accumulate=not p._dsa_fresh)
        p._dsa_fresh = False
        self._direct_ok.add(p)
        if self._hooks_on:
            self._on_grad_ready(p)

    def _direct_write(self, p: torch.Tensor, write):
        """Gradient writer for kernels that produce a parameter's gradient themselves:
        ``write(dst, accumulate)`` fills (first micro-batch) or adds into ``p.grad``."""
        write(p.grad, not p._dsa_fresh)
        p._dsa_fresh = False
        self._direct_ok.add(p)
        if self._hooks_on:
            self._on_grad_ready(p)

    def _on_grad_ready(self, p: torch.Tensor):
        """Count ``p`` down in its bucket; the bucket's reduce-scatter / AdamW start at zero.

        A parameter whose gradient a kernel writes directly (GEMM sink, norm writer) reports from
        inside its op's backward, and PyTorch then STILL runs its post-accumulate-grad hook (the
        op returned None for it: the hook fires with an undefined gradient).  Without the
        ``_reported`` set that second report counted the bucket down twice, so it could be
        reduce-scattered / updated before its last parameter's gradient had landed."""
        if not self.sync_grads:
            return
        if p in self._reported:
            return
        self._reported.add(p)
        b = self._bucket_of[p]
        b.pending -= 1
        if b.pending == 0:
            if self.overlap:
                self._reduce_bucket(b, async_op=True)
            if self._side is not None and not self.clip_grad_norm:
                self._update_bucket_async(b)

    def _adamw(self, b: Bucket, step: int, max_blocks: int = 0, clip_scale: float = 1.0):
        s, n = b.shard_range(self.rank, self.world)
        i = b.index
        ops.adamw_(self.flat_param[s : s + n], self.flat_grad[s : s + n], self.master[i], self.exp_avg[i],
                   self.exp_avg_sq[i], lr=self.lr, beta1=self.beta1, beta2=self.beta2, eps=self.eps,
                   weight_decay=self.weight_decay, step=step,
                   # the 1/world of the average (and the clip factor) are fused into AdamW
                   grad_scale=clip_scale / self.world, max_blocks=max_blocks)

    def _grad_norm(self, buckets) -> float:
        """L2 norm of the averaged gradient: each rank's reduced shards, summed over ranks."""
        sq = torch.zeros((), dtype=torch.float32, device=self.flat_grad.device)
        for b in buckets:
            s, n = b.shard_range(self.rank, self.world)
            sq += torch.linalg.vector_norm(self.flat_grad[s : s + n], dtype=torch.float32).square()
        if self.collectives:
            dist.all_reduce(sq, group=self.group)
        return float(sq.sqrt().item()) / self.world

    def _all_gather(self, b: Bucket):
        s, n = b.shard_range(self.rank, self.world)
        full = self.flat_param[b.start : b.start + b.numel]
        # in place: sendbuff == recvbuff + rank * sendcount (the same call on RCCL and, in the CPU
        # tests, on gloo, so the multi-rank tests run the code path the GPUs run)
        b.ag_work = dist.all_gather_into_tensor(full, self.flat_param[s : s + n], group=self.group, async_op=True)

    @torch.no_grad()
    def _update_bucket_async(self, b: Bucket):
        """Called from backward as soon as bucket ``b`` holds its final gradients.  Ordering:
        compute stream (grads written, and the bucket's weights already read by its dgrad GEMMs,
        which ops.linear issues before the weight-gradient sink) -> [reduce-scatter] -> side
        stream: AdamW -> [all-gather].  ``step()`` joins the side stream."""
        side = self._side
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            if b.work is not None:
                b.work.wait()  # the side stream waits for the reduce-scatter
                b.work = None
            self._adamw(b, self.step_count + 1, self._side_blocks)
            if self.collectives:
                self._all_gather(b)
        b.updated = True

    def _reduce_bucket(self, b: Bucket, async_op: bool):
        if not self.collectives:
            return
        s, n = b.shard_range(self.rank, self.world)
        full = self.flat_grad[b.start : b.start + b.numel]
        out = self.flat_grad[s : s + n]
        # in place: RCCL reduce-scatters when recvbuff == sendbuff + rank * recvcount
        b.work = dist.reduce_scatter_tensor(
            out, full, op=dist.ReduceOp.SUM, group=self.group, async_op=async_op
        )

    def zero_grad(self):
        """Zero only what backward accumulates into through autograd (norm weights, embedding)
        and the bucket padding; GEMM weight gradients are overwritten by the first micro-batch."""
        for b in self.buckets:
            for p in b.params:
                if p in self._direct_ok:
                    p._dsa_fresh = True
                else:
                    p.grad.zero_()
        for off, n in self._pads:
            self.flat_grad[off : off + n].zero_()
        self._direct_ok = set()
        self._arm()

    # ---- checkpointing (reference: none -- dstack leaves ML checkpoints to the job) ----
    def shard_state(self) -> dict:
        """This rank's fp32 AdamW state (master weights, first and second moments) by bucket."""
        out = {}
        for i in range(len(self.buckets)):
            out[f"master.{i}"] = self.master[i]
            out[f"exp_avg.{i}"] = self.exp_avg[i]
            out[f"exp_avg_sq.{i}"] = self.exp_avg_sq[i]
        return out

    @torch.no_grad()
    def load_state(self, flat_param: torch.Tensor, shard: dict, step_count: int):
        """Restore from :meth:`shard_state` of the same rank in a job of the same world size and
        the full bf16 parameter buffer."""
        if flat_param.numel() != self.total_numel:
            raise ValueError(f"checkpoint has {flat_param.numel()} parameters, this model {self.total_numel}")
        self.flat_param.copy_(flat_param.to(self.flat_param.device, self.flat_param.dtype))
        for i in range(len(self.buckets)):
            for name, dst in (("master", self.master), ("exp_avg", self.exp_avg), ("exp_avg_sq", self.exp_avg_sq)):
                src = shard[f"{name}.{i}"]
                if src.numel() != dst[i].numel():
                    raise ValueError(f"{name}.{i}: shard of {src.numel()} elements, expected {dst[i].numel()} "
                                     "(checkpoints restore only into the same world size)")
                dst[i].copy_(src.to(dst[i].device))
        self.step_count = step_count
        self._wgen += 1

    @torch.no_grad()
    def step(self):
        self.wait_params()  # no forward ran since the last step: finish its all-gathers first
        self.step_count += 1
        self._wgen += 1
        pending = [b for b in self.buckets if not b.updated]
        if self.collectives:
            for b in pending:
                if b.work is None:  # not overlapped (or a param received no grad)
                    self._reduce_bucket(b, async_op=False)
                else:
                    b.work.wait()
                    b.work = None
        clip_scale = 1.0
        if self.clip_grad_norm:
            norm = self._grad_norm(self.buckets)  # all-reduced: every rank sees the same value
            self.last_grad_norm = norm
            if not math.isfinite(norm):
                # an inf/NaN gradient would poison the fp32 master weights and both moments for
                # good: skip the update on every rank (the same decision everywhere, so shards and
                # step counts stay consistent; parameters are unchanged, nothing to all-gather)
                self.step_count -= 1
                self.skipped_steps += 1
                for b in self.buckets:
                    b.updated = False
                return
            if norm > self.clip_grad_norm:
                clip_scale = self.clip_grad_norm / (norm + 1e-6)
        for b in pending:
            self._adamw(b, self.step_count, clip_scale=clip_scale)
        if self.collectives:
            # gather the updated shards in forward order (buckets are stored in backward order);
            # with prefetch hooks installed the next forward waits per bucket, so the all-gather
            # of later layers overlaps the compute of earlier ones
            for b in reversed(pending):
                self._all_gather(b)
        if self._side is not None:
            torch.cuda.current_stream().wait_stream(self._side)
        for b in self.buckets:
            b.updated = False
        if self.collectives and not self._prefetch:
            self.wait_params()

    def wait_params(self, buckets=None):
        """Block until the all-gathered parameters of ``buckets`` (default: all) have landed."""
        for b in buckets if buckets is not None else self.buckets:
            if b.ag_work is not None:
                b.ag_work.wait()
                b.ag_work = None

    def install_prefetch_hooks(self, model: nn.Module):
        """Overlap the parameter all-gather with the next forward: each module waits only for
        the buckets holding its own parameters (forward pre-hook); anything not covered by a
        hook is waited for before backward / the next optimizer step."""
        if not self.collectives:
            return
        self._prefetch = True
        for mod in model.modules():
            if hasattr(mod, "param_waiter"):
                # the module waits itself, right before each of its parameters is used
                mod.param_waiter = lambda params: self.wait_params(self._buckets_of(params))
                continue
            own = [p for p in mod.parameters(recurse=False) if p.requires_grad]
            if not own:
                continue
            buckets = self._buckets_of(own)
            self._hooks.append(mod.register_forward_pre_hook(lambda m, a, _b=buckets: self.wait_params(_b)))

    def close(self):
        """Detach from the model so that the optimizer, its flat buffers and the model can be
        freed: the post-accumulate-grad and forward pre-hooks are held by the autograd engine's C++
        side (a reference cycle Python's gc cannot see through), and the per-parameter sinks point
        back at this object.  Waits for in-flight side-stream work first."""
        self.wait_params()
        if self._side is not None:
            self._side.synchronize()
        for h in self._hooks:
            h.remove()
        self._hooks = []
        for b in self.buckets:
            for p in b.params:
                for a in ("_dsa_grad_sink", "_dsa_grad_writer", "_dsa_wgen", "_dsa_wt", "_dsa_fresh"):
                    if hasattr(p, a):
                        delattr(p, a)
                p.grad = None
        for mod in self.model.modules():
            if getattr(mod, "param_waiter", None) is not None:
                mod.param_waiter = None
        self.acc32 = None

    def _buckets_of(self, params):
        return [self.buckets[i] for i in sorted({self._bucket_of[p].index for p in params})]

    def state_bytes(self) -> int:
        return sum(t.numel() * 4 for t in self.master + self.exp_avg + self.exp_avg_sq)


def _round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m
