"""Llama-3 pre-training step on MI355X: one process per GPU, ZeRO-1 DP over RCCL/xGMI.

This is the workload behind the headline benchmark ("tokens/sec of an 8-GPU Llama-3-8B task via
dstack apply", BASELINE.json). It is launched either directly by ``bench.py`` or by a
``type: task`` run (``examples/llama3-8b-train.dstack.yml``) whose runner exports the rendezvous
env (``DSTACK_MASTER_NODE_IP``, ``DSTACK_NODE_RANK``, …, plus ``MASTER_ADDR``/``RANK``/…).

Data is synthetic (uniform random token ids) and weights are random-init: there is no network.
"""

from __future__ import annotations

import time

_T_IMPORT = time.time()  # before torch: the stage split below starts here

import argparse  # noqa: E402
import datetime  # noqa: E402
import json  # noqa: E402
import os  # noqa: E402
import shutil  # noqa: E402
from dataclasses import dataclass  # noqa: E402

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

_T_TORCH = time.time()


def process_start_time() -> float | None:
    """Wall-clock time this process was exec'd (Linux /proc), so a job's stage split can start
    from the interpreter launch rather than from the first line of Python.  Computed against
    /proc/uptime (10 ms resolution), not /proc/stat's btime, which is whole seconds."""
    try:
        now = time.time()
        with open("/proc/uptime") as f:
            uptime = float(f.read().split()[0])
        with open("/proc/self/stat") as f:
            fields = f.read().rsplit(")", 1)[1].split()
        start_s = int(fields[19]) / os.sysconf("SC_CLK_TCK")  # field 22 (starttime), after the ")" of comm
        return now - (uptime - start_s)
    except (OSError, ValueError, IndexError):
        return None

from dstack_amd.models.llama import CONFIGS, Llama
from dstack_amd.parallel.zero import ZeroOptimizer
from dstack_amd.workloads.data import SyntheticLM


@dataclass
class DistEnv:
    rank: int = 0
    world: int = 1
    local_rank: int = 0

    @property
    def distributed(self) -> bool:
        return self.world > 1


def init_distributed(backend: str | None = None) -> DistEnv:
    """Reads torchrun's env (or the dstack runner's RCCL rendezvous env) and joins the group."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    env = DistEnv(rank, world, local_rank)
    if torch.cuda.is_available():
        torch.cuda.set_device(local_rank)
    # DSTACK_AMD_ZERO_FORCE_COLLECTIVES=1 at world 1: a 1-rank RCCL group, so the ZeRO-1
    # reduce-scatter / all-gather path of a multi-GPU job runs on a single GPU (validation)
    force = os.environ.get("DSTACK_AMD_ZERO_FORCE_COLLECTIVES", "0") not in ("0", "", "false")
    if (world > 1 or force) and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"  # "nccl" is RCCL on ROCm
        # an explicit collective timeout (torch's default is 10 min): a slow first step on a cold
        # node, a checkpoint save on a shared volume or rank 0 writing results must not trip the
        # watchdog, while a truly hung peer still fails the job instead of holding the GPUs forever
        kwargs = {"timeout": datetime.timedelta(seconds=float(os.environ.get("DSTACK_AMD_PG_TIMEOUT_S", "1800")))}
        if backend == "nccl":
            kwargs["device_id"] = torch.device("cuda", local_rank)
        if world == 1 and "MASTER_ADDR" not in os.environ:
            kwargs.update(store=dist.HashStore(), rank=0, world_size=1)
        dist.init_process_group(backend=backend, **kwargs)
    return env


def _gemm_grid(mode: int) -> None:
    """Set the in-tree GEMM's grid form (-1 default, 0 per tile, 1 persistent) if the extension is
    loaded (host-side setting, read at each launch)."""
    from dstack_amd.ops import _ext

    if _ext.available():
        _ext.require().gemm_nt_set_grid(mode)


class Trainer:
    def __init__(self, model_name: str, seq_len: int, micro_batch: int, device, lr: float = 3e-4,
                 seed: int = 0, bucket_numel: int = 256 * 1024 * 1024, grad_accum: int = 1,
                 lr_warmup: int = 0, lr_decay_steps: int = 0, min_lr_ratio: float = 0.1, data: str = "synthetic-lm",
                 data_rows: int = 4, clip_grad_norm: float = 0.0, lm_head_std: float | None = None):
        self.cfg = CONFIGS[model_name]
        # LR schedule: linear warmup over ``lr_warmup`` optimizer steps, then constant, or cosine
        # decay to ``min_lr_ratio * lr`` at step ``lr_decay_steps`` when that is set.  A random-init
        # model hit with the full Adam step at step 1 overshoots (the loss climbs back above
        # ln(vocab) within a few steps); the warmup is what keeps it descending.
        self.base_lr = lr
        self.lr_warmup = lr_warmup
        self.lr_decay_steps = lr_decay_steps
        self.min_lr_ratio = min_lr_ratio
        self.seq_len = seq_len
        self.micro_batch = micro_batch
        self.grad_accum = grad_accum
        self.device = device
        dtype = torch.bfloat16 if device.type == "cuda" else torch.float32
        # parameters allocated in their final dtype: constructing in fp32 and converting allocated
        # and copied twice the model (27-66 ms of the start-up, profiles/init_split_r9n.txt)
        prev = torch.get_default_dtype()
        torch.set_default_dtype(dtype)
        try:
            with torch.device(device):
                model = Llama(self.cfg)
        finally:
            torch.set_default_dtype(prev)
        model.to(dtype)  # (a no-op unless a submodule pins its own dtype)
        model.init_weights(seed=seed, lm_head_std=lm_head_std)
        self.model = model
        self.opt = ZeroOptimizer(model, lr=lr, bucket_numel=bucket_numel, clip_grad_norm=clip_grad_norm)
        self.opt.install_prefetch_hooks(model)
        rank = dist.get_rank() if dist.is_initialized() else 0
        # data: "synthetic-lm" = a fresh structured batch every micro-step (workloads/data.py, the
        # bench's data); "tokens:<glob>" = token shards through the native loader (workloads/
        # tokens.py); "fixed" = ``data_rows`` uniform-random rows cycled (a memorisation check)
        self.data_kind = data
        self.stream = None
        if data == "synthetic-lm":
            self.stream = SyntheticLM(self.cfg.vocab_size, seq_len, micro_batch, device, seed=1234 + rank)
        elif data.startswith("tokens:"):
            from dstack_amd.workloads.tokens import TokenShards

            world = dist.get_world_size() if dist.is_initialized() else 1
            self.stream = TokenShards(data.split(":", 1)[1], seq_len, micro_batch, device, seed=seed, rank=rank,
                                      world=world, vocab_size=self.cfg.vocab_size)
        elif data == "fixed":
            g = torch.Generator(device=device).manual_seed(1234 + rank)
            n = micro_batch * (seq_len + 1)
            self.data = torch.randint(0, self.cfg.vocab_size, (data_rows, n), device=device, generator=g)
        else:
            raise ValueError(f"unknown data kind {data!r}")
        self._i = 0
        self.trace_next_step = False
        self.last_split = None
        # grid form of the in-tree GEMM for the last micro-batch, whose backward runs beside the
        # reduce-scatter / AdamW / all-gather (DSTACK_AMD_GEMM_GRID_LAST = tile | persistent | auto):
        # auto = one workgroup per tile when there are collectives (a persistent grid waits for the
        # CUs the collective's workgroups hold), the default form otherwise
        mode = os.environ.get("DSTACK_AMD_GEMM_GRID_LAST", "auto").lower()
        self._last_grid = {"tile": 0, "persistent": 1}.get(mode)
        if mode == "auto":
            self._last_grid = 0 if self.opt.collectives else None

    def batch(self):
        if self.stream is not None:
            out = self.stream.batch(self._i)
        else:
            row = self.data[self._i % self.data.shape[0]].view(self.micro_batch, self.seq_len + 1)
            out = row[:, :-1], row[:, 1:]
        self._i += 1
        return out

    def close(self):
        """Release the GPU memory of the model and optimizer (see ZeroOptimizer.close): after
        this, dropping the trainer frees its tensors and ``torch.cuda.empty_cache`` returns them."""
        self.opt.close()
        self.stream = None
        self.data = None

    def lr_at(self, step: int) -> float:
        """Learning rate of optimizer step ``step`` (1-based)."""
        import math

        if self.lr_warmup and step <= self.lr_warmup:
            return self.base_lr * step / self.lr_warmup
        if self.lr_decay_steps and self.lr_decay_steps > self.lr_warmup:
            t = min(1.0, (step - self.lr_warmup) / (self.lr_decay_steps - self.lr_warmup))
            lo = self.min_lr_ratio * self.base_lr
            return lo + 0.5 * (self.base_lr - lo) * (1 + math.cos(math.pi * t))
        return self.base_lr

    def step(self) -> torch.Tensor:
        """One optimizer step = ``grad_accum`` micro-batches; the gradient reduce-scatter is armed
        only for the last micro-batch so it overlaps that backward."""
        # set before backward: with optimizer-in-backward AdamW runs per bucket during it
        self.opt.lr = self.lr_at(self.opt.step_count + 1)
        trace = self.trace_next_step  # diagnostic: synchronised split of this step (first_step_split)
        self.trace_next_step = False
        split = {"batch": 0.0, "fwd": 0.0, "bwd": 0.0, "opt": 0.0}

        def mark(k, t0):
            if trace:
                if self.device.type == "cuda":
                    torch.cuda.synchronize(self.device)
                split[k] += time.time() - t0
            return time.time()

        self.opt.zero_grad()
        total = None
        grid = _gemm_grid if self._last_grid is not None and self.device.type == "cuda" else None
        for i in range(self.grad_accum):
            t0 = time.time()
            tokens, targets = self.batch()
            t0 = mark("batch", t0)
            self.opt.sync_grads = i == self.grad_accum - 1
            loss = self.model.loss(tokens, targets)
            t0 = mark("fwd", t0)
            if grid is not None and self.opt.sync_grads:
                grid(self._last_grid)
            try:
                (loss / self.grad_accum if self.grad_accum > 1 else loss).backward()
            finally:
                if grid is not None and self.opt.sync_grads:
                    grid(-1)
            mark("bwd", t0)
            total = loss.detach() if total is None else total + loss.detach()
        t0 = time.time()
        self.opt.step()
        if trace:
            mark("opt", t0)
            self.last_split = {k: round(v, 4) for k, v in split.items()}
        return total / self.grad_accum

    # ---- checkpoints: safetensors, one optimizer shard per rank, written to a directory that is
    # usually a dstack volume (the reference leaves checkpointing to the job).
    #
    # Layout: ``<dir>/step-<N>/`` holds ``optim-rank<r>-of-<w>.safetensors`` (every rank),
    # ``params.safetensors`` and ``meta.json`` (local rank 0 of every node, so node-local volumes
    # such as ``${{ dstack.node_rank }}`` ones work too); ``<dir>/latest`` names the newest complete
    # step directory and is replaced atomically only after every rank has finished writing, so a
    # save cut short is never loaded.  Older step directories beyond ``keep`` are pruned. ----
    def save_checkpoint(self, path: str, keep: int = 2):
        from safetensors.torch import save_file

        rank, world, local_rank = _ranks()
        # the all-gathers of the last step may still be in flight (prefetch hooks defer the wait
        # to the next forward): the saved bf16 params must be the fully gathered buffer
        self.opt.wait_params()
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        step = self.opt.step_count
        sdir = os.path.join(path, f"step-{step:08d}")
        os.makedirs(sdir, exist_ok=True)
        shard = {k: v.detach().cpu().contiguous() for k, v in self.opt.shard_state().items()}
        _atomic_save(save_file, shard, os.path.join(sdir, f"optim-rank{rank:05d}-of-{world:05d}.safetensors"), rank)
        if local_rank == 0:
            _atomic_save(save_file, {"flat_param": self.opt.flat_param.detach().cpu()},
                         os.path.join(sdir, "params.safetensors"), rank)
            _atomic_write(os.path.join(sdir, "meta.json"),
                          json.dumps({"step": step, "world": world, "data_index": self._i,
                                      "total_numel": self.opt.total_numel, "model": self.cfg.name}), rank)
        if dist.is_initialized():
            dist.barrier()  # every shard of this step is on disk before ``latest`` points at it
        if local_rank == 0:
            _atomic_write(os.path.join(path, "latest"), os.path.basename(sdir), rank)
            olds = sorted(d for d in os.listdir(path) if d.startswith("step-") and d != os.path.basename(sdir))
            for d in olds[: max(0, len(olds) - (keep - 1))]:
                shutil.rmtree(os.path.join(path, d), ignore_errors=True)
        if dist.is_initialized():
            dist.barrier()

    @staticmethod
    def checkpoint_step(path: str | None) -> int | None:
        """The step of the newest complete checkpoint under ``path`` (None if there is none)."""
        if not path:
            return None
        try:
            with open(os.path.join(path, "latest")) as f:
                name = f.read().strip()
            with open(os.path.join(path, name, "meta.json")) as f:
                return int(json.load(f)["step"])
        except (OSError, ValueError, KeyError):
            return None

    def resume_step(self, path: str | None) -> int | None:
        """Collective: rank 0 decides whether to resume (and from which step) and broadcasts it;
        every rank then checks that it can read that step's files, so a directory that is not
        shared across nodes (or a node that lost its volume) fails on every rank at once instead
        of leaving some ranks resumed and others hanging in a collective."""
        step = self.checkpoint_step(path)
        if not dist.is_initialized():
            return step
        dev = self.device if self._backend_is_nccl() else torch.device("cpu")
        t = torch.tensor([-1 if step is None else step], dtype=torch.int64, device=dev)
        dist.broadcast(t, src=0)
        step = None if t.item() < 0 else int(t.item())
        if step is None:
            return None
        rank, world, _ = _ranks()
        sdir = os.path.join(path, f"step-{step:08d}")
        ok = all(os.path.exists(os.path.join(sdir, f)) for f in
                 ("meta.json", "params.safetensors", f"optim-rank{rank:05d}-of-{world:05d}.safetensors"))
        flag = torch.tensor([0 if ok else 1], dtype=torch.int64, device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.SUM)
        if flag.item():
            raise RuntimeError(f"{int(flag.item())} rank(s) cannot read checkpoint step {step} under {path}: "
                               "--checkpoint-dir must be shared by the ranks of a node (one volume per node, "
                               "or one network volume for all nodes)")
        return step

    def _backend_is_nccl(self) -> bool:
        return dist.is_initialized() and dist.get_backend() == "nccl"

    def load_checkpoint(self, path: str, step: int | None = None) -> int:
        """Restore a checkpoint written by :meth:`save_checkpoint`; returns its step."""
        from safetensors.torch import load_file

        rank, world, _ = _ranks()
        if step is None:
            step = self.checkpoint_step(path)
            if step is None:
                raise FileNotFoundError(f"no complete checkpoint under {path}")
        sdir = os.path.join(path, f"step-{step:08d}")
        with open(os.path.join(sdir, "meta.json")) as f:
            meta = json.load(f)
        if meta["world"] != world:
            raise ValueError(f"checkpoint written by {meta['world']} ranks, this job has {world}")
        params = load_file(os.path.join(sdir, "params.safetensors"))["flat_param"]
        shard = load_file(os.path.join(sdir, f"optim-rank{rank:05d}-of-{world:05d}.safetensors"))
        self.opt.load_state(params, shard, meta["step"])
        self._i = meta["data_index"]
        return meta["step"]

    @property
    def tokens_per_step(self) -> int:
        return self.micro_batch * self.seq_len * self.grad_accum


def _ranks() -> tuple[int, int, int]:
    if dist.is_initialized():
        return dist.get_rank(), dist.get_world_size(), int(os.environ.get("LOCAL_RANK", dist.get_rank()))
    return 0, 1, 0


def _atomic_save(save_file, tensors: dict, dst: str, rank: int = 0):
    tmp = f"{dst}.tmp{rank}"  # per-writer temp name: ranks of different nodes may share a volume
    save_file(tensors, tmp)
    os.replace(tmp, dst)


def _atomic_write(dst: str, text: str, rank: int = 0):
    tmp = f"{dst}.tmp{rank}"
    with open(tmp, "w") as f:
        f.write(text)
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, dst)


def _sync(env: DistEnv):
    if env.distributed:
        dist.barrier()
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def run(model: str, seq_len: int, micro_batch: int, steps: int, warmup: int, log_every: int = 1,
        grad_accum: int = 1, checkpoint_dir: str | None = None, save_every: int = 0, lr: float = 3e-4,
        lr_warmup: int = 300, lr_decay_steps: int = 0, clip_grad_norm: float = 0.0, data: str = "synthetic-lm"):
    # wall-clock stamps of the task's start-up (rank 0 prints them after the first optimizer step):
    # process exec -> imports -> rendezvous -> HIP extension -> GEMM selections -> model -> step 1
    stages = {"proc_start": process_start_time(), "import_start": _T_IMPORT, "torch_imported": _T_TORCH}
    env = init_distributed()
    stages["dist_ready"] = time.time()
    device = torch.device("cuda", env.local_rank) if torch.cuda.is_available() else torch.device("cpu")
    if device.type == "cuda":
        from dstack_amd.ops import _ext

        _ext.require()  # the HIP extension (.so) is mapped here, not at the first kernel
    stages["extension_loaded"] = time.time()
    from dstack_amd.ops import gemm_tuning

    gemm_mode = gemm_tuning.setup(device_index=env.local_rank if device.type == "cuda" else 0)
    stages["gemm_tuning_loaded"] = time.time()
    # the library GEMMs' first-call set-up runs beside the model's initialisation
    warm = gemm_tuning.prewarm(gemm_tuning.llama_shapes(CONFIGS[model], micro_batch * seq_len), device) \
        if model in CONFIGS else None
    t0 = time.time()
    tr = Trainer(model, seq_len, micro_batch, device, grad_accum=grad_accum, lr=lr, lr_warmup=lr_warmup,
                 lr_decay_steps=lr_decay_steps, clip_grad_norm=clip_grad_norm, data=data)
    # DSTACK_AMD_PREWARM_JOIN=late: the first step starts while the prewarm thread still loads the
    # later (backward) GEMMs' kernels; joined after the first step instead of before it
    late_join = os.environ.get("DSTACK_AMD_PREWARM_JOIN", "early") == "late"
    if warm is not None and not late_join:
        warm.join()
    stages["model_ready"] = time.time()
    if env.rank == 0:
        print(f"[train] model={model} params={tr.cfg.num_params()/1e9:.2f}B world={env.world} "
              f"init={time.time()-t0:.1f}s gemm_tuning={gemm_mode}", flush=True)
    if checkpoint_dir:
        # --steps is the job's total number of optimizer steps: a resumed job (retry after an
        # interruption) trains only the remainder and skips the warmup; saves fall on global
        # step numbers (opt.step_count % save_every == 0)
        resumed = tr.resume_step(checkpoint_dir)
        if resumed is not None:
            tr.load_checkpoint(checkpoint_dir, resumed)
            warmup = 0
            if env.rank == 0:
                print(f"[train] resumed from {checkpoint_dir} at step {resumed}", flush=True)
        warmup = max(0, min(warmup, steps - tr.opt.step_count))
        steps = max(0, steps - tr.opt.step_count - warmup)

    def _maybe_save():
        if checkpoint_dir and save_every and tr.opt.step_count % save_every == 0:
            tr.save_checkpoint(checkpoint_dir)

    # DSTACK_AMD_FIRST_STEP_SPLIT=1: the first step synchronises around its batches / forwards /
    # backwards / optimizer step and reports the sums (diagnostic: it slows that step slightly)
    tr.trace_next_step = os.environ.get("DSTACK_AMD_FIRST_STEP_SPLIT", "0") == "1"

    def _first_step_done():
        if warm is not None and late_join:
            warm.join()
        if "first_step_done" not in stages:
            stages["first_step_done"] = time.time()
            if tr.last_split is not None:
                stages["first_step_split"] = tr.last_split
            if env.rank == 0:
                print("[train] stages " + json.dumps(stages), flush=True)

    warm_losses = []
    for i in range(warmup):
        loss = tr.step()
        warm_losses.append(loss.item())
        _first_step_done()
        if env.rank == 0:
            print(f"[train] warmup {i} loss={loss.item():.4f}", flush=True)
        _maybe_save()
    _sync(env)
    t_start = time.perf_counter()
    losses = []
    for i in range(steps):
        losses.append(tr.step())
        if i == 0 and "first_step_done" not in stages:
            losses[-1].item()  # (only when there was no warmup: the stamp needs the step finished)
            _first_step_done()
        if log_every and env.rank == 0 and (i + 1) % log_every == 0:
            print(f"[train] step {tr.opt.step_count} loss={losses[-1].item():.4f}", flush=True)
        _maybe_save()  # inside the timed loop only when asked for
    _sync(env)
    elapsed = time.perf_counter() - t_start
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    if env.distributed:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = t.item()
    tok_s = tr.tokens_per_step * env.world * steps / elapsed if steps else 0.0
    result = {
        "tokens_per_s": tok_s,
        "ms_per_step": elapsed / steps * 1e3 if steps else 0.0,
        "world": env.world,
        "flops_per_token": tr.cfg.flops_per_token(seq_len),
        "final_loss": losses[-1].item() if losses else None,
        "max_mem_gb": torch.cuda.max_memory_allocated(device) / 2**30 if device.type == "cuda" else None,
    }
    result["tflops_per_gpu"] = tok_s / env.world * result["flops_per_token"] / 1e12
    result["losses"] = [round(x.item(), 4) for x in losses]  # read after the timed region
    result["warmup_losses"] = [round(x, 4) for x in warm_losses]
    if isinstance(tr.stream, SyntheticLM):
        result["loss_floor"] = round(tr.stream.loss_floor, 4)
        result["unigram_entropy"] = round(tr.stream.unigram_entropy, 4)
    result["gemm_tuning"] = gemm_mode
    result["stages"] = stages
    if env.rank == 0:
        print("[train] result " + json.dumps(result), flush=True)
    return env, tr, result


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--seq-len", type=int, default=8192)
    ap.add_argument("--micro-batch", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10,
                    help="timed steps; with --checkpoint-dir the job's total optimizer steps (warmup included)")
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--grad-accum", type=int, default=1)
    ap.add_argument("--checkpoint-dir", default=None,
                    help="resume from here if it holds a checkpoint (e.g. a dstack volume mount)")
    ap.add_argument("--save-every", type=int, default=0,
                    help="save a checkpoint whenever the optimizer step count is a multiple of N")
    ap.add_argument("--lr", type=float, default=3e-4)
    # 300 warmup steps (1e-6 per step at lr 3e-4): on the bench stream the loss falls 12.56 -> 8.4
    # in 30 steps; 100 steps gives a noisier curve with excursions back to ~12-14, and global-norm
    # clipping at 1.0 does not tame them (profiles/lr_sweep_*_r4k.log, loss_{no,}clip_r4n.log)
    ap.add_argument("--lr-warmup", type=int, default=300, help="linear LR warmup (optimizer steps)")
    ap.add_argument("--lr-decay-steps", type=int, default=0, help="cosine decay to 0.1*lr at this step (0: constant)")
    ap.add_argument("--clip-grad-norm", type=float, default=0.0, help="global gradient-norm clipping (0: off)")
    ap.add_argument("--data", default="synthetic-lm",
                    help="synthetic-lm (structured synthetic stream) or tokens:<glob>[,<glob>] (token shards)")
    args = ap.parse_args(argv)
    env, tr, _ = run(args.model, args.seq_len, args.micro_batch, args.steps, args.warmup,
                     grad_accum=args.grad_accum, checkpoint_dir=args.checkpoint_dir, save_every=args.save_every,
                     lr=args.lr, lr_warmup=args.lr_warmup, lr_decay_steps=args.lr_decay_steps,
                     clip_grad_norm=args.clip_grad_norm, data=args.data)
    if args.checkpoint_dir and not (args.save_every and tr.opt.step_count % args.save_every == 0):
        tr.save_checkpoint(args.checkpoint_dir)  # (a step that is a multiple of save_every is saved)
    if env.distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
