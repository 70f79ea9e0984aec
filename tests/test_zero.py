"""ZeRO-1 optimizer correctness on CPU (fp32): the flat-buffer / direct-wgrad / sharded-AdamW path
must match plain autograd + a reference AdamW, for one process and for world_size 2 over gloo
(the data-parallel average over ranks == one process on the concatenated batch)."""

import copy
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from dstack_amd.models.llama import CONFIGS, Llama
from dstack_amd.ops import reference as ref
from dstack_amd.parallel.zero import ZeroOptimizer

CFG = CONFIGS["llama-tiny"]
SEQ = 32
LR, BETAS, EPS, WD = 1e-3, (0.9, 0.95), 1e-8, 0.1
# Adam normalises tiny gradients to ~sign(g): rank-sum vs single-process summation order can flip
# the sign of near-zero gradient entries, so the cross-process comparison uses a large eps that
# keeps the update linear in g (the reduction itself is what is under test)
EPS_DIST = 1e-2


def _model(seed=0):
    torch.manual_seed(seed)
    m = Llama(CFG)
    m.init_weights(seed=seed)
    return m


def _batches(n, per, seed=1):
    g = torch.Generator().manual_seed(seed)
    return [torch.randint(0, CFG.vocab_size, (per, SEQ + 1), generator=g) for _ in range(n)]


def _reference_steps(model, steps_batches, grad_accum, clip=0.0, norms=None):
    """Plain autograd (ops.linear without a sink) + reference AdamW over full parameters (with
    ``clip``: torch's global-norm clipping first)."""
    params = list(model.parameters())
    master = [p.detach().clone().float() for p in params]
    m = [torch.zeros_like(x) for x in master]
    v = [torch.zeros_like(x) for x in master]
    for step, micro in enumerate(steps_batches, 1):
        for p in params:
            p.grad = None
        for b in micro:
            loss = model.loss(b[:, :-1], b[:, 1:])
            (loss / grad_accum).backward()
        if clip:
            n = torch.nn.utils.clip_grad_norm_(params, clip)
            if norms is not None:
                norms.append(float(n))
        with torch.no_grad():
            for i, p in enumerate(params):
                ref.adamw_(p.data.view(-1), p.grad.reshape(-1), master[i].view(-1), m[i].view(-1), v[i].view(-1),
                           LR, BETAS[0], BETAS[1], EPS, WD, step)
    return model


def _zero_steps(model, steps_batches, grad_accum, bucket_numel=1 << 20, eps=EPS, prefetch=False, clip=0.0,
                norms=None, poison_step=None):
    opt = ZeroOptimizer(model, lr=LR, betas=BETAS, eps=eps, weight_decay=WD, bucket_numel=bucket_numel,
                        clip_grad_norm=clip)
    if prefetch:
        opt.install_prefetch_hooks(model)
    for step, micro in enumerate(steps_batches):
        opt.zero_grad()
        for i, b in enumerate(micro):
            opt.sync_grads = i == len(micro) - 1
            loss = model.loss(b[:, :-1], b[:, 1:])
            if step == poison_step:
                loss = loss * float("inf")  # every gradient becomes inf/NaN
            (loss / grad_accum).backward()
        opt.step()
        if norms is not None:
            norms.append(opt.last_grad_norm)
    opt.wait_params()  # prefetch mode leaves the last all-gather in flight for the next forward
    return model, opt


def _max_diff(a, b):
    return max((x.detach() - y.detach()).abs().max().item() for x, y in zip(a.parameters(), b.parameters()))


def test_zero_single_process_matches_reference():
    base = _model()
    steps = [_batches(2, 2, seed=s) for s in range(3)]
    ref_model = _reference_steps(copy.deepcopy(base), steps, grad_accum=2)
    zero_model, opt = _zero_steps(copy.deepcopy(base), steps, grad_accum=2)
    assert len(opt.buckets) > 1  # exercise several buckets
    assert _max_diff(ref_model, zero_model) < 2e-5
    # GEMM weights took the direct-write path
    assert all(hasattr(p, "_dsa_grad_sink") for p in zero_model.parameters() if p.dim() == 2)


def test_zero_grad_norm_clipping_matches_torch():
    """clip_grad_norm: the norm of the accumulated gradient (computed from the reduced shards) and
    the clipped AdamW step equal torch.nn.utils.clip_grad_norm_ + reference AdamW."""
    base = _model()
    steps = [_batches(2, 2, seed=s) for s in range(3)]
    ref_norms, zero_norms = [], []
    ref_model = _reference_steps(copy.deepcopy(base), steps, grad_accum=2, clip=0.5, norms=ref_norms)
    zero_model, opt = _zero_steps(copy.deepcopy(base), steps, grad_accum=2, clip=0.5, norms=zero_norms)
    assert all(n > 0.5 for n in ref_norms)  # clipping is active on every step
    for a, b in zip(ref_norms, zero_norms):
        assert abs(a - b) <= 1e-4 * a, (ref_norms, zero_norms)
    assert _max_diff(ref_model, zero_model) < 2e-5
    unclipped, _ = _zero_steps(copy.deepcopy(base), steps, grad_accum=2)
    assert _max_diff(unclipped, zero_model) > 1e-4  # and it changed the trajectory


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir, prefetch=False, bucket_numel=1 << 19, clip=0.0, poison=None, nsteps=2):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(max(1, 8 // world))
    base = _model()
    steps = [_batches(2, 2 * world, seed=s) for s in range(nsteps)]
    # each rank takes its slice of every micro-batch
    mine = [[b[rank * 2:(rank + 1) * 2] for b in micro] for micro in steps]
    # poison = (rank, step): that rank's gradient of that step is inf/NaN
    model, opt = _zero_steps(base, mine, grad_accum=2, bucket_numel=bucket_numel, eps=EPS_DIST, prefetch=prefetch,
                             clip=clip, poison_step=poison[1] if poison and poison[0] == rank else None)
    torch.save({k: v.detach() for k, v in model.state_dict().items()}, os.path.join(out_dir, f"rank{rank}.pt"))
    torch.save({"step_count": opt.step_count, "skipped": opt.skipped_steps}, os.path.join(out_dir, f"opt{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("prefetch", [False, True])
def test_zero_gloo_world2_matches_single_process(tmp_path, prefetch):
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path), prefetch), nprocs=world,
                       start_method="spawn")
    states = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(world)]
    # every rank ends with identical parameters (all-gather of the updated shards)
    for k in states[0]:
        assert torch.equal(states[0][k], states[1][k]), k
    # ...equal to one process on the full batch (gradient = mean over ranks)
    base = _model()
    steps = [_batches(2, 2 * world, seed=s) for s in range(2)]
    single, _ = _zero_steps(base, steps, grad_accum=2, eps=EPS_DIST)
    for k, v in single.state_dict().items():
        assert (states[0][k] - v).abs().max().item() < 2e-6, k


def test_zero_gloo_world2_clipping_matches_single_process(tmp_path):
    """The clip norm is all-reduced over ranks' shards: 2 ranks clip exactly like one process."""
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path), True, 1 << 19, 0.5), nprocs=world,
                       start_method="spawn")
    states = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(world)]
    base = _model()
    steps = [_batches(2, 2 * world, seed=s) for s in range(2)]
    single, _ = _zero_steps(base, steps, grad_accum=2, eps=EPS_DIST, clip=0.5)
    for k, v in single.state_dict().items():
        assert (states[0][k] - v).abs().max().item() < 2e-6, k


def test_zero_gloo_world2_skips_nonfinite_step(tmp_path):
    """Clipping on, one rank's gradient of step 2 is inf/NaN: the all-reduced norm is non-finite on
    every rank, so every rank skips that AdamW update (master weights and moments stay clean, the
    step counter does not advance) -- the result equals one process that never saw step 2."""
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path), True, 1 << 19, 0.5, (1, 1), 3),
                       nprocs=world, start_method="spawn")
    states = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(world)]
    for r in range(world):
        o = torch.load(tmp_path / f"opt{r}.pt", weights_only=True)
        assert o == {"step_count": 2, "skipped": 1}, o
    for k in states[0]:
        assert torch.isfinite(states[0][k]).all() and torch.equal(states[0][k], states[1][k]), k
    base = _model()
    steps = [_batches(2, 2 * world, seed=s) for s in (0, 2)]
    single, _ = _zero_steps(base, steps, grad_accum=2, eps=EPS_DIST, clip=0.5)
    for k, v in single.state_dict().items():
        assert (states[0][k] - v).abs().max().item() < 2e-6, k


@pytest.mark.slow
@pytest.mark.parametrize("world", [4, 8])
def test_zero_gloo_many_ranks_uneven_buckets(tmp_path, world):
    """4 and 8 ranks with a bucket size that is no multiple of anything: buckets hold different
    numbers of parameters, every bucket is padded to world*64 and each rank's shard boundary falls
    inside a parameter; all ranks must still end identical and equal the single process."""
    bucket = (1 << 18) + 12345
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path), True, bucket), nprocs=world,
                       start_method="spawn")
    states = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(world)]
    for r in range(1, world):
        for k in states[0]:
            assert torch.equal(states[0][k], states[r][k]), (r, k)
    base = _model()
    steps = [_batches(2, 2 * world, seed=s) for s in range(2)]
    single, opt = _zero_steps(base, steps, grad_accum=2, eps=EPS_DIST, bucket_numel=bucket)
    assert len(opt.buckets) > 2 and len({len(b.params) for b in opt.buckets}) > 1
    for k, v in single.state_dict().items():
        assert (states[0][k] - v).abs().max().item() < 5e-6, k


@pytest.mark.parametrize("bucket_numel", [1 << 16, 1 << 30])
def test_zero_bucket_layout_is_padded_and_reverse_ordered(bucket_numel):
    model = _model()
    opt = ZeroOptimizer(model, bucket_numel=bucket_numel)
    for b in opt.buckets:
        assert b.numel % 64 == 0
    first = opt.buckets[0].params[0]
    assert first is list(model.parameters())[-1]  # last-registered param first (backward order)
    assert opt.total_numel >= sum(p.numel() for p in model.parameters())


def test_bucket_completes_once_after_all_its_gradients():
    """Every bucket is counted down exactly once per parameter in the synchronising backward and
    completes only after all of its parameters' gradients were produced -- also for parameters whose
    gradient a kernel writes directly (PyTorch still runs their post-accumulate-grad hook, with an
    undefined gradient, after the op already reported them)."""
    model = _model()
    opt = ZeroOptimizer(model, lr=LR, bucket_numel=1 << 18)
    assert len(opt.buckets) > 2
    seen, completions = set(), []
    orig = ZeroOptimizer._on_grad_ready

    def on_ready(p):
        if opt.sync_grads and p.grad is not None:
            seen.add(p)
        before = opt._bucket_of[p].pending
        orig(opt, p)
        b = opt._bucket_of[p]
        if before == 1 and b.pending == 0:
            completions.append((b.index, {id(q) for q in seen}))

    opt._on_grad_ready = on_ready
    opt._hooks_on = True
    for p in model.parameters():
        p.register_post_accumulate_grad_hook(on_ready)
    batches = _batches(2, 2, seed=3)
    opt.zero_grad()
    for i, b in enumerate(batches):
        opt.sync_grads = i == len(batches) - 1
        model.loss(b[:, :-1], b[:, 1:]).backward()
    assert sorted(i for i, _ in completions) == list(range(len(opt.buckets)))  # each exactly once
    for i, seen_ids in completions:
        assert {id(p) for p in opt.buckets[i].params} <= seen_ids, f"bucket {i} completed early"
    assert all(b.pending == 0 for b in opt.buckets)


def test_mm_into_f32_fallback_modes():
    """The fp32 gradient-accumulator contract on the torch fallback (the HIP path is
    test_ops_gpu.py::test_gemm_km_f32_modes_and_strides): 0 stores, 1 adds, 2 writes bf16(acc + a@b)."""
    import torch

    from dstack_amd.ops import functional as F

    g = torch.Generator().manual_seed(0)
    a = torch.randn(64, 32, generator=g).bfloat16()
    b = torch.randn(32, 48, generator=g).bfloat16()
    acc = torch.zeros(64, 48)
    out = torch.zeros(64, 48, dtype=torch.bfloat16)
    prod = a.float() @ b.float()
    F.mm_into_f32(a, b, acc, out, 0)
    assert torch.allclose(acc, prod) and out.abs().max() == 0
    F.mm_into_f32(a, b, acc, out, 1)
    assert torch.allclose(acc, 2 * prod)
    F.mm_into_f32(a, b, acc, out, 2)
    assert torch.equal(out, (2 * prod + prod).bfloat16())


def test_zero_grad_accum_fp32_only_for_bf16_params(monkeypatch):
    import torch
    import torch.nn as nn

    from dstack_amd.parallel.zero import ZeroOptimizer

    monkeypatch.setenv("DSTACK_AMD_GRAD_ACCUM_FP32", "1")
    m32 = nn.Linear(64, 64, bias=False)
    assert not ZeroOptimizer(m32).grad_accum_fp32  # fp32 params: nothing to gain
    m16 = nn.Linear(64, 64, bias=False).to(torch.bfloat16)
    opt = ZeroOptimizer(m16)
    assert opt.grad_accum_fp32 and opt.acc32 is None  # allocated at the first non-final micro-batch
    w = next(m16.parameters())
    assert opt._acc32_view(w).shape == w.shape and opt.acc32.dtype == torch.float32


def test_trainer_close_frees_model_and_optimizer(monkeypatch):
    """With collectives or optimizer-in-backward, ZeroOptimizer's autograd hooks are held from the
    C++ side of the engine: a dropped trainer stays alive (on a GPU: every byte of the model and its
    optimizer, which is what made the 1-GPU cold start under a launcher OOM).  Trainer.close()
    detaches it so that it is freed."""
    import gc
    import weakref

    import torch.distributed as dist

    from dstack_amd.workloads.train_llama import run

    monkeypatch.setenv("DSTACK_AMD_ZERO_FORCE_COLLECTIVES", "1")  # a 1-rank gloo group: hooks on
    env, tr, _ = run("llama-tiny", 64, 1, 1, 0, log_every=0, grad_accum=2)
    try:
        assert tr.opt._hooks
        wm, wo = weakref.ref(tr.model), weakref.ref(tr.opt)
        tr.close()
        del tr
        gc.collect()
        assert wm() is None and wo() is None
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_trainer_picks_gemm_grid_for_the_communicating_micro_batch(monkeypatch):
    """DSTACK_AMD_GEMM_GRID_LAST: auto = the per-tile GEMM grid for the last micro-batch only when
    the optimizer runs collectives (a persistent grid waits for CUs held by RCCL's workgroups);
    tile / persistent force it; the setting is restored after the backward."""
    from dstack_amd.workloads import train_llama
    from dstack_amd.workloads.train_llama import Trainer

    calls = []
    monkeypatch.setattr(train_llama, "_gemm_grid", lambda m: calls.append(m))
    for env, want in (("auto", None), ("tile", 0), ("persistent", 1)):
        monkeypatch.setenv("DSTACK_AMD_GEMM_GRID_LAST", env)
        tr = Trainer("llama-tiny", 32, 2, torch.device("cpu"), grad_accum=3)
        assert tr._last_grid == want, env
        tr.close()
    # on CPU no grid is ever set (the switch is for the GPU GEMM); with collectives it would be
    monkeypatch.setenv("DSTACK_AMD_GEMM_GRID_LAST", "tile")
    tr = Trainer("llama-tiny", 32, 2, torch.device("cpu"), grad_accum=3)
    tr.step()
    assert calls == []
    tr.device = torch.device("cuda")  # exercise the switch logic without a GPU: only the grid calls
    monkeypatch.setattr(tr.model, "loss", lambda tok, tgt: (tr.model.embed.float().sum() * 0.0) + 1.0)
    tr.opt.step = lambda: None
    tr.step()
    assert calls == [0, -1]
    tr.close()
