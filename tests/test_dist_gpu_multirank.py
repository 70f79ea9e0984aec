"""ZeRO-1 with two real ranks on the GPU box's one MI355X.

tests/test_dist_gpu.py runs the RCCL calls in a 1-rank communicator, where reduce-scatter and
all-gather are identities.  Here two processes share cuda:0 over gloo (RCCL refuses two ranks on
one device), so the parts that only exist at world > 1 run on the GPU with the HIP kernels: each
rank's gradient buckets are reduce-scattered into a half-size shard, the fused AdamW kernel
updates only that shard on the side stream, and the all-gather reassembles the bf16 weights that
the next forward reads through the prefetch hooks.  Each rank trains on its half of every
micro-batch; the result must equal one process on the whole batch (data-parallel mean == full
batch) to within that single-process run's own run-to-run noise."""

import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu

GRAD_ACCUM = 2
STEPS = 3
PER_RANK = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _data(cfg, world):
    g = torch.Generator().manual_seed(7)
    return [[torch.randint(0, cfg.vocab_size, (PER_RANK * world, 257), generator=g) for _ in range(GRAD_ACCUM)]
            for _ in range(STEPS)]


def _train(steps_batches, dev, rank=0, world=1):
    from dstack_amd.models.llama import CONFIGS, Llama
    from dstack_amd.parallel.zero import ZeroOptimizer

    cfg = CONFIGS["llama-tiny"]
    torch.manual_seed(0)
    with torch.device(dev):
        m = Llama(cfg)
    m.init_weights(seed=1)
    m = m.to(torch.bfloat16)
    opt = ZeroOptimizer(m, lr=1e-3, bucket_numel=(1 << 20) + 4096, overlap_update=True)
    opt.install_prefetch_hooks(m)
    losses = []
    for micro in steps_batches:
        opt.zero_grad()
        for i, b in enumerate(micro):
            tok = b[rank * PER_RANK:(rank + 1) * PER_RANK].to(dev) if world > 1 else b.to(dev)
            opt.sync_grads = i == GRAD_ACCUM - 1
            loss = m.loss(tok[:, :-1], tok[:, 1:])
            (loss / GRAD_ACCUM).backward()
        opt.step()
        losses.append(loss.item())
    opt.wait_params()
    torch.cuda.synchronize()
    return m, opt, losses


def _worker(rank, world, port, out_dir):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dstack_amd.models.llama import CONFIGS
        from dstack_amd.ops import _ext

        _ext.require()
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        m, opt, _ = _train(_data(CONFIGS["llama-tiny"], world), dev, rank, world)
        assert opt.collectives and opt.world == world
        info = {"nbuckets": len(opt.buckets), "shard_numel": sum(b.shard_numel for b in opt.buckets)
                if hasattr(opt.buckets[0], "shard_numel") else None}
        torch.save({"state": {k: v.detach().cpu() for k, v in m.state_dict().items()}, "info": info},
                   os.path.join(out_dir, f"rank{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_zero_two_ranks_on_one_gpu_match_single_process(gpu, tmp_path):
    import torch.multiprocessing as mp

    from dstack_amd.models.llama import CONFIGS

    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, start_method="spawn")
    ranks = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(world)]
    assert ranks[0]["info"]["nbuckets"] > 2
    # the all-gather leaves every rank with identical weights
    for k, v in ranks[0]["state"].items():
        assert torch.equal(v, ranks[1]["state"][k]), k
    data = _data(CONFIGS["llama-tiny"], world)
    single_a, _, la = _train(data, gpu)
    single_b, _, lb = _train(data, gpu)
    # the single-process run's own noise bounds how close the 2-rank result can be
    noise = max((a.float() - b.float()).norm().item() / (b.float().norm().item() + 1e-12)
                for a, b in zip(single_a.state_dict().values(), single_b.state_dict().values()))
    worst = ("", 0.0)
    for k, v in single_a.state_dict().items():
        d = ranks[0]["state"][k].float()
        rel = (d - v.detach().cpu().float()).norm().item() / (v.float().norm().item() + 1e-12)
        if rel > worst[1]:
            worst = (k, rel)
    assert worst[1] < max(1e-2, 10 * noise), (worst, noise)
    # and training moved the weights (the comparison is not between two initial states)
    init = _train([], gpu)[0]
    moved = max((a.float() - b.float()).norm().item() / (b.float().norm().item() + 1e-12)
                for a, b in zip(single_a.state_dict().values(), init.state_dict().values()))
    assert moved > 10 * worst[1], (moved, worst)
