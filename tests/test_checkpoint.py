"""Training checkpoints (safetensors; one AdamW shard per rank): a job resumed from a checkpoint
continues with exactly the losses of the uninterrupted job, single process and 2-rank gloo.
The reference leaves ML checkpointing to the job; this is the bundled workload's."""

import json
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from dstack_amd.workloads.train_llama import Trainer


def _trainer(device="cpu"):
    return Trainer("llama-tiny", seq_len=32 if device == "cpu" else 256, micro_batch=2, device=torch.device(device),
                   grad_accum=2, bucket_numel=64 * 1024)


def _losses(tr, n):
    return [tr.step().item() for _ in range(n)]


def _resume_matches(path, device="cpu"):
    a = _trainer(device)
    _losses(a, 2)
    a.save_checkpoint(path)
    expect = _losses(a, 3)
    b = _trainer(device)
    with torch.no_grad():
        b.opt.flat_param.mul_(0.5)  # make sure the load really overwrites
    assert b.load_checkpoint(path) == 2
    return expect, _losses(b, 3)


def test_resume_continues_identically(tmp_path):
    expect, got = _resume_matches(str(tmp_path / "ckpt"))
    assert got == expect
    assert (tmp_path / "ckpt" / "latest").read_text() == "step-00000002"
    sdir = tmp_path / "ckpt" / "step-00000002"
    meta = json.loads((sdir / "meta.json").read_text())
    assert meta["step"] == 2 and meta["world"] == 1
    assert sorted(os.listdir(sdir)) == ["meta.json", "optim-rank00000-of-00001.safetensors", "params.safetensors"]


def test_incomplete_save_is_never_loaded(tmp_path):
    """A save interrupted before ``latest`` moved leaves the previous checkpoint in force; old
    step directories beyond ``keep`` are pruned."""
    a = _trainer()
    _losses(a, 1)
    a.save_checkpoint(str(tmp_path))
    _losses(a, 1)
    a.save_checkpoint(str(tmp_path))
    _losses(a, 1)
    a.save_checkpoint(str(tmp_path))
    assert sorted(d for d in os.listdir(tmp_path) if d.startswith("step-")) == ["step-00000002", "step-00000003"]
    (tmp_path / "step-00000004").mkdir()  # a save cut short: some shards, no pointer update
    (tmp_path / "step-00000004" / "optim-rank00000-of-00001.safetensors").write_bytes(b"partial")
    assert Trainer.checkpoint_step(str(tmp_path)) == 3
    assert _trainer().load_checkpoint(str(tmp_path)) == 3


def test_world_size_mismatch_rejected(tmp_path):
    a = _trainer()
    _losses(a, 1)
    a.save_checkpoint(str(tmp_path))
    mpath = tmp_path / "step-00000001" / "meta.json"
    meta = json.loads(mpath.read_text())
    meta["world"] = 8
    mpath.write_text(json.dumps(meta))
    with pytest.raises(ValueError, match="8 ranks"):
        _trainer().load_checkpoint(str(tmp_path))


def _worker(rank, world, port, path, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(max(1, 8 // world))
    try:
        expect, got = _resume_matches(path)
        q.put((rank, expect, got))
    finally:
        dist.destroy_process_group()


def _gathered_worker(rank, world, port, path, q):
    """The saved bf16 buffer must be the fully all-gathered one: with prefetch hooks the step
    returns before the all-gathers finish, and the save has to wait for them itself."""
    from safetensors.torch import load_file

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(max(1, 8 // world))
    try:
        tr = _trainer()
        assert tr.opt._prefetch
        _losses(tr, 2)
        tr.save_checkpoint(path)
        saved = load_file(os.path.join(path, "step-00000002", "params.safetensors"))["flat_param"]
        tr.opt.wait_params()
        ok = torch.equal(saved, tr.opt.flat_param.detach().cpu())
        # each rank's own shard must equal its fp32 master rounded to bf16, i.e. the update landed
        for b, master in zip(tr.opt.buckets, tr.opt.master):
            for r in range(world):
                s, n = b.shard_range(r, world)
                ok = ok and not torch.equal(saved[s:s + n], torch.zeros(n, dtype=saved.dtype))
            s, n = b.shard_range(rank, world)
            ok = ok and torch.equal(saved[s:s + n], master.to(saved.dtype))
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


def _resume_target_worker(rank, world, port, path, q):
    """--steps is a global target: a job resumed at step 2 of 4 trains 2 more steps, no warmup."""
    from dstack_amd.workloads import train_llama

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(max(1, 8 // world))
    try:
        _, tr1, _ = train_llama.run("llama-tiny", 32, 2, steps=2, warmup=1, log_every=0,
                                    checkpoint_dir=path, save_every=1)
        first = tr1.opt.step_count
        _, tr2, _ = train_llama.run("llama-tiny", 32, 2, steps=4, warmup=1, log_every=0,
                                    checkpoint_dir=path, save_every=2)
        q.put((rank, first, tr2.opt.step_count, train_llama.Trainer.checkpoint_step(path)))
    finally:
        dist.destroy_process_group()


def _spawn(target, path, world=2):
    from dstack_amd.server.testing import free_port

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, path, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_two_rank_save_holds_gathered_params(tmp_path):
    for _, ok in _spawn(_gathered_worker, str(tmp_path)):
        assert ok


def test_resume_counts_steps_globally(tmp_path):
    for _, first, final, saved in _spawn(_resume_target_worker, str(tmp_path)):
        assert (first, final, saved) == (2, 4, 4)


def test_resume_two_ranks_gloo(tmp_path):
    for _, expect, got in _spawn(_worker, str(tmp_path)):
        assert got == expect
    assert len([f for f in os.listdir(tmp_path / "step-00000002") if f.startswith("optim-rank")]) == 2


@pytest.mark.slow
@pytest.mark.parametrize("world", [4, 8])
def test_resume_many_ranks_gloo(tmp_path, world):
    """4 and 8 shards (bucket size 64 Ki elements: the shard boundaries fall inside parameters)."""
    res = _spawn(_worker, str(tmp_path), world=world)
    assert sorted(r for r, _, _ in res) == list(range(world))
    for _, expect, got in res:
        assert got == expect
    assert len([f for f in os.listdir(tmp_path / "step-00000002") if f.startswith("optim-rank")]) == world
    for _, ok in _spawn(_gathered_worker, str(tmp_path / "g"), world=world):
        assert ok


@pytest.mark.gpu
def test_resume_continues_on_gpu(gpu, tmp_path):
    """bf16 flat buffers on the GPU with the HIP kernels; library GEMMs may pick kernels whose
    reduction order varies, so allow 0.1 % of the loss."""
    expect, got = _resume_matches(str(tmp_path / "ckpt"), device="cuda")
    for e, g in zip(expect, got):
        assert abs(e - g) <= 1e-3 * abs(e), (expect, got)
