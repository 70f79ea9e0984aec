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
    meta = json.loads((tmp_path / "ckpt" / "meta.json").read_text())
    assert meta["step"] == 2 and meta["world"] == 1
    assert sorted(os.listdir(tmp_path / "ckpt")) == ["meta.json", "optim-rank00000-of-00001.safetensors",
                                                     "params.safetensors"]


def test_world_size_mismatch_rejected(tmp_path):
    a = _trainer()
    _losses(a, 1)
    a.save_checkpoint(str(tmp_path))
    meta = json.loads((tmp_path / "meta.json").read_text())
    meta["world"] = 8
    (tmp_path / "meta.json").write_text(json.dumps(meta))
    with pytest.raises(ValueError, match="8 ranks"):
        _trainer().load_checkpoint(str(tmp_path))


def _worker(rank, world, port, path, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        expect, got = _resume_matches(path)
        q.put((rank, expect, got))
    finally:
        dist.destroy_process_group()


def test_resume_two_ranks_gloo(tmp_path):
    from dstack_amd.server.testing import free_port

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, str(tmp_path), q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, expect, got in res:
        assert got == expect
    assert len([f for f in os.listdir(tmp_path) if f.startswith("optim-rank")]) == 2


@pytest.mark.gpu
def test_resume_continues_on_gpu(gpu, tmp_path):
    """bf16 flat buffers on the GPU with the HIP kernels; library GEMMs may pick kernels whose
    reduction order varies, so allow 0.1 % of the loss."""
    expect, got = _resume_matches(str(tmp_path / "ckpt"), device="cuda")
    for e, g in zip(expect, got):
        assert abs(e - g) <= 1e-3 * abs(e), (expect, got)
