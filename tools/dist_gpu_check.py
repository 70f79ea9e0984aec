"""Data-parallel ZeRO-1 check on ONE GPU: two ranks over gloo (RCCL refuses two ranks on one
device) share cuda:0, so the GPU path of ``ZeroOptimizer`` — side-stream optimizer-in-backward,
prefetch hooks, direct weight-gradient GEMMs into the flat buffer, HIP AdamW — runs with
world_size 2.  Launch: ``torchrun --nproc-per-node 2 --master-addr 127.0.0.1 tools/dist_gpu_check.py``.

Checks: (1) both ranks hold bitwise-identical parameters after every step; (2) the result matches
one process that trains on the union of the two ranks' micro-batches (grad_accum 4) within bf16 /
Adam-sign noise; (3) losses are finite.  Prints one JSON line from rank 0, exit 0 on success."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from dstack_amd.models.llama import CONFIGS, Llama  # noqa: E402
from dstack_amd.parallel.zero import ZeroOptimizer  # noqa: E402

CFG = CONFIGS["llama-tiny"]
SEQ, STEPS, LR = 256, 3, 1e-3


def _model(dev):
    with torch.device(dev):
        m = Llama(CFG)
    m.to(torch.bfloat16)
    m.init_weights(seed=0)
    return m


def _data(dev):
    g = torch.Generator(device="cpu").manual_seed(7)
    # [step][rank][micro] token rows
    return torch.randint(0, CFG.vocab_size, (STEPS, 2, 2, 1, SEQ + 1), generator=g).to(dev)


def _train(model, opt, batches_per_step):
    losses = []
    for micro in batches_per_step:
        opt.zero_grad()
        for i, b in enumerate(micro):
            opt.sync_grads = i == len(micro) - 1
            loss = model.loss(b[:, :-1], b[:, 1:])
            (loss / len(micro)).backward()
            losses.append(loss.item())
        opt.step()
    opt.wait_params()
    return losses


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    assert world == 2
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    data = _data(dev)
    model = _model(dev)
    opt = ZeroOptimizer(model, lr=LR, eps=1e-2, bucket_numel=1 << 20)
    opt.install_prefetch_hooks(model)
    assert opt._side is not None and opt.overlap, "GPU path must run optimizer-in-backward with overlap"
    losses = _train(model, opt, [list(data[s, rank]) for s in range(STEPS)])
    flat = opt.flat_param.float()
    gathered = [torch.empty_like(flat) for _ in range(world)]
    dist.all_gather(gathered, flat)
    same = torch.equal(gathered[0], gathered[1])
    out = {"ranks_identical": same, "losses_finite": all(map(lambda x: x == x and abs(x) < 1e4, losses))}
    if rank == 0:
        # single process on the union of both ranks' micro-batches (mean over 4 == DP average of 2x2)
        ref = _model(dev)
        # a private single-rank optimizer: present the process as non-distributed while building it
        import dstack_amd.parallel.zero as zmod

        orig = zmod.dist.is_initialized
        zmod.dist.is_initialized = lambda: False
        try:
            ref_opt = ZeroOptimizer(ref, lr=LR, eps=1e-2, bucket_numel=1 << 20)
        finally:
            zmod.dist.is_initialized = orig
        _train(ref, ref_opt, [list(data[s, 0]) + list(data[s, 1]) for s in range(STEPS)])
        diff = (opt.flat_param.float() - ref_opt.flat_param.float()).abs().max().item()
        out["max_param_diff_vs_single"] = diff
        out["tol"] = 4 * LR * STEPS
        out["ok"] = bool(same and out["losses_finite"] and diff <= out["tol"])
        print(json.dumps(out), flush=True)
        code = 0 if out["ok"] else 1
    else:
        code = 0 if same else 1
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(code)


if __name__ == "__main__":
    main()
