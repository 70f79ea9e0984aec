"""The ZeRO-1 collective path on RCCL, on a single GPU.

An 8-GPU job's data-parallel step issues in-place ``reduce_scatter_tensor`` from autograd hooks,
joins it from the AdamW side stream, and ``all_gather_into_tensor`` from that side stream, waited
on per bucket by the forward prefetch hooks.  With ``force_collectives`` those exact calls run in
a 1-rank RCCL communicator (``init_process_group("nccl")`` world 1), so they execute on the GPU box
we have; at world 1 they are identities, so the result must equal the non-distributed path to
within that path's own run-to-run noise."""

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu

GRAD_ACCUM = 4


def _train(gpu, steps=3, force=False):
    from dstack_amd.models.llama import CONFIGS, Llama
    from dstack_amd.parallel.zero import ZeroOptimizer

    cfg = CONFIGS["llama-tiny"]
    torch.manual_seed(0)
    with torch.device(gpu):
        m = Llama(cfg)
    m.init_weights(seed=1)
    m = m.to(torch.bfloat16)
    # small buckets: several RS/AG per step, uneven last bucket
    opt = ZeroOptimizer(m, lr=1e-3, bucket_numel=(1 << 20) + 4096, overlap_update=True, force_collectives=force)
    opt.install_prefetch_hooks(m)
    g = torch.Generator(device=gpu).manual_seed(7)
    # the same micro-batches every step: the loss must fall (memorisation), not just wander
    data = [torch.randint(0, cfg.vocab_size, (2, 257), device=gpu, generator=g) for _ in range(GRAD_ACCUM)]
    losses = []
    for _ in range(steps):
        opt.zero_grad()
        for i in range(GRAD_ACCUM):
            tok = data[i]
            opt.sync_grads = i == GRAD_ACCUM - 1
            loss = m.loss(tok[:, :-1], tok[:, 1:])
            (loss / GRAD_ACCUM).backward()
        opt.step()
        losses.append(loss.item())
    opt.wait_params()
    torch.cuda.synchronize()
    return m, opt, losses


def test_zero_rccl_one_rank_matches_non_distributed(gpu, monkeypatch):
    import dstack_amd.parallel.zero as zmod

    m_a, _, l_a = _train(gpu)
    _, _, l_b = _train(gpu)
    calls = {"rs": 0, "ag": 0}
    rs, ag = zmod.dist.reduce_scatter_tensor, zmod.dist.all_gather_into_tensor

    def count_rs(*a, **k):
        calls["rs"] += 1
        return rs(*a, **k)

    def count_ag(*a, **k):
        calls["ag"] += 1
        return ag(*a, **k)

    monkeypatch.setattr(zmod.dist, "reduce_scatter_tensor", count_rs)
    monkeypatch.setattr(zmod.dist, "all_gather_into_tensor", count_ag)
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1, device_id=gpu)
    try:
        assert dist.get_backend() == "nccl"
        m_r, opt, l_r = _train(gpu, force=True)
        _, _, l_r2 = _train(gpu, force=True)
    finally:
        dist.destroy_process_group()
    assert opt.collectives and opt.overlap and opt._prefetch and opt._side is not None
    nb = len(opt.buckets)
    assert nb > 2
    # one reduce-scatter and one all-gather per bucket per optimizer step, from the hooks
    assert calls["rs"] == calls["ag"] == 2 * 3 * nb, calls
    noise = max(max(abs(x - y) for x, y in zip(l_a, l_b)), max(abs(x - y) for x, y in zip(l_r, l_r2)))
    diff = max(abs(x - y) for x, y in zip(l_a, l_r))
    assert diff <= 10 * noise + 1e-4 * abs(l_a[-1]), (l_a, l_b, l_r, l_r2)
    for (n, a), (_, b) in zip(m_a.named_parameters(), m_r.named_parameters()):
        rel = ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()
        assert rel < 1e-2, f"{n}: {rel}"
    assert l_r[-1] < l_r[0]
