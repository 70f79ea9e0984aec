"""Order of gradient-ready reports and bucket completions (optimizer-in-backward) for one step of
the tiny model, with the norm-weight writer on and off."""
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

import dstack_amd.parallel.zero as zmod  # noqa: E402
from dstack_amd.models.llama import CONFIGS, Llama  # noqa: E402

dev = torch.device("cuda", 0)


def run(writer):
    cfg = CONFIGS["llama-tiny"]
    torch.manual_seed(0)
    with torch.device(dev):
        m = Llama(cfg)
    m.init_weights(seed=1)
    m = m.to(torch.bfloat16)
    opt = zmod.ZeroOptimizer(m, lr=1e-3, bucket_numel=1 << 20, overlap_update=True)
    names = {id(p): n for n, p in m.named_parameters()}
    if not writer:
        for p in m.parameters():
            if hasattr(p, "_dsa_grad_writer"):
                del p._dsa_grad_writer
    log = []
    orig = opt._on_grad_ready

    def rec(p):
        b = opt._bucket_of[p]
        if opt.sync_grads:
            log.append(f"{names[id(p)]}->b{b.index}({b.pending - 1})")
        orig(p)
    opt._on_grad_ready = rec
    g = torch.Generator(device=dev).manual_seed(7)
    opt.zero_grad()
    for i in range(2):
        tok = torch.randint(0, cfg.vocab_size, (2, 257), device=dev, generator=g)
        opt.sync_grads = i == 1
        (m.loss(tok[:, :-1], tok[:, 1:]) / 2).backward()
    opt.step()
    torch.cuda.synchronize()
    print("writer" if writer else "hooks ", " ".join(log), flush=True)
    print("buckets", [[names[id(p)] for p in b.params] for b in opt.buckets], flush=True)


run(False)
run(True)
