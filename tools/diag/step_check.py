"""Does the first optimizer step change the weights on the GPU path?  Prints per-step loss and
the relative change of a few parameters, with and without optimizer-in-backward."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from dstack_amd.workloads.train_llama import Trainer  # noqa: E402

model = os.getenv("MODEL", "llama-tiny")
seq = int(os.getenv("SEQ", "256"))
tr = Trainer(model, seq, 1, torch.device("cuda"), grad_accum=2)
m = tr.model
names = ["lm_head", "embed", "layers.0.wqkv", "layers.0.attn_norm"]
params = dict(m.named_parameters())
for i in range(4):
    before = {n: params[n].detach().float().clone() for n in names}
    loss = tr.step().item()
    torch.cuda.synchronize()
    ch = {n: ((params[n].detach().float() - before[n]).norm() / before[n].norm()).item() for n in names}
    print(f"step {i} loss={loss:.6f} " + " ".join(f"{n}={v:.2e}" for n, v in ch.items()), flush=True)
