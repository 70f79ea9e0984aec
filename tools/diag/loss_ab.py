"""Loss trace of the training workload under one ops path (hip | torch): same init, same synthetic
stream, so two runs are comparable step by step.  Usage:
  DSTACK_AMD_OPS=torch python tools/diag/loss_ab.py --layers 32 --steps 12 --lr 3e-4 --lr-warmup 100"""
import argparse
import dataclasses
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from dstack_amd.models.llama import CONFIGS  # noqa: E402
from dstack_amd.workloads.train_llama import Trainer  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--layers", type=int, default=32)
ap.add_argument("--steps", type=int, default=12)
ap.add_argument("--grad-accum", type=int, default=8)
ap.add_argument("--seq-len", type=int, default=8192)
ap.add_argument("--lr", type=float, default=3e-4)
ap.add_argument("--lr-warmup", type=int, default=100)
ap.add_argument("--data", default="synthetic-lm")
ap.add_argument("--clip", type=float, default=0.0, help="global grad-norm clip (needs DSTACK_AMD_OPT_OVERLAP=0)")
a = ap.parse_args()
CONFIGS["ab"] = dataclasses.replace(CONFIGS["llama-3-8b"], name="ab", n_layers=a.layers)
tr = Trainer("ab", a.seq_len, 1, torch.device("cuda", 0), lr=a.lr, lr_warmup=a.lr_warmup, grad_accum=a.grad_accum,
             data=a.data, data_rows=1)
norms = []
_orig_step = tr.opt.step


def _step():
    g = tr.opt.flat_grad
    n = g.float().norm().item()
    norms.append(round(n, 3))
    if a.clip and n > a.clip:
        g.mul_(a.clip / (n + 1e-6))
    _orig_step()


tr.opt.step = _step
losses = []
t0 = time.time()
for i in range(a.steps):
    losses.append(round(tr.step().item(), 4))
    print(f"step {i + 1} loss={losses[-1]} gnorm={norms[-1] if norms else None} t={time.time() - t0:.1f}s",
          flush=True)
print(json.dumps({"ops": os.environ.get("DSTACK_AMD_OPS", "hip"), "layers": a.layers, "lr": a.lr,
                  "lr_warmup": a.lr_warmup, "clip": a.clip, "losses": losses, "grad_norms": norms}), flush=True)
