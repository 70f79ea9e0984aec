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
ap.add_argument("--clip", type=float, default=0.0, help="global grad-norm clip (ZeroOptimizer clip_grad_norm)")
ap.add_argument("--lm-head-std", type=float, default=None, help="output head init std (0 = zero-init)")
a = ap.parse_args()
CONFIGS["ab"] = dataclasses.replace(CONFIGS["llama-3-8b"], name="ab", n_layers=a.layers)
tr = Trainer("ab", a.seq_len, 1, torch.device("cuda", 0), lr=a.lr, lr_warmup=a.lr_warmup, grad_accum=a.grad_accum,
             data=a.data, data_rows=1, clip_grad_norm=a.clip, lm_head_std=a.lm_head_std)
norms = []
_orig_step = tr.opt.step


def _step():
    if not a.clip:  # the optimizer computes it only when clipping; measure it here otherwise
        norms.append(round(tr.opt.flat_grad.float().norm().item(), 3))
    _orig_step()
    if a.clip:
        norms.append(round(tr.opt.last_grad_norm, 3))


tr.opt.step = _step
losses = []
t0 = time.time()
times = []
for i in range(a.steps):
    torch.cuda.synchronize()
    t1 = time.time()
    losses.append(round(tr.step().item(), 4))
    times.append(round(time.time() - t1, 3))
    print(f"step {i + 1} loss={losses[-1]} gnorm={norms[-1] if norms else None} t={time.time() - t0:.1f}s",
          flush=True)
print(json.dumps({"ops": os.environ.get("DSTACK_AMD_OPS", "hip"), "layers": a.layers, "lr": a.lr,
                  "lr_warmup": a.lr_warmup, "clip": a.clip, "lm_head_std": a.lm_head_std, "losses": losses, "grad_norms": norms, "step_s": times}), flush=True)
