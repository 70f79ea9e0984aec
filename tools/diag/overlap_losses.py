"""Losses of the tiny-model ZeRO training with and without optimizer-in-backward (2 runs each),
plus overlap variants that isolate the norm-weight gradient writer."""
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

import dstack_amd.parallel.zero as zmod  # noqa: E402
from tests.test_ops_gpu import _train_tiny  # noqa: E402

dev = torch.device("cuda", 0)
for mode in (True, False):
    _, _, l = _train_tiny(dev, overlap_update=mode)
    print("overlap" if mode else "plain  ", [round(x, 6) for x in l], flush=True)

if hasattr(zmod.ZeroOptimizer, "_direct_write"):
    orig_init = zmod.ZeroOptimizer.__init__

    def no_writer(self, model, *a, **k):
        orig_init(self, model, *a, **k)
        for p in model.parameters():
            if hasattr(p, "_dsa_grad_writer"):
                del p._dsa_grad_writer
    zmod.ZeroOptimizer.__init__ = no_writer
    _, _, l = _train_tiny(dev, overlap_update=True)
    print("overlap, writer off", [round(x, 6) for x in l], flush=True)
    zmod.ZeroOptimizer.__init__ = orig_init

    orig_dw = zmod.ZeroOptimizer._direct_write

    def synced(self, p, write):
        write(p.grad, not p._dsa_fresh)
        torch.cuda.synchronize()
        p._dsa_fresh = False
        self._direct_ok.add(p)
        if self._hooks_on:
            self._on_grad_ready(p)
    zmod.ZeroOptimizer._direct_write = synced
    _, _, l = _train_tiny(dev, overlap_update=True)
    print("overlap, synced writer", [round(x, 6) for x in l], flush=True)
    zmod.ZeroOptimizer._direct_write = orig_dw
