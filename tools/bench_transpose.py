"""HIP transpose2d bandwidth at the Llama-3-8B activation shapes (read + write bytes / time)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dstack_amd.ops import _ext  # noqa: E402


def main():
    C = _ext.require()
    out = {}
    for cols in (4096, 6144, 14336, 28672):
        x = torch.randn(8192, cols, device="cuda", dtype=torch.bfloat16)
        for _ in range(3):
            C.transpose2d(x)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(20):
            C.transpose2d(x)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) / 20 * 1e3
        out[cols] = {"ms": ms, "TBps": 2 * x.numel() * 2 / ms / 1e9}
        assert torch.equal(C.transpose2d(x), x.t().contiguous())
    print(json.dumps(out))


if __name__ == "__main__":
    main()
