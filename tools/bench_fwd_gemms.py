"""Forward projection GEMMs of the Llama-3-8B step (y = x @ W^T, bf16, 8192 tokens) with the
shipped TunableOp selections: the hipBLASLt bar an owned fused-epilogue GEMM would have to meet
(docs/reference/performance.md, "MLP: what an owned GEMM epilogue could remove").  Random
uniform [-1, 1) operands (zero-filled ones run faster under the power cap).  One JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dstack_amd.ops import gemm_tuning  # noqa: E402


def timeit(fn, iters=20, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e3


def main():
    gemm_tuning.setup("use")
    dev = torch.device("cuda")
    T = int(os.getenv("T", "8192"))
    # (out, in): qkv, o, gate|up, down, and the down projection's input gradient (da = dy @ Wdown)
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
              "down_dgrad": (14336, 4096)}
    out = {"T": T}
    for name, (n, k) in shapes.items():
        x = torch.rand(T, k, device=dev, dtype=torch.bfloat16) * 2 - 1
        w = torch.rand(n, k, device=dev, dtype=torch.bfloat16) * 2 - 1
        ms = timeit(lambda: x @ w.t())
        out[name] = {"ms": round(ms, 4), "tflops": round(2 * T * n * k / ms / 1e9, 1)}
        del x, w
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
