"""Weight-gradient GEMM (dW = dY^T X) at the Llama-3-8B shapes: HIP gemm_tn vs hipBLASLt/rocBLAS
(torch.mm with the shipped TunableOp selections), plus accuracy against an fp32 matmul."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dstack_amd.ops import _ext, gemm_tuning  # noqa: E402


def timeit(fn, iters=10, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e3


def main():
    C = _ext.require()
    gemm_tuning.setup("use")
    dev = torch.device("cuda")
    T = int(os.getenv("T", "8192"))
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
              "lm_head": (128256, 4096)}
    only = os.getenv("SHAPES")
    out = {}
    for name, (P, Q) in shapes.items():
        if only and name not in only.split(","):
            continue
        torch.manual_seed(0)
        pad = int(os.getenv("PAD", "0"))  # leading-dimension padding (elements) for stride experiments
        g = torch.randn(T, P + pad, device=dev, dtype=torch.bfloat16)[:, :P]
        x = torch.randn(T, Q + pad, device=dev, dtype=torch.bfloat16)[:, :Q]
        w = torch.empty(P, Q, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * P * Q * T
        t_hip = timeit(lambda: C.gemm_tn(g, x, w, False))
        t_acc = timeit(lambda: C.gemm_tn(g, x, w, True))
        t_lib = timeit(lambda: torch.mm(g.t(), x, out=w))
        C.gemm_tn(g, x, w, False)
        ref = g.float().t() @ x.float()
        if os.getenv("DSTACK_AMD_GEMM_TN") == "noload":
            ref = w.float()
        err = ((w.float() - ref).norm() / ref.norm()).item()
        w2 = w.clone()
        C.gemm_tn(g, x, w2, True)
        err_acc = ((w2.float() - (w.float() + ref)).norm() / ref.norm()).item()
        out[name] = {"P": P, "Q": Q, "T": T, "hip_ms": t_hip, "hip_tflops": fl / t_hip / 1e9,
                     "hip_acc_ms": t_acc, "lib_ms": t_lib, "lib_tflops": fl / t_lib / 1e9,
                     "rel_err": err, "rel_err_acc": err_acc}
        print(name, json.dumps(out[name]), flush=True)
        del g, x, w, w2, ref
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
