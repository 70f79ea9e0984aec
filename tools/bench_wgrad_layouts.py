"""Which operand layout makes the weight-gradient GEMM fast on MI355X?  dW[P,Q] = g[T,P]^T x[T,Q]
timed as (a) torch.mm(g.t(), x) (both operands reduction-dim-strided, today's path), (b) with g
pre-transposed (gT[P,T] @ x: NN), (c) both pre-transposed (gT @ xT.t(): both reduction-contiguous),
plus the cost of a plain transpose copy.  TunableOp tunes the new layouts into a scratch file
(TUNE=1) so every layout runs its best hipBLASLt solution."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dstack_amd.ops import gemm_tuning  # noqa: E402


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
    if os.getenv("TUNE") == "1":
        import shutil
        shutil.copy(gemm_tuning.results_path(), "/tmp/wgrad_layouts_tune.csv")
        os.environ["DSTACK_AMD_GEMM_TUNING_FILE"] = "/tmp/wgrad_layouts_tune.csv"
        gemm_tuning.setup("tune")
    else:
        gemm_tuning.setup("use")
    dev = torch.device("cuda")
    T = 8192
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}
    out = {}
    for name, (P, Q) in shapes.items():
        torch.manual_seed(0)
        g = torch.randn(T, P, device=dev, dtype=torch.bfloat16)
        x = torch.randn(T, Q, device=dev, dtype=torch.bfloat16)
        gT = g.t().contiguous()
        xT = x.t().contiguous()
        w = torch.empty(P, Q, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * P * Q * T
        r = {}
        r["a_both_strided"] = timeit(lambda: torch.mm(g.t(), x, out=w))
        r["b_gT_nn"] = timeit(lambda: torch.mm(gT, x, out=w))
        r["b2_xT"] = timeit(lambda: torch.mm(g.t(), xT.t(), out=w))
        r["c_both_contig"] = timeit(lambda: torch.mm(gT, xT.t(), out=w))
        buf = torch.empty_like(gT)
        r["transpose_g_ms"] = timeit(lambda: buf.copy_(g.t()))
        res = {k: {"ms": v, "tflops": fl / v / 1e9} if not k.startswith("transpose") else v for k, v in r.items()}
        out[name] = res
        print(name, json.dumps(res), flush=True)
        del g, x, gT, xT, w, buf
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
