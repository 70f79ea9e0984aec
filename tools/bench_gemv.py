"""Decode-projection GEMV (csrc/gemv.hip; fp8 weights: csrc/fp8.hip) vs hipBLASLt (torch.mm with the shipped serving TunableOp
selections) at M = 1/2/4 on the Llama-3-70B / 8B projection shapes: weight-stream TB/s."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dstack_amd.ops import _ext, gemm_tuning  # noqa: E402


def timeit(fn, iters=50, warm=5):
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
    gemm_tuning.setup("use", kind="serving")
    shapes = {"70b.qkv": (10240, 8192), "70b.o": (8192, 8192), "70b.gate_up": (57344, 8192),
              "70b.down": (8192, 28672), "70b.lm_head": (128256, 8192), "8b.gate_up": (28672, 4096),
              "8b.down": (4096, 14336)}
    out = {}
    for name, (N, K) in shapes.items():
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
        for M in (1, 2, 4):
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            tg = timeit(lambda: C.gemv(x, w))
            tl = timeit(lambda: x @ w.t())
            err = ((C.gemv(x, w).float() - (x @ w.t()).float()).norm() / (x @ w.t()).float().norm()).item()
            out[f"{name}.M{M}"] = {"gemv_ms": tg, "gemv_TBps": N * K * 2 / tg / 1e9, "lib_ms": tl,
                                   "lib_TBps": N * K * 2 / tl / 1e9, "rel_err": err}
            if C.gemv_fp8_supported(M, K):  # e4m3 weights: half the bytes (--quantization fp8)
                q, sc = C.quant_fp8_rows(w)
                t8 = timeit(lambda: C.gemv_fp8(x, q, sc))
                out[f"{name}.M{M}"].update(fp8_ms=t8, fp8_TBps=N * K / t8 / 1e9)
                del q, sc
            print(name, M, json.dumps(out[f"{name}.M{M}"]), flush=True)
        del w
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
