"""hipBLASLt fp8 GEMM (torch._scaled_mm) on the Llama-3-70B prefill shapes: row-wise scales
(per-token x per-output-channel, what the serving engine uses) against tensor-wise scales (one
scalar each), bf16 output.  Prints one JSON line per shape."""
import json
import os
import time

import torch


def bench(fn, iters=20, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e3


def main():
    dev = torch.device("cuda")
    M = int(os.environ.get("M", "16384"))
    shapes = {"qkv": (10240, 8192), "o": (8192, 8192), "gate_up": (57344, 8192), "down": (8192, 28672)}
    for name, (N, K) in shapes.items():
        x = (torch.randn(M, K, device=dev) * 0.5).to(torch.float8_e4m3fn)
        w = (torch.randn(N, K, device=dev) * 0.5).to(torch.float8_e4m3fn)
        xs = torch.rand(M, 1, device=dev) + 0.5
        ws = torch.rand(1, N, device=dev) + 0.5
        one = torch.ones((), device=dev)
        row = lambda: torch._scaled_mm(x, w.t(), scale_a=xs, scale_b=ws, out_dtype=torch.bfloat16)
        ten = lambda: torch._scaled_mm(x, w.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
        tr, tt = bench(row), bench(ten)
        fl = 2.0 * M * N * K
        # the tensor-wise product times the scales equals the row-wise one up to bf16 rounding
        ref = row().float()
        alt = (ten().float() * xs * ws)
        err = ((alt - ref).norm() / ref.norm()).item()
        print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "rowwise_ms": round(tr, 4),
                          "tensorwise_ms": round(tt, 4), "rowwise_pf": round(fl / tr / 1e12, 3),
                          "tensorwise_pf": round(fl / tt / 1e12, 3), "rel_diff_after_scaling": err}), flush=True)
        del x, w


if __name__ == "__main__":
    main()
