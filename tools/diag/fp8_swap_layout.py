"""Decode-batch fp8 GEMMs (Llama-3-70B projections, M = 256 token rows) in hipBLASLt with the operands
swapped: y^T = w . x^T (the weight as the M-side operand, the 256 tokens as the narrow N side) against
the engine's y = x . w^T, both with row-wise scales and bf16 output.  The swapped product is
transposed back (a [N][256] -> [256][N] copy, timed with it).  Run with PYTORCH_TUNABLEOP_ENABLED=1
PYTORCH_TUNABLEOP_TUNING=1 to compare each layout's best hipBLASLt solution.  One JSON line per shape."""
import json
import os
import time

import torch


def bench(fn, iters=200, warm=20):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e6


def main():
    dev = torch.device("cuda")
    M = int(os.environ.get("M", "256"))
    shapes = {"qkv": (10240, 8192), "o": (8192, 8192), "gate_up": (57344, 8192), "down": (8192, 28672)}
    for name, (N, K) in shapes.items():
        x = (torch.randn(M, K, device=dev) * 0.5).to(torch.float8_e4m3fn)
        w = (torch.randn(N, K, device=dev) * 0.5).to(torch.float8_e4m3fn)
        xs = torch.rand(M, 1, device=dev) + 0.5
        ws = torch.rand(1, N, device=dev) + 0.5
        wsT, xsT = ws.t().contiguous(), xs.t().contiguous()
        std = lambda: torch._scaled_mm(x, w.t(), scale_a=xs, scale_b=ws, out_dtype=torch.bfloat16)
        swp = lambda: torch._scaled_mm(w, x.t(), scale_a=wsT, scale_b=xsT, out_dtype=torch.bfloat16)
        swp_t = lambda: swp().t().contiguous()
        ref = std().float()
        err = ((swp_t().float() - ref).norm() / ref.norm()).item()
        ts, tw, twt = bench(std), bench(swp), bench(swp_t)
        tb = N * K / 1e12
        print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "std_us": round(ts, 2), "swapped_us": round(tw, 2),
                          "swapped_plus_transpose_us": round(twt, 2), "std_tb_s": round(tb / ts * 1e6, 3),
                          "swapped_tb_s": round(tb / tw * 1e6, 3), "rel_diff": err,
                          "tunableop": os.environ.get("PYTORCH_TUNABLEOP_TUNING", "0")}), flush=True)
        del x, w


if __name__ == "__main__":
    main()
