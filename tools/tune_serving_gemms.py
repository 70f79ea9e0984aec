"""Tune (``--mode tune``) or time (``--mode use``/``off``) the decode-step GEMMs of the serving
engine: y[M, N] = x[M, K] @ W[N, K]^T for every hipGraph batch bucket M and every projection of
the given models.  Decode GEMMs are weight-streaming (M <= 256 rows against GBs of weights), so the
figure of merit is weight bytes / time (TB/s) against HBM3E.  Tune mode writes
``dstack_amd/ops/tuned/gemm_tunableop_serving_gfx950.csv`` (or $DSTACK_AMD_GEMM_TUNING_FILE).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="llama-3-8b,llama-3-70b")
    ap.add_argument("--mode", default="use", choices=["tune", "use", "off"])
    ap.add_argument("--buckets", default="")
    ap.add_argument("--prefill-m", default="", help="extra row counts, e.g. 16384,32000 (prefill steps)")
    ap.add_argument("--max-batch", type=int, default=256)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp8"],
                    help="fp8: the e4m3 projections of --quantization fp8 (torch._scaled_mm, row-wise scales; "
                         "M padded to 16 as the model does; the LM head stays bf16)")
    ap.add_argument("--scaling", default="row", choices=["row", "tensor"],
                    help="fp8 scale form: row-wise (decode) or scalar (the deferred-scale prefill GEMMs, "
                         "model.py RawScaled); TunableOp keys the two separately")
    ap.add_argument("--weights", default="", help="comma-separated subset of wqkv,wo,wgu,wdown,lm_head")
    args = ap.parse_args()
    import torch

    from dstack_amd.models.llama import CONFIGS
    from dstack_amd.ops import gemm_tuning
    from dstack_amd.serving.engine import _buckets

    mode = gemm_tuning.setup(args.mode, kind="serving")
    buckets = [int(b) for b in args.buckets.split(",")] if args.buckets else _buckets(args.max_batch)
    buckets += [int(m) for m in args.prefill_m.split(",") if m]
    dev = torch.device("cuda")
    out = []
    for name in args.models.split(","):
        c = CONFIGS[name]
        nh = c.n_heads + 2 * c.n_kv_heads
        shapes = {"wqkv": (nh * c.head_dim, c.dim), "wo": (c.dim, c.n_heads * c.head_dim),
                  "wgu": (2 * c.ffn_dim, c.dim), "wdown": (c.dim, c.ffn_dim), "lm_head": (c.vocab_size, c.dim)}
        fp8 = args.dtype == "fp8"
        f8 = torch.float8_e4m3fn
        for wname, (N, K) in shapes.items():
            if fp8 and wname == "lm_head":
                continue
            if args.weights and wname not in args.weights.split(","):
                continue
            w = torch.randn(N, K, device=dev).to(torch.bfloat16)
            if fp8:
                w8, sw = w.to(f8), torch.rand(1, N, device=dev) + 0.5
                if args.scaling == "tensor":
                    sw = torch.ones((), device=dev)
            for M in sorted({(m + 15) // 16 * 16 for m in buckets} if fp8 else buckets):
                x = torch.randn(M, K, device=dev).to(torch.bfloat16)
                if fp8:
                    x8, sx = x.to(f8), torch.rand(M, 1, device=dev) + 0.5
                    if args.scaling == "tensor":
                        sx = torch.ones((), device=dev)

                    def mm():
                        return torch._scaled_mm(x8, w8.t(), scale_a=sx, scale_b=sw, out_dtype=torch.bfloat16)
                else:
                    def mm():
                        return x @ w.t()
                for _ in range(3):
                    y = mm()
                torch.cuda.synchronize()
                it = 20
                t0 = time.perf_counter()
                for _ in range(it):
                    y = mm()
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t0) / it
                tbs = (N * K * (1 if fp8 else 2) + (M * K + M * N) * 2) / dt / 1e12
                out.append({"model": name, "w": wname, "dtype": args.dtype, "scaling": args.scaling, "M": M, "N": N, "K": K,
                            "us": round(dt * 1e6, 1),
                            "TBps": round(tbs, 2)})
                print(json.dumps(out[-1]), flush=True)
                del y
    print(json.dumps({"mode": mode, "file": str(gemm_tuning.results_path(kind="serving"))}))


if __name__ == "__main__":
    main()
