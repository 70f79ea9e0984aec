"""Llama-3-70B decode projections at a batch of 256 rows: the weight-streaming fp8 GEMM
(csrc/fp8_gemm.hip fp8_stream_gemm, split-K variants, row-major or pre-shuffled weights) against hipBLASLt's row-scaled fp8 GEMM with
the serving engine's tuned selections (torch._scaled_mm) and the LDS-staged in-tree form
(fp8_rows_gemm).  One JSON line per shape.

    python tools/bench_fp8_stream.py        # ROWS=256 (comma list), MODEL=8b for the Llama-3-8B shapes
"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dstack_amd.ops import _ext, gemm_tuning  # noqa: E402
from dstack_amd.ops import reference as ref  # noqa: E402
from dstack_amd.ops.serving import fp8_rows_shuffle, fp8_stream_shuffle  # noqa: E402

SHAPES = {"qkv": (10240, 8192), "o": (8192, 8192), "gate_up": (57344, 8192), "down": (8192, 28672)}
if os.getenv("MODEL") == "8b":  # Llama-3-8B projections
    SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}


def timed(fn, iters=50):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    C = _ext.require()
    gemm_tuning.setup("use", kind="serving")
    for M in [int(m) for m in os.getenv("ROWS", "256").split(",")]:
        for name, (N, K) in SHAPES.items():
            torch.manual_seed(0)
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
            xq, xs = C.quant_fp8_rows(x)
            wq, ws = ref.quant_fp8_rows(w)
            wq = wq.view(torch.uint8)
            del w
            lib = lambda: torch._scaled_mm(xq.view(torch.float8_e4m3fn), wq.view(torch.float8_e4m3fn).t(),  # noqa: E731
                                           scale_a=xs.view(-1, 1), scale_b=ws.view(1, -1), out_dtype=torch.bfloat16)
            ref_y = lib().float()
            cands = {"lib": lib}
            wsh = {(1, 0): fp8_stream_shuffle(wq, 16)}
            for g in (256, 224):
                if N % g == 0:
                    wsh[(2, g)] = fp8_stream_shuffle(wq, g)
            for rw in (64, 32, 28):
                g = 224 if rw == 28 else 256
                for sp in (1, 2, 4, 7, 8):
                    if C.fp8_stream_gemm_supported(M, N, K, rw, sp):
                        if rw != 28:
                            cands[f"stream_r{rw}_s{sp}"] = (
                                lambda sp=sp, rw=rw: C.fp8_stream_gemm(xq, xs, wq, ws, rw, sp))
                        for m, key in ((1, (1, 0)), (2, (2, g))):
                            cands[f"stream_sh{m}_r{rw}_s{sp}"] = (
                                lambda sp=sp, rw=rw, m=m, key=key: C.fp8_stream_gemm(xq, xs, wsh[key], ws, rw, sp, m))
                        if rw == 32:  # weights three K-steps ahead
                            cands[f"stream_sh2d3_r{rw}_s{sp}"] = (
                                lambda sp=sp, key=(2, g): C.fp8_stream_gemm(xq, xs, wsh[key], ws, 32, sp, 2, 3))
            if C.fp8_rows_gemm_supported(M, N, K, 64, 1):
                wimg = fp8_rows_shuffle(wq)
                cands["rows_bm64"] = lambda: C.fp8_rows_gemm(xq, xs, wq, ws, 64, 1)
                cands["rows_img_bm64"] = lambda: C.fp8_rows_gemm(xq, xs, wimg, ws, 64, 1, None, None, True)
                if C.fp8_rows_gemm_supported(M, N, K, 128, 1):
                    cands["rows_img_bm128"] = lambda: C.fp8_rows_gemm(xq, xs, wimg, ws, 128, 1, None, None, True)
            out = {"shape": name, "M": M, "N": N, "K": K}
            for k, fn in cands.items():
                err = ((fn().float() - ref_y).norm() / ref_y.norm()).item()
                if not err < 1e-2:  # reported, not timed
                    out[k + "_rel_err"] = err
                    continue
                t = statistics.median(timed(fn) for _ in range(5))
                out[k + "_us"] = round(t, 2)
                out[k + "_tb_s"] = round(N * K / t / 1e6, 3)
            best = min((v, k) for k, v in out.items() if k.endswith("_us") and k.startswith("stream"))
            wimg = None
            out["best_stream"] = best[1][:-3]
            out["speedup_vs_lib"] = round(out["lib_us"] / best[0], 3)
            print(json.dumps(out), flush=True)
            del xq, wq, wsh
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
