"""Decode-batch fp8 projections of Llama-3-70B (one GPU, M = batch rows): the in-tree fp8 GEMM
(csrc/fp8_gemm.hip) against hipBLASLt's row-scaled fp8 GEMM (torch._scaled_mm, as serving/model.py
calls it), with the weight-stream rate of each.

    python tools/bench_fp8_decode.py            # M = 256, 128
"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dstack_amd.ops import _ext, gemm_tuning  # noqa: E402
from dstack_amd.ops import reference as ref  # noqa: E402

SHAPES = {"qkv": (10240, 8192), "o": (8192, 8192), "gate_up": (57344, 8192), "down": (8192, 28672)}


def timed(fn, iters=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def main():
    C = _ext.require()
    gemm_tuning.setup("use", kind="serving")
    rows = [int(m) for m in os.getenv("ROWS", "256,128").split(",")]
    res = {}
    for M in rows:
        for name, (N, K) in SHAPES.items():
            torch.manual_seed(0)
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
            xq, xs = C.quant_fp8_rows(x)
            wq, ws = ref.quant_fp8_rows(w)
            wq = wq.view(torch.uint8)
            del w
            variants = {}
            for bm, sp in ((64, 1), (128, 1), (128, 2), (128, 4), (64, 2)):
                if not C.fp8_rows_gemm_supported(M, N, K, bm, sp):
                    continue
                part = torch.empty(sp * 256 * N, device="cuda", dtype=torch.float32)
                cnt = torch.zeros((N // 128) * ((M + bm - 1) // bm), device="cuda", dtype=torch.int32)
                variants[f"bm{bm}s{sp}"] = (lambda bm=bm, sp=sp, part=part, cnt=cnt:
                                            C.fp8_rows_gemm(xq, xs, wq, ws, bm, sp, part, cnt))
            ours = variants["bm64s1"]
            pad = -M % 16
            xq_l = torch.nn.functional.pad(xq, (0, 0, 0, pad)) if pad else xq
            xs_l = torch.nn.functional.pad(xs, (0, pad), value=1.0) if pad else xs
            lib = lambda: torch._scaled_mm(xq_l.view(torch.float8_e4m3fn), wq.view(torch.float8_e4m3fn).t(),  # noqa: E731
                                           scale_a=xs_l.view(-1, 1), scale_b=ws.view(1, -1), out_dtype=torch.bfloat16)
            y0, y1 = ours(), lib()[:M]
            err = ((y0.float() - y1.float()).norm() / y1.float().norm()).item()
            to, tl, tv = [], [], {k: [] for k in variants}
            for _ in range(5):
                to.append(timed(ours))
                tl.append(timed(lib))
                for k, fn in variants.items():
                    tv[k].append(timed(fn))
            wb = N * K
            r = {"M": M, "N": N, "K": K, "ours_us": statistics.median(to) * 1e3,
                 "lib_us": statistics.median(tl) * 1e3, "ours_tb_s": wb / statistics.median(to) / 1e9,
                 "lib_tb_s": wb / statistics.median(tl) / 1e9, "rel_diff": err}
            r["speedup"] = r["lib_us"] / r["ours_us"]
            r.update({k + "_us": statistics.median(v) * 1e3 for k, v in tv.items()})
            for k in tv:
                assert ((variants[k]().float() - y1.float()).norm() / y1.float().norm()).item() < 1e-2, k
            res[f"{name}_m{M}"] = r
            print(f"{name}_m{M}", json.dumps({k: round(v, 4) if isinstance(v, float) else v for k, v in r.items()}),
                  flush=True)
            del xq, wq
            torch.cuda.empty_cache()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
