"""The in-tree 256x256-tile GEMM in its e4m3 form (csrc/gemm_nt.hip, F8: scaled 16x16x128 MFMA over
the bf16 kernel's LDS-DMA ring) against hipBLASLt's fp8 GEMM with scalar unit scales
(torch._scaled_mm) -- both give the raw product that the serving engine's deferred-scale consumers
take -- on the Llama-3-70B projections at a decode batch (M = 256) and a prefill batch (M = 16384).

    python tools/bench_fp8_nt.py            # ROWS=256,16384
"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dstack_amd.ops import _ext  # noqa: E402

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


def swiglu_mode(C, rows):
    """gate/up + SwiGLU + per-token quantization (Llama-3-70B, F = 28672): the fused in-tree path
    against hipBLASLt's raw product + the deferred-scale SwiGLU-quant kernel, and against the
    decode path (row-wise scaled hipBLASLt + SwiGLU-quant)."""
    from dstack_amd.ops import reference as ref

    F, K = int(os.getenv("F", "28672")), 8192
    one = torch.ones((), device="cuda", dtype=torch.float32)
    res = {}
    for M in rows:
        torch.manual_seed(0)
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        xq, xs = C.quant_fp8_rows(x)
        xs = xs.reshape(-1).contiguous()
        wq = torch.empty(2 * F, K, device="cuda", dtype=torch.float8_e4m3fn)
        ws = torch.empty(2 * F, device="cuda")
        for i in range(0, 2 * F, 8192):  # quantize in slices (the bf16 weight is 0.9 GB)
            q, s_ = ref.quant_fp8_rows(torch.randn(min(8192, 2 * F - i), K, device="cuda") * 0.02)
            wq[i:i + q.shape[0]], ws[i:i + q.shape[0]] = q, s_
        ours = lambda: C.gemm_nt_f8_swiglu_quant(xq.view(torch.uint8), wq.view(torch.uint8), xs, ws)  # noqa: E731

        def deferred():
            raw = torch._scaled_mm(xq.view(torch.float8_e4m3fn), wq.t(), scale_a=one, scale_b=one,
                                   out_dtype=torch.bfloat16)
            return C.swiglu_quant_fp8_rows(raw, xs, ws)

        def rowwise():
            y = torch._scaled_mm(xq.view(torch.float8_e4m3fn), wq.t(), scale_a=xs.view(-1, 1), scale_b=ws.view(1, -1),
                                 out_dtype=torch.bfloat16)
            return C.swiglu_quant_fp8_rows(y)

        q1, s1, _ = ours()
        q2, s2 = deferred()
        same = (q1.view(torch.uint8) == q2.view(torch.uint8)).float().mean().item()
        t = {k: [] for k in ("fused", "deferred", "rowwise")}
        for _ in range(5):
            t["fused"].append(timed(ours, 10))
            t["deferred"].append(timed(deferred, 10))
            t["rowwise"].append(timed(rowwise, 10))
        r = {"M": M, "F": F, "K": K, "q_bytes_equal": same}
        r.update({k + "_us": statistics.median(v) * 1e3 for k, v in t.items()})
        r["speedup_vs_deferred"] = r["deferred_us"] / r["fused_us"]
        r["speedup_vs_rowwise"] = r["rowwise_us"] / r["fused_us"]
        res[f"swiglu_m{M}"] = r
        print(f"swiglu_m{M}", json.dumps({k: round(v, 4) if isinstance(v, float) else v for k, v in r.items()}),
              flush=True)
        del wq, ws, xq
        torch.cuda.empty_cache()
    print(json.dumps(res))


def main():
    C = _ext.require()
    if os.getenv("MODE") == "swiglu":
        return swiglu_mode(C, [int(m) for m in os.getenv("ROWS", "256,16384").split(",")])
    rows = [int(m) for m in os.getenv("ROWS", "256,16384").split(",")]
    only = os.getenv("ONLY")
    one = torch.ones((), device="cuda", dtype=torch.float32)
    res = {}
    for M in rows:
        for name, (N, K) in SHAPES.items():
            if only and name not in only.split(","):
                continue
            torch.manual_seed(0)
            xq = (torch.randn(M, K, device="cuda") * 2).to(torch.float8_e4m3fn)
            wq = (torch.randn(N, K, device="cuda") * 2).to(torch.float8_e4m3fn)
            out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            ours = lambda: C.gemm_nt_f8(xq.view(torch.uint8), wq.view(torch.uint8), out)  # noqa: E731
            lib = lambda: torch._scaled_mm(xq, wq.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16)  # noqa: E731
            ours()
            y1 = lib()
            err = ((out.float() - y1.float()).norm() / y1.float().norm()).item()
            to, tl = [], []
            for _ in range(5):
                to.append(timed(ours))
                tl.append(timed(lib))
            fl = 2.0 * M * N * K
            r = {"M": M, "N": N, "K": K, "ours_us": statistics.median(to) * 1e3, "lib_us": statistics.median(tl) * 1e3,
                 "rel_diff": err}
            r["ours_pf"] = fl / r["ours_us"] / 1e9
            r["lib_pf"] = fl / r["lib_us"] / 1e9
            r["ours_tb_s"] = N * K / r["ours_us"] / 1e6
            r["speedup"] = r["lib_us"] / r["ours_us"]
            res[f"{name}_m{M}"] = r
            print(f"{name}_m{M}", json.dumps({k: round(v, 4) if isinstance(v, float) else v for k, v in r.items()}),
                  flush=True)
            del xq, wq, out, y1
            torch.cuda.empty_cache()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
