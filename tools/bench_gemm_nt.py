"""In-tree NT GEMM (csrc/gemm_nt.hip) against hipBLASLt (torch.mm with the shipped TunableOp
selections) on every GEMM shape of the Llama-3-8B training step (T = 8192 tokens), random
uniform [-1, 1) operands, interleaved rounds in one process; plus the fused SwiGLU epilogues
against the unfused kernels.

    python tools/bench_gemm_nt.py                 # all shapes
    SHAPES=fwd_gu,dgrad_gu python tools/bench_gemm_nt.py
    SHAPES=km python tools/bench_gemm_nt.py        # weight gradients on token-major operands

km: the KM form (dW = dY^T X with dY, X token-major, ``gemm_km``) against hipBLASLt on the same
operands (its token-major "TT" form) and against what the step did before: transposes of both
operands (HIP transpose kernel) + hipBLASLt on the token-contiguous layout.
"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dstack_amd.ops import _ext, gemm_tuning  # noqa: E402

T = int(os.getenv("T", "8192"))
D, F, QKV, V = 4096, 14336, 6144, 128256
SHAPES = {  # name: (M, N, K) of C[M][N] = A[M][K] B[N][K]^T
    "fwd_qkv": (T, QKV, D), "fwd_o": (T, D, D), "fwd_gu": (T, 2 * F, D), "fwd_down": (T, D, F),
    "fwd_lm": (T, V, D),
    "dgrad_qkv": (T, D, QKV), "dgrad_o": (T, D, D), "dgrad_gu": (T, D, 2 * F), "dgrad_down": (T, F, D),
    "dgrad_lm": (T, D, V),
    "wgrad_qkv": (QKV, D, T), "wgrad_o": (D, D, T), "wgrad_gu": (2 * F, D, T), "wgrad_down": (D, F, T),
    "wgrad_lm": (V, D, T),
}


def timed(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def rand(*shape):
    return (torch.rand(*shape, device="cuda", dtype=torch.float32) * 2 - 1).to(torch.bfloat16)


def main():
    C = _ext.require()
    gemm_tuning.setup("use")
    rounds, iters = int(os.getenv("ROUNDS", "5")), int(os.getenv("ITERS", "10"))
    only = os.getenv("SHAPES")
    res = {}
    for name, (M, N, K) in SHAPES.items():
        if only and name not in only.split(","):
            continue
        torch.manual_seed(0)
        a, b = rand(M, K), rand(N, K)
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        C.gemm_nt(a, b, out, False)
        ref = a.float() @ b.float().t()
        err = ((out.float() - ref).norm() / ref.norm()).item()
        lib = torch.mm(a, b.t())
        err_lib = ((lib.float() - ref).norm() / ref.norm()).item()
        acc = out.clone()
        C.gemm_nt(a, b, acc, True)
        err_acc = ((acc.float() - 2 * ref).norm() / (2 * ref).norm()).item()
        del ref, lib, acc
        th, tl = [], []
        for _ in range(rounds):
            th.append(timed(lambda: C.gemm_nt(a, b, out, False), iters))
            tl.append(timed(lambda: torch.mm(a, b.t(), out=out), iters))
        fl = 2.0 * M * N * K
        r = {"M": M, "N": N, "K": K, "hip_ms": statistics.median(th), "lib_ms": statistics.median(tl),
             "hip_tflops": fl / statistics.median(th) / 1e9, "lib_tflops": fl / statistics.median(tl) / 1e9,
             "hip_min_ms": min(th), "lib_min_ms": min(tl), "rel_err": err, "rel_err_lib": err_lib,
             "rel_err_acc": err_acc}
        r["speedup"] = r["lib_ms"] / r["hip_ms"]
        res[name] = r
        print(name, json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
        del a, b, out
        torch.cuda.empty_cache()
    if not only or "km" in only.split(","):
        for name in ("wgrad_qkv", "wgrad_o", "wgrad_gu", "wgrad_down"):
            M, N, K = SHAPES[name]
            torch.manual_seed(0)
            g, x = rand(K, M), rand(K, N)  # token-major dY [T][P], X [T][Q]
            out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            C.gemm_km(g, x, out)
            ref = g.float().t() @ x.float()
            err = ((out.float() - ref).norm() / ref.norm()).item()
            acc = out.clone()
            C.gemm_km(g, x, acc, 1)
            err_acc = ((acc.float() - 2 * ref).norm() / (2 * ref).norm()).item()
            del ref, acc
            tk, ttt, tnt, ttr = [], [], [], []
            gT, xT = C.transpose2d(g), C.transpose2d(x)
            for _ in range(rounds):
                tk.append(timed(lambda: C.gemm_km(g, x, out), iters))
                ttt.append(timed(lambda: torch.mm(g.t(), x, out=out), iters))
                tnt.append(timed(lambda: torch.mm(gT, xT.t(), out=out), iters))
                ttr.append(timed(lambda: (C.transpose2d(g), C.transpose2d(x)), iters))
            fl = 2.0 * M * N * K
            md = statistics.median
            r = {"M": M, "N": N, "K": K, "km_ms": md(tk), "lib_tt_ms": md(ttt), "lib_nt_ms": md(tnt),
                 "transposes_ms": md(ttr), "km_tflops": fl / md(tk) / 1e9, "lib_nt_tflops": fl / md(tnt) / 1e9,
                 "rel_err": err, "rel_err_acc": err_acc,
                 "speedup_vs_step": (md(tnt) + md(ttr)) / md(tk)}
            res["km_" + name] = r
            print("km_" + name, json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()}),
                  flush=True)
            del g, x, out, gT, xT
            torch.cuda.empty_cache()
    if not only or "swiglu" in only:
        torch.manual_seed(1)
        x, w = rand(T, D), rand(2 * F, D) * 0.05
        gu, a, aT = C.gemm_nt_swiglu(x, w)
        gu_ref = torch.mm(x, w.t())
        a_ref, aT_ref = C.swiglu_fwd_t(gu_ref)
        e_gu = ((gu.float() - gu_ref.float()).norm() / gu_ref.float().norm()).item()
        e_a = ((a.float() - a_ref.float()).norm() / a_ref.float().norm()).item()
        e_at = ((aT.float() - aT_ref.float()).norm() / aT_ref.float().norm()).item()
        tf, tu = [], []
        for _ in range(rounds):
            tf.append(timed(lambda: C.gemm_nt_swiglu(x, w), iters))
            tu.append(timed(lambda: C.swiglu_fwd_t(torch.mm(x, w.t())), iters))
        r = {"fused_ms": statistics.median(tf), "unfused_ms": statistics.median(tu), "err_gu": e_gu, "err_a": e_a,
             "err_aT": e_at}
        gu2, a2, _ = C.gemm_nt_swiglu(x, w, False)
        r["err_gu_r"] = ((gu2.float() - gu_ref.float()).norm() / gu_ref.float().norm()).item()
        r["err_a_r"] = ((a2.float() - a_ref.float()).norm() / a_ref.float().norm()).item()
        r["fused_r_ms"] = statistics.median([timed(lambda: C.gemm_nt_swiglu(x, w, False), iters) for _ in range(rounds)])
        res["swiglu_fwd"] = r
        print("swiglu_fwd", json.dumps(r), flush=True)
        dy, wdT = rand(T, D), rand(F, D) * 0.05
        dgu, dguT = C.gemm_nt_swiglu_bwd(dy, wdT, gu_ref)
        da = torch.mm(dy, wdT.t())
        dgu_ref, dguT_ref = C.swiglu_bwd_t(da, gu_ref)
        e1 = ((dgu.float() - dgu_ref.float()).norm() / dgu_ref.float().norm()).item()
        e2 = ((dguT.float() - dguT_ref.float()).norm() / dguT_ref.float().norm()).item()
        tf, tu = [], []
        for _ in range(rounds):
            tf.append(timed(lambda: C.gemm_nt_swiglu_bwd(dy, wdT, gu_ref), iters))
            tu.append(timed(lambda: C.swiglu_bwd_t(torch.mm(dy, wdT.t()), gu_ref), iters))
        r = {"fused_ms": statistics.median(tf), "unfused_ms": statistics.median(tu), "err_dgu": e1, "err_dguT": e2}
        dgu2, _ = C.gemm_nt_swiglu_bwd(dy, wdT, gu_ref, False)
        r["err_dgu_r"] = ((dgu2.float() - dgu_ref.float()).norm() / dgu_ref.float().norm()).item()
        r["fused_r_ms"] = statistics.median([timed(lambda: C.gemm_nt_swiglu_bwd(dy, wdT, gu_ref, False), iters)
                                             for _ in range(rounds)])
        res["swiglu_bwd"] = r
        print("swiglu_bwd", json.dumps(r), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
