"""KM form vs NT form of the in-tree GEMM on one weight-gradient shape (same FLOPs, same tile
count): store / no-store (mode 2) timings, to separate the tile stream from the epilogue.

    SHAPE=28672,4096,8192 python tools/diag/km_vs_nt.py
"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from dstack_amd.ops import _ext  # noqa: E402


def timed(fn, iters=10):
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
    M, N, K = (int(x) for x in os.getenv("SHAPE", "28672,4096,8192").split(","))
    g = torch.randn(K, M, device="cuda").to(torch.bfloat16)
    x = torch.randn(K, N, device="cuda").to(torch.bfloat16)
    gT, xT = g.t().contiguous(), x.t().contiguous()
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    res = {}
    for name, fn in (("km", lambda m: C.gemm_km(g, x, out, m)), ("nt", lambda m: C.gemm_nt_mode(gT, xT, out, m))):
        for mode in (0, 1, 2):
            ts = [timed(lambda: fn(mode)) for _ in range(int(os.getenv("ROUNDS", "5")))]
            res[f"{name}_mode{mode}_ms"] = round(statistics.median(ts), 4)
    fl = 2.0 * M * N * K
    res.update({k.replace("_ms", "_tflops"): round(fl / v / 1e9, 1) for k, v in list(res.items())})
    print(json.dumps({"M": M, "N": N, "K": K, **res}), flush=True)
    if os.getenv("PROFILE_ONLY"):  # one form only, for a --pmc pass
        form = os.getenv("PROFILE_ONLY")
        for _ in range(5):
            (C.gemm_km(g, x, out, 0) if form == "km" else C.gemm_nt_mode(gT, xT, out, 0))
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
