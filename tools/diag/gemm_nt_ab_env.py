"""Interleaved same-process A/B of one env switch read by the NT GEMM launcher at each call
(e.g. DSTACK_AMD_GEMM_NT_NTSTORE=0/1): python tools/diag/gemm_nt_ab_env.py NAME v0 v1"""
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
    name, vals = sys.argv[1], sys.argv[2:]
    shapes = [(8192, 28672, 4096), (8192, 4096, 4096), (28672, 4096, 8192), (8192, 14336, 4096)]
    if os.getenv("SHAPES"):  # "M,N,K;M,N,K"
        shapes = [tuple(int(x) for x in sh.split(",")) for sh in os.environ["SHAPES"].split(";")]
    for M, N, K in shapes:
        a = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
        b = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        t = {v: [] for v in vals}
        for _ in range(5):
            for v in vals:
                os.environ[name] = v
                t[v].append(timed(lambda: C.gemm_nt(a, b, out, False)))
        fl = 2.0 * M * N * K
        print(f"{M}x{N}x{K}: " + ", ".join(f"{name}={v}: {statistics.median(t[v]):.4f} ms "
                                           f"({fl / statistics.median(t[v]) / 1e9:.0f} TF)" for v in vals), flush=True)


if __name__ == "__main__":
    main()
