"""What the in-tree NT GEMM's epilogue costs: the same kernel with and without its stores
(timing-only mode 2 of gemm_nt_mode), interleaved rounds, on the training shapes."""
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
    for M, N, K in [(8192, 28672, 4096), (8192, 4096, 4096), (8192, 4096, 14336), (28672, 4096, 8192)]:
        a = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
        b = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        ts, tn = [], []
        for _ in range(5):
            ts.append(timed(lambda: C.gemm_nt_mode(a, b, out, 0)))
            tn.append(timed(lambda: C.gemm_nt_mode(a, b, out, 2)))
        fl = 2.0 * M * N * K
        s, n = statistics.median(ts), statistics.median(tn)
        tiles = (M // 256) * (N // 256)
        print(f"{M}x{N}x{K}: with stores {s:.4f} ms ({fl / s / 1e9:.0f} TF), without {n:.4f} ms ({fl / n / 1e9:.0f} TF), "
              f"epilogue {1e3 * (s - n) / max(1, tiles / 256):.1f} us per tile-round", flush=True)


if __name__ == "__main__":
    main()
