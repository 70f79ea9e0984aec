"""Per-phase cycle breakdown of the in-tree NT GEMM's K-loop (csrc/gemm_nt.hip TRACE build):
workgroup 0, wave 0 (group 0) and wave 4 (group 1), K-iterations 8..11, four s_memtime stamps per
phase: start, fragment reads + DMA retired (before the first barrier), MFMA start (after it), MFMA
issue end (before the second barrier).

    python tools/diag/gemm_nt_phases.py [M N K]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from dstack_amd.ops import _ext  # noqa: E402


def main():
    C = _ext.require()
    M, N, K = (int(x) for x in sys.argv[1:4]) if len(sys.argv) >= 4 else (8192, 4096, 8192)
    a = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    b = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        C.gemm_nt(a, b, out, False)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(5):
        C.gemm_nt(a, b, out, False)
    e.record()
    e.synchronize()
    ms = s.elapsed_time(e) / 5
    nphase = (K // 128) * 4 * ((M // 256) * (N // 256) // 256 or 1)
    print(f"M={M} N={N} K={K}: {ms:.3f} ms, {2 * M * N * K / ms / 1e9:.0f} TFLOP/s, "
          f"{ms * 1e3 / nphase:.3f} us per phase (if tiles/CU >= 1)")
    for rep in range(3):
        tr = C.gemm_nt_trace(a, b, out).cpu()
        print(f"--- run {rep}: per phase [reads+DMA wait | barrier-1 wait | MFMA issue | barrier-2 wait]")
        for wv, name in ((0, "wave0 (group 0)"), (1, "wave4 (group 1)")):
            t = tr[wv, :64].tolist()
            segs = []
            for ph in range(16):
                s0, s1, s2, s3 = t[4 * ph:4 * ph + 4]
                nxt = t[4 * ph + 4] if ph < 15 else None
                segs.append((s1 - s0, s2 - s1, s3 - s2, (nxt - s3) if nxt is not None else None))
            full = [x for x in segs[:-1]]
            mean = [sum(x[i] for x in full) / len(full) for i in range(4)]
            print(f"  {name}: mean {[round(v) for v in mean]} total {round(sum(mean))}")
            print("     P1..P4 of one iteration:", segs[4:8])


if __name__ == "__main__":
    main()
