"""What the first optimizer step's first forward pays (profiles/first_step_r8b.txt: 1.2 s vs 0.1 s):
wall time of the FIRST torch.mm call per Llama-3-8B training shape (hipBLASLt through TunableOp
with the shipped selections), then of a second call.  ``--warm-thread`` first runs one tiny GEMM on
a background thread while the main thread sleeps, to see whether the cost is a one-time library
initialisation that can overlap other start-up work."""
import argparse
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--warm-thread", action="store_true")
    ap.add_argument("--tuning", default="use")
    a = ap.parse_args()
    from dstack_amd.ops import gemm_tuning

    t0 = time.time()
    torch.cuda.set_device(0)
    torch.zeros(1, device="cuda")
    torch.cuda.synchronize()
    print(f"cuda init {time.time() - t0:.3f}s", flush=True)
    t0 = time.time()
    gemm_tuning.setup(a.tuning)
    print(f"gemm_tuning.setup {time.time() - t0:.3f}s", flush=True)
    if a.warm_thread:
        def warm():
            w0 = time.time()
            x = torch.zeros(256, 256, device="cuda", dtype=torch.bfloat16)
            torch.mm(x, x.t())
            torch.cuda.synchronize()
            print(f"warm thread {time.time() - w0:.3f}s", flush=True)
        th = threading.Thread(target=warm)
        th.start()
        th.join()
    T, D, F, QKV, V = 8192, 4096, 14336, 6144, 128256
    shapes = [("qkv", T, QKV, D), ("o", T, D, D), ("down", T, D, F), ("lm", T, V, D), ("dgrad_qkv", T, D, QKV),
              ("dgrad_gu", T, D, 2 * F), ("dgrad_lm", T, D, V)]
    for name, M, N, K in shapes:
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
        torch.cuda.synchronize()
        ts = []
        for _ in range(2):
            t0 = time.time()
            torch.mm(x, w.t())
            torch.cuda.synchronize()
            ts.append(round(time.time() - t0, 4))
        print(f"{name} {M}x{N}x{K}: first {ts[0]}s second {ts[1]}s", flush=True)
        del x, w


if __name__ == "__main__":
    main()
