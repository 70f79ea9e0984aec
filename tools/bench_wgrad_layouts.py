"""Weight-gradient GEMM layouts at the Llama-3-8B training shapes (T = 8192 tokens per micro-batch):
dW = G^T X with G [T, M] and X [T, N] token-major, as the forward/backward produce them, against
the "TN" form the step uses today (both operands transposed to token-contiguous copies first).
Both forms go through hipBLASLt with TunableOp tuning each shape on first use.  Prints one JSON
line per shape: ms of each form (the TN time excludes the transposes it needs; ``tn_with_t`` adds
them)."""
import json
import os
import sys
import time

os.environ.setdefault("PYTORCH_TUNABLEOP_ENABLED", "1")
os.environ.setdefault("PYTORCH_TUNABLEOP_TUNING", "1")
os.environ.setdefault("PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS", "100")
os.environ.setdefault("PYTORCH_TUNABLEOP_FILENAME", "/tmp/wgrad_tunableop.csv")
import torch  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o_proj": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
          "lm_head": (128256, 4096)}


def timeit(fn, iters=20, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e3


def main():
    T = int(os.getenv("T", "8192"))
    only = sys.argv[1:] or list(SHAPES)
    for name in only:
        M, N = SHAPES[name]
        g = torch.randn(T, M, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
        gt, xt = g.t().contiguous(), x.t().contiguous()
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        nt = timeit(lambda: torch.mm(g.t(), x, out=out))          # token-major operands as produced
        tn = timeit(lambda: torch.mm(gt, xt.t(), out=out))        # token-contiguous copies (today)
        tr = timeit(lambda: (g.t().contiguous(), x.t().contiguous()))
        ref = torch.mm(gt, xt.t())
        err = ((torch.mm(g.t(), x).float() - ref.float()).norm() / ref.float().norm()).item()
        fl = 2.0 * T * M * N
        print(json.dumps({"shape": name, "M": M, "N": N, "T": T, "nt_ms": round(nt, 4), "tn_ms": round(tn, 4),
                          "transposes_ms": round(tr, 4), "tn_with_t_ms": round(tn + tr, 4),
                          "nt_tflops": round(fl / nt / 1e9, 1), "tn_tflops": round(fl / tn / 1e9, 1),
                          "rel_diff": err}), flush=True)
        del g, x, gt, xt, out, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
