"""Where the first optimizer step's extra time goes (bench_apply stage first_step_s is ~1.8 s
longer than a steady step): per micro-batch forward/backward times of steps 1 and 2 with a
synchronize around each, optionally after pre-allocating the caching allocator's pool
(--prealloc-gb) -- run each arm in a fresh process."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prealloc-gb", type=float, default=0)
    ap.add_argument("--grad-accum", type=int, default=8)
    ap.add_argument("--cprofile", action="store_true", help="cProfile the first micro-batch's forward")
    ap.add_argument("--prewarm", action="store_true", help="the library-GEMM prewarm thread, as run() does")
    ap.add_argument("--warm-data", action="store_true", help="generate one throwaway batch before step 0")
    ap.add_argument("--pool-gb", type=float, default=0,
                    help="as run() with DSTACK_AMD_ACT_POOL_GB: reserve the activation pool beside model init")
    a = ap.parse_args()
    from dstack_amd.ops import _ext, gemm_tuning
    from dstack_amd.workloads.train_llama import Trainer

    t0 = time.time()
    _ext.require()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    gemm_tuning.setup()
    if a.prealloc_gb:
        x = torch.empty(int(a.prealloc_gb * 2**30), dtype=torch.uint8, device=dev)
        del x
    t1 = time.time()
    warm = None
    if a.prewarm or a.pool_gb:
        from dstack_amd.models.llama import CONFIGS

        os.environ["DSTACK_AMD_ACT_POOL_GB"] = str(a.pool_gb)
        shapes = gemm_tuning.llama_shapes(CONFIGS["llama-3-8b"], 8192) if a.prewarm else []
        warm = gemm_tuning.prewarm(shapes, dev)
    tr = Trainer("llama-3-8b", 8192, 1, dev, grad_accum=a.grad_accum)
    if warm is not None:
        warm.join()
    torch.cuda.synchronize()
    t2 = time.time()
    print(f"setup {t1 - t0:.3f}s (prealloc {a.prealloc_gb} GB), model init {t2 - t1:.3f}s", flush=True)
    if a.warm_data:
        w0 = time.time()
        tr.stream.batch(1 << 40)
        torch.cuda.synchronize()
        print(f"throwaway batch {time.time() - w0:.3f}s", flush=True)
    for step in range(3):
        ts = time.time()
        tr.opt.zero_grad()
        torch.cuda.synchronize()
        tz = time.time() - ts
        times, tb = [], 0.0
        for i in range(a.grad_accum):
            b0 = time.time()
            tokens, targets = tr.batch()
            torch.cuda.synchronize()
            tb += time.time() - b0
            tr.opt.sync_grads = i == a.grad_accum - 1
            f0 = time.time()
            if a.cprofile and step == 0 and i == 0:
                import cProfile
                import pstats

                prof = cProfile.Profile()
                prof.enable()
                loss = tr.model.loss(tokens, targets)
                torch.cuda.synchronize()
                prof.disable()
                st = pstats.Stats(prof)
                st.sort_stats("cumulative").print_stats(30)
                st.sort_stats("tottime").print_stats(20)
            else:
                loss = tr.model.loss(tokens, targets)
            torch.cuda.synchronize()
            f1 = time.time()
            (loss / a.grad_accum).backward()
            torch.cuda.synchronize()
            f2 = time.time()
            times.append((round(f1 - f0, 3), round(f2 - f1, 3)))
        o0 = time.time()
        tr.opt.step()
        torch.cuda.synchronize()
        print(f"step {step}: total {time.time() - ts:.3f}s, zero_grad {tz:.3f}s, batches {tb:.3f}s, "
              f"opt {time.time() - o0:.3f}s, (fwd, bwd) per micro-batch {times}", flush=True)


if __name__ == "__main__":
    main()
