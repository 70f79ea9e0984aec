"""FP8 (OCP e4m3) GEMM availability and speed on this GPU through torch._scaled_mm (hipBLASLt):
per-tensor and row-wise scales, decode (M=256) and prefill (M=8192) shapes of Llama-3-70B, against
bf16.  Prints one JSON line per case."""
import json
import time

import torch


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e3


def main():
    dev = torch.device("cuda")
    print(json.dumps({"device": torch.cuda.get_device_name(0), "arch": torch.cuda.get_device_properties(0).gcnArchName,
                      "torch": torch.__version__}), flush=True)
    f8 = torch.float8_e4m3fn
    for (M, N, K) in [(256, 10240, 8192), (256, 57344, 8192), (256, 8192, 28672), (8192, 57344, 8192),
                      (1, 8192, 8192), (32, 57344, 8192)]:
        a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
        ref = a.float() @ w.float().t()
        tb = bench(lambda: a @ w.t())
        out = {"M": M, "N": N, "K": K, "bf16_ms": round(tb, 4), "bf16_tflops": round(2 * M * N * K / tb / 1e9, 1)}
        for mode in ("tensor", "rowwise"):
            try:
                if mode == "tensor":
                    sa = (a.abs().max().float() / 448.0).reshape(())
                    sw = (w.abs().max().float() / 448.0).reshape(())
                    sa_, sw_ = sa, sw
                else:
                    sa = a.abs().amax(dim=1, keepdim=True).float() / 448.0
                    sw = w.abs().amax(dim=1, keepdim=True).float() / 448.0
                    sa_, sw_ = sa, sw.t()
                a8 = (a.float() / sa).to(f8)
                w8 = (w.float() / sw).to(f8)
                fn = lambda: torch._scaled_mm(a8, w8.t(), scale_a=sa_, scale_b=sw_, out_dtype=torch.bfloat16)
                y = fn()
                err = ((y.float() - ref).norm() / ref.norm()).item()
                t8 = bench(fn)
                out[mode] = {"ms": round(t8, 4), "tflops": round(2 * M * N * K / t8 / 1e9, 1), "rel_err": round(err, 4)}
            except Exception as e:  # noqa: BLE001
                out[mode] = {"error": str(e)[:200]}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
