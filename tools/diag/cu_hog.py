"""What a GEMM pays when a concurrent kernel holds some CUs (as RCCL's reduce-scatter / all-gather
blocks do during ZeRO-1's overlapped backward / forward on a multi-GPU node): the in-tree GEMM
(persistent grid: one workgroup per CU looping over its XCD's tiles; or one workgroup per tile with
DSTACK_AMD_GEMM_NT_PERSISTENT=0) and hipBLASLt, alone and started right after a hog kernel that
holds HOG_BLOCKS workgroup slots for HOG_US microseconds on a second stream."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from dstack_amd.ops import _ext  # noqa: E402


def main():
    C = _ext.require()
    dev = torch.device("cuda", 0)
    T, D, F = 8192, 4096, 14336
    x = torch.randn(T, D, device=dev).bfloat16()
    wgu = (torch.randn(2 * F, D, device=dev) * 0.02).bfloat16()
    wd = (torch.randn(D, F, device=dev) * 0.02).bfloat16()
    a = torch.randn(T, F, device=dev).bfloat16()
    out = torch.empty(T, D, device=dev, dtype=torch.bfloat16)
    sink = torch.zeros(1, device=dev, dtype=torch.int32)
    side = torch.cuda.Stream(device=dev)
    cases = {
        "in-tree gate/up+SwiGLU": lambda: C.gemm_nt_swiglu(x, wgu, False),
        "in-tree down (NT)": lambda: C.gemm_nt(a, wd, out, False),
        "hipBLASLt down": lambda: torch.mm(a, wd.t(), out=out),
    }
    hog_us = float(os.environ.get("HOG_US", "1500"))
    res = {}
    for name, fn in cases.items():
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        for blocks in (0, 32, 112):
            times = []
            for _ in range(5):
                torch.cuda.synchronize()
                if blocks:
                    with torch.cuda.stream(side):
                        C.cu_hog(blocks, 256, 48 * 1024, hog_us, sink)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                torch.cuda.synchronize()
                times.append(e0.elapsed_time(e1))
            times.sort()
            res[f"{name} | hog {blocks} blocks x {hog_us:.0f} us"] = round(times[len(times) // 2], 3)
    for k, v in res.items():
        print(f"{k:55s} {v:8.3f} ms", flush=True)
    print(json.dumps({"persistent": os.environ.get("DSTACK_AMD_GEMM_NT_PERSISTENT", "1"), **res}), flush=True)


if __name__ == "__main__":
    main()
