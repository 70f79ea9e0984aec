"""SwiGLU + per-row e4m3 quantization of a decode step's gate/up product (Llama-3-70B: 256 rows x
2 x 28672), scaled and unscaled forms, and the fused add + RMSNorm -> e4m3 (256 x 8192), timed with
events; one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from dstack_amd.ops import _ext  # noqa: E402

C = _ext.require()
M, F = int(os.getenv("ROWS", "256")), int(os.getenv("F", "28672"))
gu = torch.randn(M, 2 * F, device="cuda", dtype=torch.bfloat16)
rs, cs = torch.rand(M, device="cuda") + 0.5, torch.rand(2 * F, device="cuda") + 0.5
out = {"M": M, "F": F}
D = int(os.getenv("D", "8192"))
x, dl = torch.randn(M, D, device="cuda", dtype=torch.bfloat16), torch.randn(M, D, device="cuda", dtype=torch.bfloat16)
wn = torch.rand(D, device="cuda", dtype=torch.bfloat16) + 0.5
for name, fn in (("unscaled", lambda: C.swiglu_quant_fp8_rows(gu)), ("scaled", lambda: C.swiglu_quant_fp8_rows(gu, rs, cs)),
                 ("add_rmsnorm_fp8", lambda: C.rms_norm_fp8(x, dl, wn, 1e-5)), ("quant_rows", lambda: C.quant_fp8_rows(x))):
    for _ in range(10):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(200):
        fn()
    b.record()
    b.synchronize()
    us = a.elapsed_time(b) / 200 * 1e3
    out[name + "_us"] = round(us, 2)
    nbytes = {"add_rmsnorm_fp8": M * D * 2 * 3 + M * D, "quant_rows": M * D * 3}.get(name, M * 2 * F * 2 + M * F)
    out[name + "_tb_s"] = round(nbytes / us / 1e6, 2)
print(json.dumps(out), flush=True)
