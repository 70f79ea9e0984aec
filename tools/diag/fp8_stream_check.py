"""Where a weight-streaming fp8 GEMM result goes wrong: for each (rows, N, K, split, rw, shuffled 0|1|2) case
prints the relative error, the count of non-finite outputs and the first bad rows / column blocks.
CASES="200,256,2048,2,64,0;..." python tools/diag/fp8_stream_check.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from dstack_amd.ops import _ext  # noqa: E402
from dstack_amd.ops import reference as ref  # noqa: E402
from dstack_amd.ops.serving import fp8_stream_shuffle  # noqa: E402

C = _ext.require()
cases = os.getenv("CASES", "200,256,2048,2,64,0;256,256,2048,2,64,0;256,256,2048,1,64,0;200,256,2048,1,64,0;"
                  "200,256,2048,2,64,1;256,256,4096,2,32,0")
for case in cases.split(";"):
    M, N, K, S, rw, sh = (int(v) for v in case.split(","))
    torch.manual_seed(0)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
    xq, xs = ref.quant_fp8_rows(x)
    wq, ws = ref.quant_fp8_rows(w)
    want = (xq.float() * xs[:, None]) @ (wq.float() * ws[:, None]).t()
    wk = fp8_stream_shuffle(wq, {1: 16, 2: 224 if rw == 28 else 256}[sh]) if sh else wq
    y = C.fp8_stream_gemm(xq.view(torch.uint8), xs, wk.view(torch.uint8), ws, rw, S, sh).float()
    torch.cuda.synchronize()
    bad = ~torch.isfinite(y)
    d = (y - want).abs()
    tol = 0.02 * want.abs().max().item()
    wrong = (d > tol) | bad
    rows = wrong.any(1).nonzero().flatten().tolist()
    cols = wrong.any(0).nonzero().flatten().tolist()
    err = ((torch.where(bad, torch.zeros_like(y), y) - want).norm() / want.norm()).item()
    print(f"M={M} N={N} K={K} S={S} rw={rw} sh={sh}: rel_err(finite)={err:.3e} nonfinite={int(bad.sum())} "
          f"wrong={int(wrong.sum())} rows[{len(rows)}]={rows[:8]} cols[{len(cols)}]={cols[:8]}", flush=True)
