"""One shape of the weight-streaming fp8 GEMM, repeated (for rocprofv3 counter passes):
SHAPE=N,K ROWS=256 RW=64 SPLIT=1 SH=0|1|2 python tools/diag/fp8_stream_one.py  (SH: shuffled weight layout)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from dstack_amd.ops import _ext  # noqa: E402
from dstack_amd.ops import reference as ref  # noqa: E402
from dstack_amd.ops.serving import fp8_stream_shuffle  # noqa: E402

C = _ext.require()
N, K = (int(v) for v in os.getenv("SHAPE", "57344,8192").split(","))
M, rw, sp = int(os.getenv("ROWS", "256")), int(os.getenv("RW", "64")), int(os.getenv("SPLIT", "1"))
sh = int(os.getenv("SH", "0"))
x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
xq, xs = C.quant_fp8_rows(x)
wq, ws = ref.quant_fp8_rows(w)
wq = wq.view(torch.uint8)
if sh:
    wq = fp8_stream_shuffle(wq, 16 if sh == 1 else (224 if rw == 28 else 256))
for _ in range(20):
    C.fp8_stream_gemm(xq, xs, wq, ws, rw, sp, sh)
torch.cuda.synchronize()
print("ok", M, N, K, rw, sp, sh)
