"""Microbenchmarks of the HIP kernels at Llama-3-8B shapes (T=8192 tokens) vs PyTorch-ROCm."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F
from dstack_amd import ops
from dstack_amd.ops import reference as ref

def timeit(fn, iters=20, warm=3):
    for _ in range(warm): fn()
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(iters): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - t) / iters * 1e3

dev = torch.device("cuda")
res = {}
T, D, F_, V = 8192, 4096, 14336, 128256
x = torch.randn(T, D, device=dev, dtype=torch.bfloat16)
w = torch.ones(D, device=dev, dtype=torch.bfloat16)
C = ops._ext.require()
res["rmsnorm_fwd_ms"] = timeit(lambda: C.rms_norm_fwd(x, w, 1e-5))
y, rstd = C.rms_norm_fwd(x, w, 1e-5)
res["rmsnorm_bwd_ms"] = timeit(lambda: C.rms_norm_bwd(x, x, w, rstd, None))
res["torch_rmsnorm_fwd_ms"] = timeit(lambda: F.rms_norm(x, (D,), w, 1e-5))
gu = torch.randn(T, 2 * F_, device=dev, dtype=torch.bfloat16)
res["swiglu_fwd_ms"] = timeit(lambda: C.swiglu_fwd(gu))
a = C.swiglu_fwd(gu)
res["swiglu_bwd_ms"] = timeit(lambda: C.swiglu_bwd(a, gu))
res["torch_swiglu_fwd_ms"] = timeit(lambda: F.silu(gu[:, :F_]) * gu[:, F_:])
qkv = torch.randn(1, T, 48 * 128, device=dev, dtype=torch.bfloat16)
cos, sin = ref.rope_cos_sin(T, 128, 500000.0, dev)
res["rope_ms"] = timeit(lambda: C.rope_qkv(qkv, cos, sin, 40, 128, False))
logits = torch.randn(T, V, device=dev, dtype=torch.bfloat16)
tgt = torch.randint(0, V, (T,), device=dev)
res["ce_fwd_ms"] = timeit(lambda: C.cross_entropy_fwd(logits, tgt))
loss, lse = C.cross_entropy_fwd(logits, tgt)
sc = torch.ones(1, device=dev)
res["ce_bwd_ms"] = timeit(lambda: C.cross_entropy_bwd(logits, tgt, lse, sc, False))
n = 512 * 1024 * 1024
p = torch.zeros(n, device=dev, dtype=torch.bfloat16); g = torch.zeros_like(p)
mst = torch.zeros(n, device=dev); m = torch.zeros(n, device=dev); v = torch.zeros(n, device=dev)
t = timeit(lambda: C.adamw(p, g, mst, m, v, 1e-3, .9, .95, 1e-8, .1, .5, .5, 1.0, 0), iters=5)
res["adamw_512M_ms"] = t; res["adamw_TBps"] = n * 30 / t / 1e9
del p, g, mst, m, v
for name in ["rmsnorm_fwd", "swiglu_fwd", "swiglu_bwd", "rope", "ce_fwd", "ce_bwd"]:
    pass
res["bytes_GBps"] = {
    "rmsnorm_fwd": 2 * T * D * 2 / res["rmsnorm_fwd_ms"] / 1e6,
    "rmsnorm_bwd": 3 * T * D * 2 / res["rmsnorm_bwd_ms"] / 1e6,
    "swiglu_fwd": 3 * T * F_ * 2 / res["swiglu_fwd_ms"] / 1e6,
    "swiglu_bwd": 5 * T * F_ * 2 / res["swiglu_bwd_ms"] / 1e6,
    "rope": 2 * T * 48 * 128 * 2 / res["rope_ms"] / 1e6,
    "ce_fwd": T * V * 2 / res["ce_fwd_ms"] / 1e6,
    "ce_bwd": 2 * T * V * 2 / res["ce_bwd_ms"] / 1e6,
}
# attention
for S in (8192,):
    H, KV = 32, 8
    qkv = torch.randn(1, S, (H + 2 * KV) * 128, device=dev, dtype=torch.bfloat16)
    fl = 4 * S * S * 128 * H / 2
    tf = timeit(lambda: C.flash_attn_fwd(qkv, H, KV, True), iters=10)
    o, lse = C.flash_attn_fwd(qkv, H, KV, True)
    do = torch.randn_like(o)
    tb = timeit(lambda: C.flash_attn_bwd(do, qkv, o, lse, H, KV, True), iters=5)
    res[f"fa_fwd_S{S}"] = {"ms": tf, "tflops": fl / tf / 1e9}
    res[f"fa_bwd_S{S}"] = {"ms": tb, "tflops": 2.5 * fl / tb / 1e9}
print(json.dumps(res, indent=1))
