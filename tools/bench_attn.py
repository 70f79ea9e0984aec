"""Flash-attention kernel timing + accuracy at the Llama-3-8B training shape (S=8192, 32 q / 8 kv
heads, d=128, causal) vs PyTorch SDPA (fp32 math reference for the error)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dstack_amd.ops import _ext  # noqa: E402


def timeit(fn, iters=10, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e3


def main():
    C = _ext.require()
    dev = torch.device("cuda")
    out = {}
    S, H, KV, D = int(os.getenv("S", "8192")), 32, 8, 128
    torch.manual_seed(0)
    qkv = torch.randn(1, S, (H + 2 * KV) * D, device=dev, dtype=torch.bfloat16)
    fl = 4 * S * S * D * H / 2
    tf = timeit(lambda: C.flash_attn_fwd(qkv, H, KV, True))
    o, lse = C.flash_attn_fwd(qkv, H, KV, True)
    do = torch.randn_like(o)
    tb = timeit(lambda: C.flash_attn_bwd(do, qkv, o, lse, H, KV, True), iters=5)
    out["fwd_ms"], out["fwd_tflops"] = tf, fl / tf / 1e9
    out["bwd_ms"], out["bwd_tflops"] = tb, 2.5 * fl / tb / 1e9
    # accuracy on a shorter sequence against fp32 SDPA
    s2 = 1024
    x = torch.randn(1, s2, (H + 2 * KV) * D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    o2, l2 = C.flash_attn_fwd(x.detach(), H, KV, True)
    g = torch.randn_like(o2)
    dx = C.flash_attn_bwd(g, x.detach(), o2, l2, H, KV, True)
    xf = x.detach().float().requires_grad_(True)
    q, k, v = xf.view(1, s2, H + 2 * KV, D).split([H, KV, KV], dim=2)
    k = k.repeat_interleave(H // KV, dim=2)
    v = v.repeat_interleave(H // KV, dim=2)
    ref = torch.nn.functional.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2),
                                                           is_causal=True).transpose(1, 2).reshape(1, s2, H * D)
    ref.backward(g.float())
    out["fwd_max_err"] = (o2.float() - ref).abs().max().item()
    out["bwd_max_err"] = (dx.float() - xf.grad).abs().max().item()
    out["bwd_rel_err"] = ((dx.float() - xf.grad).norm() / xf.grad.norm()).item()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
