import sys, torch
sys.path.insert(0, '.')
from dstack_amd.ops import _ext
C = _ext.require()
torch.manual_seed(0)
for (M, N, K) in [(256, 256, 128), (512, 768, 256), (1024, 512, 1024), (2048, 2304, 640), (2304, 9472, 128), (4096, 4352, 256), (8192, 8192, 384)]:
    a = (torch.rand(M, K, device='cuda') * 2 - 1).bfloat16(); b = (torch.rand(N, K, device='cuda') * 2 - 1).bfloat16()
    out = torch.empty(M, N, device='cuda', dtype=torch.bfloat16)
    C.gemm_nt(a, b, out, False); torch.cuda.synchronize()
    ref = a.float() @ b.float().t()
    print(M, N, K, 'err', ((out.float() - ref).norm() / ref.norm()).item(), 'maxabs', (out.float() - ref).abs().max().item(), flush=True)
x = (torch.rand(512, 256, device='cuda') * 2 - 1).bfloat16(); w = (torch.rand(2 * 384, 256, device='cuda') * 2 - 1).bfloat16() * 0.1
gu, a, aT = C.gemm_nt_swiglu(x, w); torch.cuda.synchronize()
gr = torch.mm(x, w.t()); ar, atr = C.swiglu_fwd_t(gr)
print('swiglu', [((u.float() - v.float()).norm() / v.float().norm()).item() for u, v in [(gu, gr), (a, ar), (aT, atr)]], flush=True)
dy = (torch.rand(512, 256, device='cuda') * 2 - 1).bfloat16(); wd = (torch.rand(512, 256, device='cuda') * 2 - 1).bfloat16() * 0.1
gu2 = (torch.rand(512, 1024, device='cuda') * 2 - 1).bfloat16()
dgu, dguT = C.gemm_nt_swiglu_bwd(dy, wd, gu2); torch.cuda.synchronize()
d1, d2 = C.swiglu_bwd_t(torch.mm(dy, wd.t()), gu2)
print('swiglu_bwd', [((u.float() - v.float()).norm() / v.float().norm()).item() for u, v in [(dgu, d1), (dguT, d2)]], flush=True)
# accumulate path on a persistent (> CU count) grid
a = (torch.rand(4096, 512, device='cuda') * 2 - 1).bfloat16(); b = (torch.rand(4352, 512, device='cuda') * 2 - 1).bfloat16()
out = (torch.rand(4096, 4352, device='cuda') * 2 - 1).bfloat16(); ref = out.float() + a.float() @ b.float().t()
C.gemm_nt(a, b, out, True); torch.cuda.synchronize()
print('acc err', ((out.float() - ref).norm() / ref.norm()).item(), flush=True)
# swiglu on a persistent grid (T=4096, F=4096 -> 16 x 32 = 512 tiles)
x = (torch.rand(4096, 256, device='cuda') * 2 - 1).bfloat16(); w = (torch.rand(8192, 256, device='cuda') * 2 - 1).bfloat16() * 0.1
gu, a, aT = C.gemm_nt_swiglu(x, w); torch.cuda.synchronize()
gr = torch.mm(x, w.t()); ar, atr = C.swiglu_fwd_t(gr)
print('swiglu persistent', [((u.float() - v.float()).norm() / v.float().norm()).item() for u, v in [(gu, gr), (a, ar), (aT, atr)]], flush=True)
