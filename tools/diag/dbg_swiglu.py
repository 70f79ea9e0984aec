import sys, torch
sys.path.insert(0, '.')
from dstack_amd.ops import _ext
C = _ext.require()
T, D, F = 1024, 512, 768
g = torch.Generator(device='cuda').manual_seed(0)
x = torch.randn(T, D, device='cuda', generator=g).bfloat16()
w = (torch.randn(2 * F, D, device='cuda', generator=g) * 0.05).bfloat16()
gu, a, aT = C.gemm_nt_swiglu(x, w)
torch.cuda.synchronize()
a2, aT2 = C.swiglu_fwd_t(gu)
bad = (a.float() - a2.float()).abs() > 1e-3
bad |= torch.isnan(a.float())
print('a bad count', bad.sum().item(), 'of', a.numel())
idx = bad.nonzero()
print('rows', sorted(set((idx[:, 0] % 256).tolist()))[:40])
print('cols', sorted(set((idx[:, 1] % 128).tolist()))[:40])
print('tile rows', sorted(set((idx[:, 0] // 256).tolist())), 'tile cols', sorted(set((idx[:, 1] // 128).tolist())))
badT = (aT.float() - aT2.float()).abs() > 1e-3
print('aT bad', badT.sum().item(), 'gu vs ref ok')
print('gu g', gu[0, :8].float().tolist())
print('gu u', gu[0, F:F + 8].float().tolist())
print('a   ', a[0, :8].float().tolist())
print('a2  ', a2[0, :8].float().tolist())
print('a row1', a[1, :8].float().tolist(), 'a2 row1', a2[1, :8].float().tolist())
print('aT[0,:8]', aT[0, :8].float().tolist(), 'aT2', aT2[0, :8].float().tolist())
