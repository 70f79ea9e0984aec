"""GPU diagnostics: device, library GEMM ceilings for the Llama-3-8B shapes, SDPA attention time."""
import json, time, torch, subprocess, os
import torch.nn.functional as F

def timeit(fn, iters=10, warm=3):
    for _ in range(warm): fn()
    torch.cuda.synchronize(); t=time.perf_counter()
    for _ in range(iters): fn()
    torch.cuda.synchronize(); return (time.perf_counter()-t)/iters

out = {"device": torch.cuda.get_device_name(0), "mem_gb": torch.cuda.get_device_properties(0).total_memory/2**30,
       "cus": torch.cuda.get_device_properties(0).multi_processor_count, "arch": torch.cuda.get_device_properties(0).gcnArchName}
T=8192
gemms = {"qkv": (T,4096,6144), "wo": (T,4096,4096), "gu": (T,4096,28672), "down": (T,14336,4096), "lm_head": (T,4096,128256)}
for name,(m,k,n) in gemms.items():
    a=torch.randn(m,k,device="cuda",dtype=torch.bfloat16); w=torch.randn(n,k,device="cuda",dtype=torch.bfloat16)
    t=timeit(lambda: a@w.t())
    g=torch.randn(m,n,device="cuda",dtype=torch.bfloat16)
    tdx=timeit(lambda: g@w)
    tdw=timeit(lambda: g.t()@a)
    out[f"gemm_{name}"]={"fwd_tflops":2*m*k*n/t/1e12,"dgrad_tflops":2*m*k*n/tdx/1e12,"wgrad_tflops":2*m*k*n/tdw/1e12}
    del a,w,g
q=torch.randn(1,32,T,128,device="cuda",dtype=torch.bfloat16,requires_grad=True)
k=torch.randn(1,8,T,128,device="cuda",dtype=torch.bfloat16,requires_grad=True)
v=torch.randn(1,8,T,128,device="cuda",dtype=torch.bfloat16,requires_grad=True)
fl = 4*T*T*128*32/2
try:
    tf=timeit(lambda: F.scaled_dot_product_attention(q,k,v,is_causal=True,enable_gqa=True))
    o=F.scaled_dot_product_attention(q,k,v,is_causal=True,enable_gqa=True); do=torch.randn_like(o)
    def fb():
        o=F.scaled_dot_product_attention(q,k,v,is_causal=True,enable_gqa=True); o.backward(do)
    tfb=timeit(fb, iters=5)
    out["sdpa"]={"fwd_ms":tf*1e3,"fwd_tflops":fl/tf/1e12,"fwdbwd_ms":tfb*1e3,"bwd_tflops":2.5*fl/(tfb-tf)/1e12}
except Exception as e:
    out["sdpa_error"]=repr(e)[:300]
try:
    from torch.backends.cuda import flash_sdp_enabled, mem_efficient_sdp_enabled
    out["flash_sdp_enabled"]=flash_sdp_enabled(); out["mem_eff_sdp_enabled"]=mem_efficient_sdp_enabled()
except Exception as e: out["sdp_flags_err"]=repr(e)
x=torch.empty(2**30,device="cuda",dtype=torch.float32); y=torch.empty_like(x)
t=timeit(lambda: y.copy_(x)); out["copy_tb_s"]=2*x.numel()*4/t/1e12
print(json.dumps(out, indent=1))
