"""Where the applied task's start-up goes after ``import torch`` (bench_apply stages: ~0.28 s in the
"GEMM selections" stage and ~0.27 s of model init): the calls of workloads/train_llama.run() in
order, each followed by a synchronize, in a fresh process."""
import os
import sys
import time

T0 = time.perf_counter()
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

marks = [("import torch", time.perf_counter() - T0)]


def mark(name, t0):
    torch.cuda.synchronize()
    marks.append((name, time.perf_counter() - t0))
    return time.perf_counter()


def main():
    t = time.perf_counter()
    torch.cuda.set_device(0)
    t = mark("set_device", t)
    from dstack_amd.ops import _ext

    _ext.require()
    t = mark("_ext.require", t)
    props = torch.cuda.get_device_properties(0)
    t = mark("get_device_properties", t)
    torch.cuda.tunable.enable(False)
    t = mark("tunable.enable(False)", t)
    from dstack_amd.models.llama import CONFIGS, Llama
    from dstack_amd.parallel.zero import ZeroOptimizer

    t = mark("import model/zero", t)
    cfg = CONFIGS["llama-3-8b"]
    dev = torch.device("cuda", 0)
    with torch.device(dev):
        model = Llama(cfg)
    t = mark("Llama() (allocation)", t)
    model.to(torch.bfloat16)
    t = mark("model.to(bf16)", t)
    model.init_weights(seed=0)
    t = mark("init_weights", t)
    opt = ZeroOptimizer(model, bucket_numel=256 * 1024 * 1024)
    t = mark("ZeroOptimizer", t)
    x = torch.empty(8192, 4096, device=dev, dtype=torch.bfloat16)
    w = torch.empty(6144, 4096, device=dev, dtype=torch.bfloat16)
    torch.mm(x, w.t())
    t = mark("first hipBLASLt GEMM", t)
    print(f"device {props.name} {props.gcnArchName}", flush=True)
    for name, dt in marks:
        print(f"{name:28s} {dt * 1e3:9.1f} ms", flush=True)
    del opt, model


if __name__ == "__main__":
    main()
