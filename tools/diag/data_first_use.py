"""First-use cost of each op of the synthetic data stream (workloads/data.py SyntheticLM.tokens) in
a fresh process: the applied task's first optimizer step spent 0.36-0.39 s in its batches against
~5 ms in later steps (bench_apply first_step_split).  Each op is timed twice with a synchronize."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.zeros(1, device=dev).add_(1)
    torch.cuda.synchronize()
    V, n = 128256, 8193
    ranks = torch.arange(1, V + 1, dtype=torch.float64)
    q = ranks.pow(-1.1)
    q = q / q.sum()
    cdf = torch.cumsum(q, 0).to(dev)
    perm = torch.randperm(V).to(dev)
    idx = torch.arange(n, device=dev)
    row_start = (idx % 8193) == 0
    pow_a = torch.randint(0, V, (n + 1,), device=dev)
    geo_b = torch.randint(0, V, (n + 1,), device=dev)
    gen = torch.Generator(device=dev)
    torch.cuda.synchronize()
    ops = {}

    def t(name, fn):
        for rep in range(2):
            t0 = time.perf_counter()
            out = fn()
            torch.cuda.synchronize()
            ops.setdefault(name, []).append(round((time.perf_counter() - t0) * 1e3, 2))
        return out

    t("manual_seed", lambda: gen.manual_seed(1234))
    u = t("rand_f64", lambda: torch.rand(n, generator=gen, device=dev, dtype=torch.float64))
    s = t("searchsorted", lambda: torch.searchsorted(cdf, u))
    s = t("clamp_max_", lambda: s.clamp_max_(V - 1))
    z = t("index_perm", lambda: perm[s])
    c = t("rand_f32_lt", lambda: torch.rand(n, generator=gen, device=dev) < 0.5)
    c = t("and_not", lambda: c & ~row_start)
    w = t("where", lambda: torch.where(c, torch.zeros_like(idx), idx))
    last = t("cummax", lambda: torch.cummax(w, 0).values)
    k = t("sub", lambda: idx - last)
    t("gather_mul_add_mod", lambda: (pow_a[k] * z[last] + geo_b[k]) % V)
    for name, v in ops.items():
        print(f"{name:20s} first {v[0]:8.2f} ms   second {v[1]:8.2f} ms", flush=True)


if __name__ == "__main__":
    main()
