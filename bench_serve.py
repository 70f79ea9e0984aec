#!/usr/bin/env python3
"""Serving benchmark of the MI355X-native engine (``dstack_amd.serving``): offline throughput and
latency of one model replica on one GPU, random-init weights, synthetic prompts.

    python bench_serve.py --model llama-3-70b --num-prompts 256 --input-len 1024 --output-len 256
    python bench_serve.py --model llama-3-70b --latency --input-len 32000 --output-len 128

Throughput mode submits every prompt at t=0 (like ``vllm benchmark_throughput``) and reports
output and total tokens/s, TTFT / time-per-output-token percentiles, and the engine's prefill and
decode rates.  Latency mode runs single requests back to back (the reference's "single large
prompt" figure, BASELINE.md: ≈11.25 s for a ≈32k-token prompt, Llama 3.1 405B FP8 on 8×MI300X with
vLLM — a different model and GPU count, quoted for scale only).  Prints one JSON line.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def _pct(xs, q):
    if not xs:
        return None
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(round(q / 100 * (len(xs) - 1))))]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-70b")
    ap.add_argument("--num-prompts", type=int, default=256)
    ap.add_argument("--input-len", type=int, default=1024)
    ap.add_argument("--output-len", type=int, default=256)
    ap.add_argument("--max-batch", type=int, default=256)
    ap.add_argument("--max-prefill-tokens", type=int, default=16384)
    ap.add_argument("--max-model-len", type=int, default=None)
    ap.add_argument("--latency", action="store_true", help="single requests back to back")
    ap.add_argument("--repeats", type=int, default=3, help="latency mode: requests")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--temperature", type=float, default=0.0)
    ap.add_argument("--quantization", choices=["fp8"], default=None)
    ap.add_argument("--kv-cache-dtype", choices=["auto", "fp8"], default="auto")
    args = ap.parse_args()

    import numpy as np
    import torch

    from dstack_amd.serving.engine import LLMEngine, SamplingParams

    max_len = args.max_model_len or max(args.input_len + args.output_len + 64, 2048)
    t0 = time.perf_counter()
    eng = LLMEngine.from_model(args.model, max_model_len=max_len, max_batch=1 if args.latency else args.max_batch,
                               max_prefill_tokens=args.max_prefill_tokens, use_graphs=not args.no_graphs and None,
                               quantization=args.quantization, kv_cache_dtype=args.kv_cache_dtype)
    t_load = time.perf_counter() - t0
    t0 = time.perf_counter()
    eng.capture_graphs()
    t_graph = time.perf_counter() - t0
    m = eng.model
    vocab = m.cfg.vocab_size
    rng = np.random.default_rng(0)
    sp = SamplingParams(max_tokens=args.output_len, temperature=args.temperature, ignore_eos=True)

    def prompts(n):
        return [rng.integers(10, vocab - 10, size=args.input_len).tolist() for _ in range(n)]

    # warm-up: one short request through prefill and decode (hipBLASLt heuristics, allocator)
    eng.generate([prompts(1)[0][:128]], SamplingParams(max_tokens=4, ignore_eos=True))
    for k in eng.stats:
        eng.stats[k] = 0 if isinstance(eng.stats[k], int) else 0.0
    torch.cuda.synchronize() if torch.cuda.is_available() else None

    n = args.repeats if args.latency else args.num_prompts
    t0 = time.perf_counter()
    if args.latency:
        reqs = []
        for p in prompts(n):
            reqs += eng.generate([p], sp)
    else:
        reqs = eng.generate(prompts(n), sp)
    elapsed = time.perf_counter() - t0
    out_tokens = sum(len(r.output_ids) for r in reqs)
    in_tokens = sum(len(r.prompt_ids) for r in reqs)
    ttft = [r.first_token_at - r.arrival for r in reqs]
    e2e = [r.finished_at - r.arrival for r in reqs]
    tpot = [(r.finished_at - r.first_token_at) / max(1, len(r.output_ids) - 1) for r in reqs]
    st = eng.stats
    res = {
        "metric": "serving latency (s)" if args.latency else "serving output tokens/s",
        "value": round(_pct(e2e, 50), 4) if args.latency else round(out_tokens / elapsed, 1),
        "unit": "s" if args.latency else "tokens/s",
        "higher_is_better": not args.latency,
        "model": args.model, "dtype": str(m.dtype).replace("torch.", ""), "quantization": args.quantization,
        "kv_cache_dtype": args.kv_cache_dtype, "n_gpus": 1,
        "data": "synthetic prompts (uniform random token ids), random-init weights",
        "num_prompts": n, "input_len": args.input_len, "output_len": args.output_len,
        "max_batch": eng.max_batch, "elapsed_s": round(elapsed, 3),
        "output_tokens_per_s": round(out_tokens / elapsed, 1),
        "total_tokens_per_s": round((in_tokens + out_tokens) / elapsed, 1),
        "ttft_p50_s": round(_pct(ttft, 50), 4), "ttft_p99_s": round(_pct(ttft, 99), 4),
        "tpot_p50_ms": round(_pct(tpot, 50) * 1e3, 3), "e2e_p50_s": round(_pct(e2e, 50), 4),
        "prefill_tokens_per_s": round(st["prefill_tokens"] / st["prefill_s"], 1) if st["prefill_s"] else None,
        "decode_tokens_per_s": round(st["decode_tokens"] / st["decode_s"], 1) if st["decode_s"] else None,
        "engine_steps": st["steps"], "preemptions": st["preemptions"],
        "weights_gb": round(m.weight_bytes() / 1e9, 1), "kv_pages": m.num_pages, "kv_tokens": m.num_pages * 64,
        "load_s": round(t_load, 1), "graph_capture_s": round(t_graph, 1), "graphs": len(eng._graphs),
        "device": torch.cuda.get_device_name(0) if torch.cuda.is_available() else "cpu",
    }
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
