"""``python -m dstack_amd.serving --model llama-3-70b --port 8000``: one OpenAI-compatible model
replica on one GPU (the process a ``type: service`` run starts; see
``examples/llama3-70b-service/service.dstack.yml``)."""

from __future__ import annotations

import argparse
import logging
import os
import time


def main(argv=None):
    ap = argparse.ArgumentParser(prog="python -m dstack_amd.serving")
    ap.add_argument("--model", default=os.environ.get("MODEL", "llama-3-8b"),
                    help="built-in config (random weights) or an HF Llama checkpoint directory")
    ap.add_argument("--served-model-name", default=None)
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=int(os.environ.get("PORT", "8000")))
    ap.add_argument("--max-model-len", type=int, default=None)
    ap.add_argument("--max-batch", type=int, default=256)
    ap.add_argument("--max-prefill-tokens", type=int, default=16384)
    ap.add_argument("--gpu-memory-utilization", type=float, default=0.90)
    ap.add_argument("--no-graphs", action="store_true", help="run decode steps eagerly (no hipGraph capture)")
    ap.add_argument("--seed", type=int, default=0, help="random-init seed for built-in configs")
    ap.add_argument("--quantization", choices=["fp8"], default=None,
                    help="fp8: e4m3 projection weights with per-channel scales, per-token activation scales")
    ap.add_argument("--kv-cache-dtype", choices=["auto", "fp8"], default="auto",
                    help="fp8: e4m3 paged KV cache (half the bytes per decode step, twice the tokens)")
    args = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(message)s")
    log = logging.getLogger("dstack_amd.serving")

    import torch
    import uvicorn

    from dstack_amd.serving.engine import LLMEngine
    from dstack_amd.serving.server import create_app

    if torch.cuda.is_available():
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    t0 = time.time()
    eng = LLMEngine.from_model(args.model, max_model_len=args.max_model_len, seed=args.seed, max_batch=args.max_batch,
                               max_prefill_tokens=args.max_prefill_tokens, use_graphs=not args.no_graphs and None,
                               gpu_memory_utilization=args.gpu_memory_utilization, quantization=args.quantization,
                               kv_cache_dtype=args.kv_cache_dtype)
    eng.capture_graphs()
    m = eng.model
    log.info("model %s: %.1f GB weights, %d KV pages (%d tokens), max_model_len %d, %d graph buckets, ready in %.1fs",
             args.model, m.weight_bytes() / 1e9, m.num_pages, m.num_pages * 64, m.max_model_len, len(eng._graphs),
             time.time() - t0)
    name = args.served_model_name or os.path.basename(os.path.normpath(args.model))
    uvicorn.run(create_app(eng, name), host=args.host, port=args.port, log_level="info")


if __name__ == "__main__":
    main()
