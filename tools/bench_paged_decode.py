"""Paged decode attention in isolation: KV bytes / time for batch x context x page layout x split
plan (Llama-3-70B heads: 64 q / 8 kv).  ``contig`` gives each sequence consecutive pages, ``random``
a random permutation of the whole cache (what a long-running server ends up with)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from dstack_amd.ops import serving as sops

    H, KVH = int(os.environ.get("H", 64)), int(os.environ.get("KVH", 8))
    dev = "cuda"
    pages_total = 6000
    k, v = sops.alloc_cache(pages_total, KVH, torch.bfloat16, dev)
    k.normal_()
    v.normal_()
    for B in (32, 64, 256):
        for ctx in (1024, 4096):
            W = 8192 // 64
            need = B * (ctx // 64)
            if need > pages_total:
                continue
            for layout in ("contig", "random"):
                ids = torch.arange(pages_total, device=dev) if layout == "contig" else torch.randperm(pages_total, device=dev)
                tables = torch.zeros(B, W, dtype=torch.int32, device=dev)
                tables[:, : ctx // 64] = ids[:need].view(B, ctx // 64).int()
                ctx_t = torch.full((B,), ctx, dtype=torch.int32, device=dev)
                q = torch.randn(B, (H + 2 * KVH) * 128, device=dev).to(torch.bfloat16)
                out = torch.empty(B, H * 128, dtype=torch.bfloat16, device=dev)
                for tw in (2048, 4096, 8192, 16384):
                    ws = sops.DecodeWorkspace(B, H, KVH, W, dev, target_waves=tw)
                    for _ in range(3):
                        sops.paged_decode(q, k, v, tables, ctx_t, H, KVH, out=out, ws=ws)
                    torch.cuda.synchronize()
                    it = 20
                    t0 = time.perf_counter()
                    for _ in range(it):
                        sops.paged_decode(q, k, v, tables, ctx_t, H, KVH, out=out, ws=ws)
                    torch.cuda.synchronize()
                    dt = (time.perf_counter() - t0) / it
                    kv = B * ctx * KVH * 128 * 2 * 2
                    print(json.dumps({"B": B, "ctx": ctx, "layout": layout, "target_waves": tw, "nsplit": ws.nsplit,
                                      "pps": ws.pps, "us": round(dt * 1e6, 1), "TBps": round(kv / dt / 1e12, 2)}),
                          flush=True)


if __name__ == "__main__":
    main()
