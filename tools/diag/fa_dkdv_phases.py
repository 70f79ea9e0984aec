"""Where a q-tile's cycles go in the causal 8-wave dK/dV pass (S=8192, H=32, KVH=8): s_memtime
stamps of waves 0 and 4 of workgroup 0 at tile top, after S/dP, after the softmax/dS math, after
dV/dK and after the tile barrier, q-tiles 8..11 (csrc/flash_attn.hip TR variant)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from dstack_amd.ops import _ext  # noqa: E402


def main():
    C = _ext.require()
    B, S, H, KVH = 1, 8192, 32, 8
    torch.manual_seed(0)
    qkv = (torch.randn(B, S, (H + 2 * KVH) * 128, device="cuda") * 0.5).bfloat16()
    out, lse = C.flash_attn_fwd(qkv, H, KVH, True)
    dout = torch.randn_like(out)
    delta = (out.float() * dout.float()).view(B, S, H, 128).sum(-1).transpose(1, 2).contiguous()
    for rep in range(3):
        tr = C.fa_dkdv_trace(qkv, dout, lse, delta, H, KVH).cpu()
    names = ["S/dP", "softmax+dS", "dV/dK", "barrier"]
    for wv, row in zip((0, 4), tr):
        for t in range(4):
            st = [int(row[t * 5 + k]) for k in range(5)]
            nxt = int(row[(t + 1) * 5]) if t < 3 else None
            seg = {n: st[k + 1] - st[k] for k, n in enumerate(names)}
            tot = (nxt - st[0]) if nxt else sum(seg.values())
            print(f"wave {wv} tile {8 + t}: " + " ".join(f"{n} {v}" for n, v in seg.items()) + f" | tile {tot}",
                  flush=True)


if __name__ == "__main__":
    main()
