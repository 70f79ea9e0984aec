"""Numerics of every HIP kernel against the plain-PyTorch fp32 reference (``ops.reference``)."""

import math

import pytest
import torch

from dstack_amd import ops
from dstack_amd.ops import _ext
from dstack_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def _rand(*shape, device, scale=1.0, dtype=torch.bfloat16, seed=0):
    g = torch.Generator(device=device).manual_seed(seed)
    return (torch.randn(*shape, device=device, generator=g) * scale).to(dtype)


def _close(a, b, atol, rtol=0.0):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    tol = atol + rtol * b.abs().max().item()
    assert err <= tol, f"max abs err {err} > {tol}"


def test_extension_loaded(gpu):
    assert _ext.available(), "HIP extension must be built for GPU runs"


@pytest.mark.parametrize("rows", [512, 4096])  # block-per-row (<= 1024 rows) and wave-per-row kernels
@pytest.mark.parametrize("D", [256, 4096, 8192])
def test_rms_norm(gpu, D, rows):
    x = _rand(rows, D, device=gpu).requires_grad_()
    w = (1 + 0.1 * _rand(D, device=gpu, seed=1)).requires_grad_()
    y = ops.rms_norm(x, w, 1e-5)
    xr = x.detach().float().requires_grad_()
    wr = w.detach().float().requires_grad_()
    yr = ref.rms_norm(xr, wr, 1e-5)
    _close(y, yr, 2e-2, 1e-2)
    dy = _rand(rows, D, device=gpu, seed=2)
    y.backward(dy)
    yr.backward(dy.float())
    _close(x.grad, xr.grad, 3e-2, 1e-2)
    _close(w.grad, wr.grad, 0.5, 2e-2)


def test_add_rms_norm(gpu):
    D = 4096
    x = _rand(256, D, device=gpu).requires_grad_()
    d = _rand(256, D, device=gpu, seed=3).requires_grad_()
    w = (1 + 0.1 * _rand(D, device=gpu, seed=1)).requires_grad_()
    h, y = ops.add_rms_norm(x, d, w, 1e-5)
    xr, dr, wr = (t.detach().float().requires_grad_() for t in (x, d, w))
    hr = xr + dr
    yr = ref.rms_norm(hr, wr, 1e-5)
    _close(h, hr, 2e-2, 1e-2)
    _close(y, yr, 3e-2, 1e-2)
    gh, gy = _rand(256, D, device=gpu, seed=4), _rand(256, D, device=gpu, seed=5)
    (h.float() * gh.float()).sum().add((y.float() * gy.float()).sum()).backward()
    (hr * gh.float()).sum().add((yr * gy.float()).sum()).backward()
    _close(x.grad, xr.grad, 5e-2, 1e-2)
    _close(d.grad, dr.grad, 5e-2, 1e-2)


def test_swiglu(gpu):
    gu = _rand(1024, 2 * 1792, device=gpu).requires_grad_()
    a = ops.swiglu(gu)
    gr = gu.detach().float().requires_grad_()
    ar = ref.swiglu(gr)
    _close(a, ar, 2e-2, 1e-2)
    da = _rand(1024, 1792, device=gpu, seed=7)
    a.backward(da)
    ar.backward(da.float())
    _close(gu.grad, gr.grad, 3e-2, 1e-2)


def test_rope(gpu):
    B, S, H, KV, D = 2, 256, 8, 2, 128
    qkv = _rand(B, S, (H + 2 * KV) * D, device=gpu).requires_grad_()
    cos, sin = ref.rope_cos_sin(S, D, 500000.0, gpu)
    out = ops.rope(qkv, cos, sin, H + KV, D)
    x = qkv.detach().float().view(B, S, H + 2 * KV, D)
    exp = torch.cat([ref.apply_rope(x[:, :, : H + KV], cos, sin), x[:, :, H + KV :]], 2).reshape(B, S, -1)
    _close(out, exp, 2e-2, 1e-2)
    g = _rand(B, S, (H + 2 * KV) * D, device=gpu, seed=9)
    out.backward(g)
    xr = qkv.detach().float().view(B, S, H + 2 * KV, D).requires_grad_()
    er = torch.cat([ref.apply_rope(xr[:, :, : H + KV], cos, sin), xr[:, :, H + KV :]], 2).reshape(B, S, -1)
    er.backward(g.float())
    _close(qkv.grad, xr.grad.reshape(B, S, -1), 2e-2, 1e-2)


@pytest.mark.parametrize("V", [1024, 128256])
def test_cross_entropy(gpu, V):
    T = 256
    logits = _rand(T, V, device=gpu, scale=3.0).requires_grad_()
    tgt = torch.randint(0, V, (T,), device=gpu)
    loss = ops.cross_entropy(logits.clone(), tgt)
    lr_ = logits.detach().float().requires_grad_()
    lref = ref.cross_entropy(lr_, tgt)
    assert abs(loss.item() - lref.item()) < 2e-3 * max(1.0, abs(lref.item()))
    l2 = ops.cross_entropy(logits, tgt)
    l2.backward()
    lref.backward()
    _close(logits.grad, lr_.grad, 2e-4, 2e-2)


def test_adamw(gpu):
    n = 1 << 20 | 5  # exercise the scalar tail
    p = _rand(n, device=gpu)
    g = _rand(n, device=gpu, seed=11, scale=0.01)
    master = p.float()
    m = torch.zeros(n, device=gpu)
    v = torch.zeros(n, device=gpu)
    p2, master2, m2, v2 = p.clone(), master.clone(), m.clone(), v.clone()
    for step in (1, 2, 3):
        ops.adamw_(p, g, master, m, v, lr=1e-3, beta1=0.9, beta2=0.95, eps=1e-8, weight_decay=0.1, step=step,
                   grad_scale=0.5)
        ref.adamw_(p2, g, master2, m2, v2, 1e-3, 0.9, 0.95, 1e-8, 0.1, step, 0.5)
    _close(master, master2, 1e-5, 1e-5)
    _close(m, m2, 1e-7, 1e-5)
    _close(p, p2, 1e-2)


@pytest.mark.parametrize("S,H,KV", [(128, 4, 1), (256, 8, 2), (512, 4, 4), (1024, 32, 8)])
@pytest.mark.parametrize("causal", [True, False])
def test_flash_attention(gpu, S, H, KV, causal):
    B, D = 2, 128
    qkv = _rand(B, S, (H + 2 * KV) * D, device=gpu).requires_grad_()
    o = ops.attention(qkv, H, KV, causal=causal)
    xr = qkv.detach().float().requires_grad_()
    q, k, v = ops.functional.split_qkv(xr, H, KV)
    orf = ref.attention(q, k, v, causal).reshape(B, S, -1)
    _close(o, orf, 2e-2, 2e-2)
    do = _rand(B, S, H * D, device=gpu, seed=13)
    o.backward(do)
    orf.backward(do.float())
    g, gr = qkv.grad.view(B, S, H + 2 * KV, D), xr.grad.view(B, S, H + 2 * KV, D)
    for name, sl in (("dq", slice(0, H)), ("dk", slice(H, H + KV)), ("dv", slice(H + KV, H + 2 * KV))):
        a, b = g[:, :, sl].float(), gr[:, :, sl]
        err = (a - b).abs().max().item()
        scale = b.abs().max().item()
        assert err <= 3e-2 * scale + 2e-2, f"{name}: err {err} (ref max {scale})"


def _attn_check(qkv, H, KV, do, causal=True, tol=3e-2):
    B, S = qkv.shape[:2]
    D = 128
    qkv = qkv.detach().requires_grad_()
    o = ops.attention(qkv, H, KV, causal=causal)
    xr = qkv.detach().float().requires_grad_()
    q, k, v = ops.functional.split_qkv(xr, H, KV)
    orf = ref.attention(q, k, v, causal).reshape(B, S, -1)
    _close(o, orf, 2e-2, 2e-2)
    o.backward(do)
    orf.backward(do.float())
    g, gr = qkv.grad.view(B, S, H + 2 * KV, D), xr.grad.view(B, S, H + 2 * KV, D)
    for name, sl in (("dq", slice(0, H)), ("dk", slice(H, H + KV)), ("dv", slice(H + KV, H + 2 * KV))):
        a, b = g[:, :, sl].float(), gr[:, :, sl]
        err = (a - b).abs().max().item()
        scale = b.abs().max().item()
        rel = ((a - b).norm() / (b.norm() + 1e-12)).item()
        assert err <= tol * scale + 2e-2 and rel < 2e-2, f"{name}: err {err} rel {rel} (ref max {scale})"


@pytest.mark.parametrize("S", [4096, 8192])
def test_flash_attention_long_sequence(gpu, S):
    """The bench shape's sequence length (8192) and 4096, forward + all three gradients."""
    B, H, KV, D = 1, 8, 2, 128
    qkv = _rand(B, S, (H + 2 * KV) * D, device=gpu, seed=21)
    do = _rand(B, S, H * D, device=gpu, seed=22)
    _attn_check(qkv, H, KV, do)


def test_flash_attention_deferred_max_stress_long_seq(gpu):
    """Scores that grow with the key index across all 8192 keys: every query's running max keeps
    rising, so the deferred-max path rescales again and again (and the threshold is crossed
    repeatedly) — the output and gradients must still match the exact softmax."""
    B, S, H, KV, D = 1, 8192, 4, 1, 128
    g = torch.Generator(device=gpu).manual_seed(5)
    u = torch.randn(D, device=gpu, generator=g)
    u = u / u.norm()
    x = torch.randn(B, S, H + 2 * KV, D, device=gpu, generator=g) * 0.3
    ramp = torch.linspace(0, 1, S, device=gpu)
    x[:, :, :H] += 4.0 * u  # every query points along u
    x[:, :, H] += (40.0 * ramp)[None, :, None] * u  # key t scores ~ 4*40*t/S/sqrt(128) ≈ 14*t/S ... rising
    qkv = x.reshape(B, S, -1).to(torch.bfloat16)
    do = _rand(B, S, H * D, device=gpu, seed=23)
    _attn_check(qkv, H, KV, do, tol=4e-2)


def test_flash_attention_lse_rescale_branch(gpu):
    """Force the online-softmax rescale: a spike key late in the sequence for every query."""
    B, S, H, KV, D = 1, 512, 2, 1, 128
    qkv = _rand(B, S, (H + 2 * KV) * D, device=gpu, scale=0.5)
    x = qkv.view(B, S, H + 2 * KV, D)
    x[:, 300, H] = x[:, 300, 0].mean(0) * 0 + 4.0  # key 300 aligned with an all-positive direction
    x[:, :, :H] = x[:, :, :H].abs()
    qkv = x.reshape(B, S, -1).contiguous()
    o = ops.attention(qkv, H, KV, causal=True)
    q, k, v = ops.functional.split_qkv(qkv.float(), H, KV)
    orf = ref.attention(q, k, v, True).reshape(B, S, -1)
    _close(o, orf, 3e-2, 2e-2)


def test_llama_tiny_step_matches_reference(gpu, monkeypatch):
    """One fwd+bwd of the tiny Llama through the HIP path vs the fp32 reference path."""
    from dstack_amd.models.llama import CONFIGS, Llama
    import dataclasses

    cfg = dataclasses.replace(CONFIGS["llama-tiny"], dim=512, n_heads=4, n_kv_heads=2)
    torch.manual_seed(0)
    with torch.device(gpu):
        m = Llama(cfg)
    m.init_weights()
    mb = m.to(torch.bfloat16)
    tok = torch.randint(0, cfg.vocab_size, (2, 129), device=gpu)
    loss = mb.loss(tok[:, :-1], tok[:, 1:])
    loss.backward()
    grads = {n: p.grad.float().clone() for n, p in mb.named_parameters()}
    mb.zero_grad()
    monkeypatch.setenv("DSTACK_AMD_OPS", "torch")
    loss_ref = mb.loss(tok[:, :-1], tok[:, 1:])
    loss_ref.backward()
    assert abs(loss.item() - loss_ref.item()) < 2e-2
    for n, p in mb.named_parameters():
        a, b = grads[n], p.grad.float()
        rel = (a - b).norm() / (b.norm() + 1e-12)
        assert rel < 0.08, f"{n}: rel grad err {rel}"


def _train_tiny(gpu, overlap_update, steps=3, grad_accum=2):
    from dstack_amd.models.llama import CONFIGS, Llama
    from dstack_amd.parallel.zero import ZeroOptimizer

    cfg = CONFIGS["llama-tiny"]
    torch.manual_seed(0)
    with torch.device(gpu):
        m = Llama(cfg)
    m.init_weights(seed=1)
    m = m.to(torch.bfloat16)
    opt = ZeroOptimizer(m, lr=1e-3, bucket_numel=1 << 20, overlap_update=overlap_update)
    g = torch.Generator(device=gpu).manual_seed(7)
    losses = []
    for _ in range(steps):
        opt.zero_grad()
        for i in range(grad_accum):
            tok = torch.randint(0, cfg.vocab_size, (2, 257), device=gpu, generator=g)
            opt.sync_grads = i == grad_accum - 1
            loss = m.loss(tok[:, :-1], tok[:, 1:])
            (loss / grad_accum).backward()
        opt.step()
        losses.append(loss.item())
    torch.cuda.synchronize()
    return m, opt, losses


def test_optimizer_in_backward_matches_plain_step(gpu):
    """AdamW launched per bucket on a side stream during backward == AdamW after backward, to
    within the run-to-run variation of the plain path itself (library GEMMs may pick
    stream-K kernels whose partial-tile fix-up order is not fixed)."""
    m1, o1, l1 = _train_tiny(gpu, overlap_update=True)
    _, _, l1b = _train_tiny(gpu, overlap_update=True)
    m2, o2, l2 = _train_tiny(gpu, overlap_update=False)
    m3, _, l3 = _train_tiny(gpu, overlap_update=False)
    assert o1._side is not None and o2._side is None
    # run-to-run noise of either path (library GEMMs may pick stream-K kernels whose fix-up order
    # follows kernel timing, which the overlapped AdamW shifts); the two paths compute the same
    # update, so beyond that noise only 0.01 % of the loss is allowed (a bucket updated before its
    # last gradient landed -- the double-counting bug fixed in ZeroOptimizer._on_grad_ready --
    # moved the loss by 0.06 % after 3 steps)
    noise = max(max(abs(a - b) for a, b in zip(l2, l3)), max(abs(a - b) for a, b in zip(l1, l1b)))
    diff = max(abs(a - b) for a, b in zip(l1, l2))
    assert diff <= 10 * noise + 1e-4 * abs(l2[-1]), (l1, l1b, l2, l3)
    for (n, a), (_, b) in zip(m1.named_parameters(), m2.named_parameters()):
        rel = ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()
        assert rel < 1e-2, f"{n}: {rel}"
    assert l1[-1] < l1[0]  # it trains


def test_flash_attention_kernel_variants_agree(gpu, tmp_path):
    """Every kernel variant gives the same output and gradients as the defaults (8-wave forward,
    8-wave dK/dV, 8-wave dQ, prefetched forward S phase): the 4-wave dK/dV (DSTACK_AMD_FA_DKDV=4w),
    the 4-wave forward and dQ passes (DSTACK_AMD_FA_FWD_WAVES=4, DSTACK_AMD_FA_DQ_WAVES=4) and the
    forward without the S-phase prefetch (DSTACK_AMD_FA_FWD_PF=0) and the exact running max instead of
    the deferred one (DSTACK_AMD_FA_RESCALE_THR=0), and the staggered forward
    (DSTACK_AMD_FA_FWD_STAG=1), and the recompute-free dQ pass over the dS spilled by the dK/dV
    pass (DSTACK_AMD_FA_DQ=ds; also at S=1152, its 4-wave dQ form, causal and not), and dK/dV summed
    over the GQA group in one workgroup (DSTACK_AMD_FA_DKDV_GQA=1, causal and not), and the S/dP read
    pipelines: dK/dV without it or one step ahead (DSTACK_AMD_FA_DKDV_PF=0|1; the default is 2) and the
    dQ pass's (DSTACK_AMD_FA_DQ_PF=1|2, causal), and the dK/dV pass with decoupled halves
    (DSTACK_AMD_FA_DKDV_DEC=1, with and without a stagger; bit-identical to the barrier form with fp32
    partials), and the default pass with fp32 instead of bf16 per-query-head dK/dV partials
    (DSTACK_AMD_FA_DKDV_BF16=0).  The switches are read once per process, so each variant runs in a
    child process."""
    import os
    import subprocess
    import sys

    B, S, H, KV, D = 1, 1024, 8, 2, 128
    script = (
        "import sys, torch\n"
        "from dstack_amd import ops\n"
        "g = torch.Generator(device='cuda').manual_seed(0)\n"
        "S, causal = int(sys.argv[2]), sys.argv[3] == '1'\n"
        f"x = torch.randn({B}, S, {(H + 2 * KV) * D}, device='cuda', generator=g).bfloat16().requires_grad_()\n"
        f"do = torch.randn({B}, S, {H * D}, device='cuda', generator=g).bfloat16()\n"
        f"o = ops.attention(x, {H}, {KV}, causal=causal)\n"
        "o.backward(do)\n"
        "torch.save({'o': o.detach().cpu(), 'g': x.grad.cpu()}, sys.argv[1])\n"
    )
    shape = {"dq_ds_1152": (1152, True), "dq_ds_1152_nc": (1152, False), "default_1152": (1152, True),
             "default_1152_nc": (1152, False), "dkdv_gqa_nc": (1024, False), "default_nc": (1024, False),
             "dkdv_pf0_nc": (1024, False), "dkdv_dec_nc": (1024, False), "dkdv_dec_1152": (1152, True),
             "p32_1152": (1152, True), "p32_nc": (1024, False), "p32_1152_nc": (1152, False)}
    variants = {"default": {}, "dkdv4": {"DSTACK_AMD_FA_DKDV": "4w"},
                "fwd4_dq4": {"DSTACK_AMD_FA_FWD_WAVES": "4", "DSTACK_AMD_FA_DQ_WAVES": "4"},
                "fwd_pf0": {"DSTACK_AMD_FA_FWD_PF": "0"}, "exact_max": {"DSTACK_AMD_FA_RESCALE_THR": "0"},
                "fwd_stag": {"DSTACK_AMD_FA_FWD_STAG": "1"}, "half_prio": {"DSTACK_AMD_FA_HALF_PRIO": "1"},
                "dq_ds": {"DSTACK_AMD_FA_DQ": "ds"}, "dq_ds_1152": {"DSTACK_AMD_FA_DQ": "ds"},
                "dq_ds_1152_nc": {"DSTACK_AMD_FA_DQ": "ds"}, "default_1152": {}, "default_1152_nc": {},
                "dkdv_gqa": {"DSTACK_AMD_FA_DKDV_GQA": "1"}, "dkdv_gqa_nc": {"DSTACK_AMD_FA_DKDV_GQA": "1"},
                "default_nc": {}, "dkdv_pf0": {"DSTACK_AMD_FA_DKDV_PF": "0"},
                "dkdv_pf1": {"DSTACK_AMD_FA_DKDV_PF": "1"}, "dkdv_pf0_nc": {"DSTACK_AMD_FA_DKDV_PF": "0"},
                "dq_pf1": {"DSTACK_AMD_FA_DQ_PF": "1"}, "dq_pf2": {"DSTACK_AMD_FA_DQ_PF": "2"},
                "dkdv_dec": {"DSTACK_AMD_FA_DKDV_DEC": "1"},
                "dkdv_dec_stag": {"DSTACK_AMD_FA_DKDV_DEC": "1", "DSTACK_AMD_FA_DKDV_STAG": "24"},
                "dkdv_dec_nc": {"DSTACK_AMD_FA_DKDV_DEC": "1"}, "dkdv_dec_1152": {"DSTACK_AMD_FA_DKDV_DEC": "1"},
                "dkdv_dec_early": {"DSTACK_AMD_FA_DKDV_DEC": "2"},
                "p32": {"DSTACK_AMD_FA_DKDV_BF16": "0"}, "p32_1152": {"DSTACK_AMD_FA_DKDV_BF16": "0"},
                "p32_nc": {"DSTACK_AMD_FA_DKDV_BF16": "0"}, "p32_1152_nc": {"DSTACK_AMD_FA_DKDV_BF16": "0"}}
    out = {}
    for name, extra in variants.items():
        env = dict(os.environ)
        for k in ("DSTACK_AMD_FA_DKDV", "DSTACK_AMD_FA_FWD_WAVES", "DSTACK_AMD_FA_DQ_WAVES", "DSTACK_AMD_FA_FWD_PF",
                  "DSTACK_AMD_FA_RESCALE_THR", "DSTACK_AMD_FA_FWD_STAG", "DSTACK_AMD_FA_HALF_PRIO", "DSTACK_AMD_FA_DQ",
                  "DSTACK_AMD_FA_DKDV_GQA", "DSTACK_AMD_FA_DKDV_PF", "DSTACK_AMD_FA_DQ_PF", "DSTACK_AMD_FA_DKDV_DEC",
                  "DSTACK_AMD_FA_DKDV_STAG", "DSTACK_AMD_FA_DKDV_BF16"):
            env.pop(k, None)
        env.update(extra)
        sn, causal = shape.get(name, (S, True))
        subprocess.run([sys.executable, "-c", script, str(tmp_path / f"{name}.pt"), str(sn), "1" if causal else "0"],
                       env=env, check=True,
                       timeout=300, cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        out[name] = torch.load(tmp_path / f"{name}.pt", weights_only=True)
    # variants of the forward / dQ passes keep the default dK/dV pass (bf16 partials) and are compared
    # with the default; the other dK/dV forms keep fp32 partials and are compared with the default pass
    # in that form
    for name in ("dkdv4", "fwd4_dq4", "fwd_pf0", "exact_max", "fwd_stag", "half_prio", "dq_ds", "dkdv_gqa",
                 "dkdv_pf0", "dkdv_pf1", "dq_pf1", "dq_pf2", "dkdv_dec", "dkdv_dec_stag"):
        ref = "default" if name in ("fwd4_dq4", "fwd_pf0", "exact_max", "fwd_stag", "dq_pf1", "dq_pf2") else "p32"
        ref_o, ref_g = out[ref]["o"].float(), out[ref]["g"].float()
        o, g = out[name]["o"].float(), out[name]["g"].float()
        assert ((o - ref_o).norm() / ref_o.norm()).item() < 2e-3, name
        assert ((g - ref_g).norm() / ref_g.norm()).item() < 2e-3, name
    for name in ("dkdv_gqa_nc", "dkdv_pf0_nc", "dkdv_dec_nc"):
        g, rg = out[name]["g"].float(), out["p32_nc"]["g"].float()
        assert ((g - rg).norm() / rg.norm()).item() < 2e-3, name
    # bf16 partials (the default): one more bf16 rounding of each per-head partial before the
    # group sum, as flash-attention 2 stores its GQA partials
    for name, ref in (("default", "p32"), ("default_nc", "p32_nc"), ("default_1152", "p32_1152")):
        g, rg = out[name]["g"].float(), out[ref]["g"].float()
        assert ((g - rg).norm() / rg.norm()).item() < 4e-3, name
    # the decoupled dK/dV computes exactly what the barrier form does (both with fp32 partials):
    # identical gradients
    assert torch.equal(out["dkdv_dec"]["g"], out["p32"]["g"])
    assert torch.equal(out["dkdv_dec_stag"]["g"], out["p32"]["g"])
    assert torch.equal(out["dkdv_dec_early"]["g"], out["p32"]["g"])
    assert torch.equal(out["dkdv_dec_1152"]["g"], out["p32_1152"]["g"])
    # bf16 partials change only the K and V gradient columns, by at most a bf16 rounding of a partial
    qcols = H * D
    assert torch.equal(out["p32"]["g"][..., :qcols], out["default"]["g"][..., :qcols])
    assert not torch.equal(out["p32"]["g"], out["default"]["g"])
    for name in ("dq_ds_1152", "dq_ds_1152_nc"):  # the dS-spill dK/dV pass keeps fp32 partials
        ref = out[name.replace("dq_ds", "p32")]
        g, rg = out[name]["g"].float(), ref["g"].float()
        assert torch.isfinite(g).all(), name
        assert ((g - rg).norm() / rg.norm()).item() < 2e-3, name


@pytest.mark.parametrize("T,P,Q", [(64, 256, 256), (512, 768, 512), (1024, 512, 1280)])
@pytest.mark.parametrize("accumulate", [False, True])
def test_weight_grad_gemm_tn(gpu, T, P, Q, accumulate):
    """HIP gemm_tn (dW = g^T x) against an fp32 matmul, incl. accumulation into bf16."""
    C = _ext.require()
    assert C.gemm_tn_supported(P, Q, T)
    g = _rand(T, P, device=gpu, seed=3)
    x = _rand(T, Q, device=gpu, seed=4)
    base = _rand(P, Q, device=gpu, seed=5)
    out = base.clone()
    ops.weight_grad(g, x, out, accumulate=accumulate)
    refv = g.float().t() @ x.float() + (base.float() if accumulate else 0)
    err = ((out.float() - refv).norm() / refv.norm()).item()
    assert err < 4e-3, err


def test_weight_grad_strided_rows(gpu):
    """Row-strided views (a column slice of a wider buffer) are consumed in place."""
    T, P, Q = 256, 512, 256
    gw = _rand(T, P + 128, device=gpu, seed=6)
    xw = _rand(T, Q + 64, device=gpu, seed=7)
    g, x = gw[:, 64:64 + P], xw[:, :Q]
    out = torch.empty(P, Q, device=gpu, dtype=torch.bfloat16)
    ops.weight_grad(g, x, out)
    refv = g.float().t() @ x.float()
    assert ((out.float() - refv).norm() / refv.norm()).item() < 4e-3


@pytest.mark.parametrize("R,C", [(128, 64), (256, 4096), (8192, 192)])
def test_transpose2d(gpu, R, C):
    Cx = _ext.require()
    x = _rand(R, C, device=gpu, seed=8)
    assert torch.equal(Cx.transpose2d(x), x.t().contiguous())


@pytest.mark.parametrize("T,P,Q", [(256, 128, 512), (512, 1024, 256), (384, 200, 256)])
def test_linear_wgrad_layouts_agree(gpu, T, P, Q, monkeypatch):
    """dW through the token-contiguous operands (transposed x and, when P <= Q, g) equals the
    token-major GEMM; a shape the transpose kernel does not tile (P=200) keeps g token-major."""
    x = _rand(T, Q, device=gpu, seed=9).requires_grad_()
    w = _rand(P, Q, device=gpu, seed=10, scale=0.05).requires_grad_()
    g = _rand(T, P, device=gpu, seed=11)
    grads = {}
    for mode in ("auto", "strided", "km"):  # km: the in-tree KM-form GEMM where it tiles the shape
        monkeypatch.setenv("DSTACK_AMD_WGRAD", mode)
        x.grad = w.grad = None
        ops.linear(x, w).backward(g)
        grads[mode] = (x.grad.clone(), w.grad.clone())
    refw = g.float().t() @ x.detach().float()
    for mode, (_, gw) in grads.items():
        assert ((gw.float() - refw).norm() / refw.norm()).item() < 4e-3, mode
    assert torch.equal(grads["auto"][0], grads["strided"][0])


def test_linear_on_in_tree_nt_gemm(gpu, monkeypatch):
    """DSTACK_AMD_LINEAR_NT=1: the projection's forward (and a tiled shape's input gradient) on the
    in-tree NT GEMM match the fp32 reference; an untiled shape falls back to the library."""
    monkeypatch.setenv("DSTACK_AMD_LINEAR_NT", "1")
    for T, P, Q in ((512, 256, 384), (300, 256, 384)):
        x = _rand(T, Q, device=gpu, seed=15).requires_grad_()
        w = _rand(P, Q, device=gpu, seed=16, scale=0.05).requires_grad_()
        g = _rand(T, P, device=gpu, seed=17)
        y = ops.linear(x, w)
        ref_y = x.detach().float() @ w.detach().float().t()
        assert ((y.float() - ref_y).norm() / ref_y.norm()).item() < 4e-3, (T, P, Q)
        y.backward(g)
        ref_gx = g.float() @ w.detach().float()
        assert ((x.grad.float() - ref_gx).norm() / ref_gx.norm()).item() < 4e-3, (T, P, Q)


def test_swiglu_fwd_t_matches(gpu):
    Cx = _ext.require()
    gu = _rand(256, 2 * 192, device=gpu, seed=12)
    a, aT = Cx.swiglu_fwd_t(gu)
    assert torch.equal(a, Cx.swiglu_fwd(gu))
    assert torch.equal(aT, a.t().contiguous())


def test_swiglu_down_chain_wgrad_modes_agree(gpu, monkeypatch):
    """swiglu -> linear(down): the fused transposed SwiGLU output feeding the down projection's
    weight gradient gives the same gradients as the token-major path."""
    T, F, D = 256, 192, 128
    gu = _rand(T, 2 * F, device=gpu, seed=13).requires_grad_()
    w = _rand(D, F, device=gpu, seed=14, scale=0.05).requires_grad_()
    g = _rand(T, D, device=gpu, seed=15)
    res = {}
    for mode in ("auto", "strided"):
        monkeypatch.setenv("DSTACK_AMD_WGRAD", mode)
        gu.grad = w.grad = None
        a = ops.swiglu(gu)
        assert hasattr(a, "_dsa_t") == (mode == "auto")
        ops.linear(a, w).backward(g)
        res[mode] = (gu.grad.clone(), w.grad.clone())
    assert torch.equal(res["auto"][0], res["strided"][0])
    ra, rs = res["auto"][1].float(), res["strided"][1].float()
    assert ((ra - rs).norm() / rs.norm()).item() < 4e-3


def test_rms_norm_bwd_writes_weight_grad_in_place(gpu):
    """rms_norm_bwd(dw_out=..., accumulate) writes/accumulates the bf16 weight gradient in place."""
    Cx = _ext.require()
    T, D = 256, 512
    x = _rand(T, D, device=gpu, seed=18)
    w = _rand(D, device=gpu, seed=19) + 1
    dy = _rand(T, D, device=gpu, seed=20)
    _, rstd = Cx.rms_norm_fwd(x, w, 1e-5)
    dx_ref, dw_ref = Cx.rms_norm_bwd(dy, x, w, rstd)
    out = torch.full((D,), 7.0, device=gpu, dtype=torch.bfloat16)
    dx, _ = Cx.rms_norm_bwd(dy, x, w, rstd, None, out, False)
    assert torch.equal(dx, dx_ref)
    _close(out, dw_ref, 5e-2, 1e-2)
    Cx.rms_norm_bwd(dy, x, w, rstd, None, out, True)
    _close(out, 2 * dw_ref, 1e-1, 1e-2)


@pytest.mark.parametrize("accumulate", [False, True])
def test_embedding_bwd_matches_fp32_scatter(gpu, accumulate):
    """Sorted segment-sum kernel vs an fp32 index_add: repeated ids (a small vocab forces many
    repeats) summed in fp32, written (or added) into bf16 rows; untouched rows cleared/kept."""
    C = _ext.require()
    V, D, T = 512, 4096, 8192
    g = torch.Generator(device=gpu).manual_seed(3)
    tok = torch.randint(0, V // 2, (T,), device=gpu, generator=g)  # rows >= V/2 never touched
    dy = _rand(T, D, device=gpu, seed=4)
    base = _rand(V, D, device=gpu, seed=5)
    grad = base.clone()
    s, order = torch.sort(tok, stable=True)
    C.embedding_bwd(dy, s, order, grad, accumulate)
    want = torch.zeros(V, D, device=gpu, dtype=torch.float32).index_add_(0, tok, dy.float())
    if accumulate:
        want += base.float()
    _close(grad, want, 0.05, 1e-2)
    assert torch.equal(grad[V // 2:], base[V // 2:] if accumulate else torch.zeros_like(base[V // 2:]))
    # deterministic: the same call again gives the same bits
    grad2 = base.clone()
    C.embedding_bwd(dy, s, order, grad2, accumulate)
    assert torch.equal(grad, grad2)


def test_embedding_autograd_matches_torch(gpu):
    V, D = 1000, 512
    w = _rand(V, D, device=gpu, seed=6).requires_grad_()
    tok = torch.randint(0, V, (2, 384), device=gpu)
    y = ops.embedding(tok, w)
    dy = _rand(2, 384, D, device=gpu, seed=7)
    y.backward(dy)
    wr = w.detach().float().requires_grad_()
    torch.nn.functional.embedding(tok, wr).backward(dy.float())
    assert torch.equal(y, w.detach()[tok])
    _close(w.grad, wr.grad, 0.03, 1e-2)


def test_swiglu_bwd_t_matches(gpu):
    Cx = _ext.require()
    gu = _rand(256, 2 * 192, device=gpu, seed=21)
    da = _rand(256, 192, device=gpu, seed=22)
    dgu, dguT = Cx.swiglu_bwd_t(da, gu)
    assert torch.equal(dgu, Cx.swiglu_bwd(da, gu))
    assert torch.equal(dguT, dgu.t().contiguous())


def test_gate_up_chain_wgrad_modes_agree(gpu, monkeypatch):
    """linear(gate_up) -> swiglu: SwiGLU backward's dgu^T feeds the gate/up weight gradient
    (token-contiguous operands); gradients equal the token-major path's."""
    T, F, D = 256, 192, 128
    x = _rand(T, D, device=gpu, seed=23).requires_grad_()
    w = _rand(2 * F, D, device=gpu, seed=24, scale=0.05).requires_grad_()
    g = _rand(T, F, device=gpu, seed=25)
    res = {}
    seen = []
    orig = ops.functional.wgrad_operands

    def spy(g2, x2, xT=None, gT=None):
        seen.append(gT is not None)
        return orig(g2, x2, xT=xT, gT=gT)

    monkeypatch.setattr(ops.functional, "wgrad_operands", spy)
    for mode in ("auto", "strided"):
        monkeypatch.setenv("DSTACK_AMD_WGRAD", mode)
        x.grad = w.grad = None
        ops.swiglu(ops.linear(x, w)).backward(g)
        res[mode] = (x.grad.clone(), w.grad.clone())
    assert seen == [True, False], seen  # the transposed gradient reached the weight-gradient GEMM
    assert torch.equal(res["auto"][0], res["strided"][0])
    ra, rs = res["auto"][1].float(), res["strided"][1].float()
    assert ((ra - rs).norm() / rs.norm()).item() < 4e-3


def test_linear_dgrad_uses_transposed_weight_per_generation(gpu, monkeypatch):
    """With a weight generation published (ZeroOptimizer), linear's input gradient runs on a cached
    W^T; the cache is rebuilt when the generation changes, so an updated weight is never stale."""
    T, N, K = 256, 384, 256
    gen = [0]
    w = _rand(N, K, device=gpu, seed=26, scale=0.05).requires_grad_()
    w._dsa_wgen = lambda: gen[0]
    x = _rand(T, K, device=gpu, seed=27).requires_grad_()
    g = _rand(T, N, device=gpu, seed=28)
    ops.linear(x, w).backward(g)
    assert w._dsa_wt[0] == 0 and torch.equal(w._dsa_wt[1], w.detach().t().contiguous())
    _close(x.grad, g.float() @ w.detach().float(), 0.05, 1e-2)
    with torch.no_grad():
        w.mul_(-2.0)
    gen[0] = 1
    x.grad = None
    ops.linear(x, w).backward(g)
    assert w._dsa_wt[0] == 1
    _close(x.grad, g.float() @ w.detach().float(), 0.05, 1e-2)
    monkeypatch.setenv("DSTACK_AMD_DGRAD_WT", "0")
    gx_nn = torch.autograd.grad(ops.linear(x, w), x, g)[0]
    _close(x.grad, gx_nn, 0.05, 1e-2)


# ---- in-tree NT GEMM (csrc/gemm_nt.hip) and its SwiGLU epilogues ---------------------------------
@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (512, 768, 256), (2304, 9472, 128), (4096, 4352, 384)])
@pytest.mark.parametrize("accumulate", [False, True])
def test_gemm_nt_matches_fp32(gpu, M, N, K, accumulate):
    """C (+)= A B^T against an fp32 matmul; (2304, 9472) and (4096, 4352) have more tiles than CUs
    (persistent workgroups, XCD slices of unequal size)."""
    C = _ext.require()
    a, b = _rand(M, K, device=gpu), _rand(N, K, device=gpu, seed=1)
    out = _rand(M, N, device=gpu, seed=2) if accumulate else torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    ref_ = (out.float() if accumulate else 0) + a.float() @ b.float().t()
    C.gemm_nt(a, b, out, accumulate)
    err = ((out.float() - ref_).norm() / ref_.norm()).item()
    assert err < 5e-3, err


def test_gemm_nt_strided_operands(gpu):
    """Row strides larger than K / N (views into wider buffers) for A, B and C."""
    C = _ext.require()
    M, N, K = 512, 512, 256
    A = _rand(M, K + 64, device=gpu)[:, 32:32 + K]
    B = _rand(N, K + 128, device=gpu, seed=1)[:, :K]
    Cbig = torch.zeros(M, N + 256, device=gpu, dtype=torch.bfloat16)
    out = Cbig[:, 128:128 + N]
    C.gemm_nt(A, B, out, False)
    ref_ = A.float() @ B.float().t()
    assert ((out.float() - ref_).norm() / ref_.norm()).item() < 5e-3
    assert Cbig[:, :128].abs().max().item() == 0 and Cbig[:, 128 + N:].abs().max().item() == 0


def test_gemm_nt_swiglu_epilogue_matches_fp32(gpu):
    """gu, a = silu(g) * u and a^T from one GEMM against the fp32 reference (and exactly the
    separate SwiGLU kernel applied to the same gu)."""
    C = _ext.require()
    T, D, F = 1024, 512, 768
    x, w = _rand(T, D, device=gpu), _rand(2 * F, D, device=gpu, seed=1, scale=0.05)
    gu, a, aT = C.gemm_nt_swiglu(x, w)
    gur = x.float() @ w.float().t()
    assert ((gu.float() - gur).norm() / gur.norm()).item() < 5e-3
    ar = ref.swiglu(gur)
    assert ((a.float() - ar).norm() / ar.norm()).item() < 1e-2
    assert torch.equal(aT, a.t().contiguous())
    a2, aT2 = C.swiglu_fwd_t(gu)
    assert torch.equal(a, a2) and torch.equal(aT, aT2)


def test_gemm_nt_swiglu_bwd_epilogue_matches_fp32(gpu):
    C = _ext.require()
    T, D, F = 1024, 512, 768
    dy, wdT = _rand(T, D, device=gpu), _rand(F, D, device=gpu, seed=1, scale=0.05)
    gu = _rand(T, 2 * F, device=gpu, seed=2)
    dgu, dguT = C.gemm_nt_swiglu_bwd(dy, wdT, gu)
    gur = gu.float().requires_grad_()
    da = dy.float() @ wdT.float().t()
    ref.swiglu(gur).backward(da)
    assert ((dgu.float() - gur.grad).norm() / gur.grad.norm()).item() < 1e-2
    assert torch.equal(dguT, dgu.t().contiguous())


# the step's own reduction lengths (K = 4096 model dim, 14336 FFN dim, 8192 tokens for the weight
# gradients): the unit tests above stop at K <= 1024; long K exercises the ring's steady state and
# the accumulation error over many K-tiles
@pytest.mark.parametrize("M,N,K", [(2048, 4096, 4096), (1024, 4096, 14336)])
def test_gemm_nt_long_k_matches_fp32(gpu, M, N, K):
    C = _ext.require()
    a, b = _rand(M, K, device=gpu, scale=0.5), _rand(N, K, device=gpu, seed=1, scale=0.5)
    out = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    C.gemm_nt(a, b, out, False)
    ref_ = a.float() @ b.float().t()
    assert ((out.float() - ref_).norm() / ref_.norm()).item() < 5e-3


def test_gemm_nt_swiglu_epilogues_long_k(gpu):
    """The fused MLP epilogues at the step's K: gate/up (K = 4096) with SwiGLU, and the down
    projection's input gradient (K = 4096, F = 14336 columns) with the SwiGLU backward."""
    C = _ext.require()
    T, D, F = 1024, 4096, 1792
    x, w = _rand(T, D, device=gpu), _rand(2 * F, D, device=gpu, seed=1, scale=0.02)
    gu, a, _ = C.gemm_nt_swiglu(x, w, False)
    gur = x.float() @ w.float().t()
    assert ((gu.float() - gur).norm() / gur.norm()).item() < 5e-3
    ar = ref.swiglu(gur)
    assert ((a.float() - ar).norm() / ar.norm()).item() < 1e-2
    dy, wdT = _rand(T, D, device=gpu, seed=3), _rand(F, D, device=gpu, seed=4, scale=0.02)
    dgu, _ = C.gemm_nt_swiglu_bwd(dy, wdT, gu, False)
    g2 = gu.float().requires_grad_()
    ref.swiglu(g2).backward(dy.float() @ wdT.float().t())
    assert ((dgu.float() - g2.grad).norm() / g2.grad.norm()).item() < 1e-2


@pytest.mark.parametrize("M,N", [(4096, 4096), (4096, 14336)])
def test_gemm_km_k8192_matches_fp32(gpu, M, N):
    """Weight gradients at the bench's 8192 tokens per micro-batch (KM form, ds_read_b64_tr_b16)."""
    C = _ext.require()
    K = 8192
    a, b = _rand(K, M, device=gpu, scale=0.5), _rand(K, N, device=gpu, seed=1, scale=0.5)
    out = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    C.gemm_km(a, b, out, 0)
    ref_ = a.float().t() @ b.float()
    assert ((out.float() - ref_).norm() / ref_.norm()).item() < 5e-3


@pytest.mark.parametrize("M,N,K,accumulate", [(256, 256, 128, False), (768, 512, 384, True),
                                               (2304, 9472, 256, False), (1024, 4352, 1024, True)])
def test_gemm_km_matches_fp32(gpu, M, N, K, accumulate):
    """KM form (weight gradient of token-major operands): C (+)= A^T B for A [K][M], B [K][N],
    fragments by ds_read_b64_tr_b16, against an fp32 matmul."""
    C = _ext.require()
    a, b = _rand(K, M, device=gpu), _rand(K, N, device=gpu, seed=1)
    out = _rand(M, N, device=gpu, seed=2) if accumulate else torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    ref_ = (out.float() if accumulate else 0) + a.float().t() @ b.float()
    C.gemm_km(a, b, out, 1 if accumulate else 0)
    err = ((out.float() - ref_).norm() / ref_.norm()).item()
    assert err < 5e-3, err


@pytest.mark.parametrize("M,N", [(1024, 4096), (4096, 1024)])
def test_gemm_km_grad_accumulation_8_micro_batches_k8192(gpu, M, N):
    """Weight gradients over 8 micro-batches of 8192 tokens (the bench's step): the bf16 path
    (gemm_km, accumulate=1 seven times, a bf16 rounding per micro-batch) and the fp32-accumulator
    path (gemm_km_f32: modes 0, 1 x 6, 2 -- one rounding), both against the fp32 sum of the eight
    fp32 products.  The fp32 path must be at the single-rounding level and below the bf16 path."""
    C = _ext.require()
    K, n = 8192, 8
    ref_ = torch.zeros(M, N, device=gpu, dtype=torch.float32)
    out16 = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    out32 = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    acc = torch.empty(M, N, device=gpu, dtype=torch.float32)
    for i in range(n):
        # dY-like operands: scaled by 1/n, as the bench's loss / grad_accum does
        a = _rand(K, M, device=gpu, seed=10 + i, scale=1.0 / n)
        b = _rand(K, N, device=gpu, seed=100 + i)
        ref_ += a.float().t() @ b.float()
        C.gemm_km(a, b, out16, 1 if i else 0)
        C.gemm_km_f32(a, b, acc, out32 if i == n - 1 else None, 2 if i == n - 1 else (1 if i else 0))
    e16 = ((out16.float() - ref_).norm() / ref_.norm()).item()
    e32 = ((out32.float() - ref_).norm() / ref_.norm()).item()
    one = ((ref_.bfloat16().float() - ref_).norm() / ref_.norm()).item()  # one bf16 rounding
    print(f"rel err bf16-accumulated {e16:.3e}, fp32-accumulated {e32:.3e}, one rounding {one:.3e}")
    assert e32 < 1.2 * one + 1e-5, (e32, one)
    assert e32 < e16, (e32, e16)
    assert e16 < 8e-3, e16


def test_gemm_km_f32_modes_and_strides(gpu):
    """gemm_km_f32 mode 0 stores fp32, mode 1 adds, mode 2 writes bf16(acc + product) into a strided
    bf16 view without touching its neighbours; the accumulator may be a strided fp32 view too."""
    C = _ext.require()
    M, N, K = 512, 256, 256
    a, b = _rand(K, M, device=gpu), _rand(K, N, device=gpu, seed=1)
    prod = a.float().t() @ b.float()
    big = torch.zeros(M, N + 128, device=gpu, dtype=torch.float32)
    acc = big[:, 64:64 + N]
    C.gemm_km_f32(a, b, acc, None, 0)
    assert ((acc - prod).norm() / prod.norm()).item() < 1e-5
    C.gemm_km_f32(a, b, acc, None, 1)
    assert ((acc - 2 * prod).norm() / prod.norm()).item() < 2e-5
    assert big[:, :64].abs().max().item() == 0 and big[:, 64 + N:].abs().max().item() == 0
    obig = torch.zeros(M, N + 256, device=gpu, dtype=torch.bfloat16)
    out = obig[:, 128:128 + N]
    C.gemm_km_f32(a, b, acc, out, 2)
    assert ((out.float() - 3 * prod).norm() / (3 * prod).norm()).item() < 3e-3
    assert obig[:, :128].abs().max().item() == 0 and obig[:, 128 + N:].abs().max().item() == 0


def test_gemm_km_strided_operands(gpu):
    """Row strides wider than M / N (views into wider buffers) for A, B and C."""
    C = _ext.require()
    M, N, K = 512, 256, 256
    A = _rand(K, M + 64, device=gpu)[:, 32:32 + M]
    B = _rand(K, N + 128, device=gpu, seed=1)[:, :N]
    Cbig = torch.zeros(M, N + 256, device=gpu, dtype=torch.bfloat16)
    out = Cbig[:, 128:128 + N]
    C.gemm_km(A, B, out)
    ref_ = A.float().t() @ B.float()
    assert ((out.float() - ref_).norm() / ref_.norm()).item() < 5e-3
    assert Cbig[:, :128].abs().max().item() == 0 and Cbig[:, 128 + N:].abs().max().item() == 0


def test_gemm_nt_swiglu_epilogues_without_transposes(gpu):
    """The barrier-free SwiGLU epilogues (no a^T / dgu^T) write exactly what the transposing ones do."""
    C = _ext.require()
    T, D, F = 1024, 512, 768
    x, w = _rand(T, D, device=gpu), _rand(2 * F, D, device=gpu, seed=1, scale=0.05)
    gu, a, _ = C.gemm_nt_swiglu(x, w)
    gu2, a2, aT2 = C.gemm_nt_swiglu(x, w, False)
    assert torch.equal(gu, gu2) and torch.equal(a, a2) and aT2.numel() == 0
    dy, wdT = _rand(T, D, device=gpu, seed=3), _rand(F, D, device=gpu, seed=4, scale=0.05)
    dgu, _ = C.gemm_nt_swiglu_bwd(dy, wdT, gu)
    dgu2, dguT2 = C.gemm_nt_swiglu_bwd(dy, wdT, gu, False)
    assert dguT2.numel() == 0
    # same formulas; the compiler may contract them differently: at most a bf16 rounding apart
    assert ((dgu.float() - dgu2.float()).norm() / dgu.float().norm()).item() < 1e-3


@pytest.mark.parametrize("wgrad", ["auto", "km"])
def test_swiglu_mlp_fused_matches_separate_kernels(gpu, monkeypatch, wgrad):
    """ops.swiglu_mlp through the fused GEMM epilogues == linear/swiglu/linear with separate kernels,
    output and every gradient (no optimizer sinks: the gradients are returned); ``km``: weight
    gradients by the in-tree KM-form GEMM on token-major operands, no transposed copies."""
    monkeypatch.setenv("DSTACK_AMD_WGRAD", wgrad)
    T, D, F = 512, 512, 1024
    torch.manual_seed(0)
    h0 = _rand(2, T // 2, D, device=gpu)
    wgu0 = _rand(2 * F, D, device=gpu, seed=1, scale=0.03)
    wd0 = _rand(D, F, device=gpu, seed=2, scale=0.03)
    dy = _rand(2, T // 2, D, device=gpu, seed=3)

    def run():
        h, wgu, wd = (t.clone().requires_grad_() for t in (h0, wgu0, wd0))
        y = ops.swiglu_mlp(h, wgu, wd)
        y.backward(dy)
        return y.float(), h.grad.float(), wgu.grad.float(), wd.grad.float()

    assert ops.functional._mlp_fused_ok(h0, wgu0, wd0)
    fused = run()
    monkeypatch.setenv("DSTACK_AMD_MLP_FUSED", "0")
    monkeypatch.setenv("DSTACK_AMD_WGRAD", "auto")
    sep = run()
    for name, a, b in zip(["y", "dh", "dWgu", "dWdown"], fused, sep):
        rel = ((a - b).norm() / (b.norm() + 1e-12)).item()
        assert rel < 1e-2, f"{name}: rel err {rel}"


@pytest.mark.parametrize("M,N,K,bm,split", [(256, 256, 512, 64, 1), (37, 384, 512, 64, 1), (200, 256, 1024, 128, 2),
                                             (1, 128, 256, 64, 1), (64, 1024, 384, 64, 1), (256, 512, 1024, 128, 1),
                                             (130, 256, 2048, 128, 4), (256, 1024, 512, 64, 2)])
@pytest.mark.parametrize("wimg", [False, True])
def test_fp8_rows_gemm_matches_fp32(gpu, M, N, K, bm, split, wimg):
    """Decode-batch fp8 GEMM (csrc/fp8_gemm.hip: scaled 16x16x128 f8f6f4 MFMA over 64/128-row batch
    blocks, optional split-K with a last-arrival combine; weights row-major or as per-tile LDS images,
    ops.serving.fp8_rows_shuffle) against the fp32 product of the same e4m3 operands and scales;
    twice, since the split-K tickets must be left at zero."""
    from dstack_amd.ops.serving import fp8_rows_shuffle

    C = _ext.require()
    torch.manual_seed(M + N + K)
    x = torch.randn(M, K, device=gpu, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=gpu, dtype=torch.bfloat16) * 0.05
    xq, xs = ref.quant_fp8_rows(x)
    wq, ws = ref.quant_fp8_rows(w)
    want = (xq.float() * xs[:, None]) @ (wq.float() * ws[:, None]).t()
    part = torch.empty(split * 256 * N, device=gpu, dtype=torch.float32)
    cnt = torch.zeros((N // 128) * ((M + bm - 1) // bm), device=gpu, dtype=torch.int32)
    wk = fp8_rows_shuffle(wq) if wimg else wq
    for _ in range(2):
        y = C.fp8_rows_gemm(xq.view(torch.uint8), xs, wk.view(torch.uint8), ws, bm, split, part, cnt, wimg)
        err = ((y.float() - want).norm() / want.norm()).item()
        assert err < 1e-2, err
    assert int(cnt.abs().sum().item()) == 0


@pytest.mark.parametrize("shuffled", [0, 1, 2])
@pytest.mark.parametrize("rw", [64, 32, 28])
@pytest.mark.parametrize("M,N,K,split", [(256, 256, 512, 1), (256, 1024, 2048, 1), (200, 256, 2048, 2),
                                         (129, 512, 4096, 4), (256, 512, 8192, 1), (256, 256, 7168, 7),
                                         (256, 448, 2048, 1), (200, 672, 4096, 2)])
def test_fp8_stream_gemm_matches_fp32(gpu, M, N, K, split, rw, shuffled):
    """Weight-streaming decode fp8 GEMM (csrc/fp8_gemm.hip fp8_stream_gemm: each wave's weight rows
    straight into registers two K-steps ahead, activations through an LDS ring; 4 waves x 64 rows,
    8 waves x 32 rows or 7 x 32; optional split-K with a separate reduce; the weights row-major or pre-shuffled
    by ops.serving.fp8_stream_shuffle in 16-row blocks or 256-row groups) against the fp32 product of the same e4m3 operands and row-wise
    scales; padded token rows (M < 256) must not be stored."""
    from dstack_amd.ops.serving import fp8_stream_shuffle

    C = _ext.require()
    if (rw == 64 and split > 1) or N % (224 if rw == 28 else 256):  # not offered (dsa_fp8_stream_gemm_supported)
        assert not C.fp8_stream_gemm_supported(M, N, K, rw, split)
        return
    assert C.fp8_stream_gemm_supported(M, N, K, rw, split)
    torch.manual_seed(M + N + K + split)
    x = torch.randn(M, K, device=gpu, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=gpu, dtype=torch.bfloat16) * 0.05
    xq, xs = ref.quant_fp8_rows(x)
    wq, ws = ref.quant_fp8_rows(w)
    want = (xq.float() * xs[:, None]) @ (wq.float() * ws[:, None]).t()
    wk = fp8_stream_shuffle(wq, {1: 16, 2: 224 if rw == 28 else 256}[shuffled]) if shuffled else wq
    for depth in ([2, 3] if rw == 32 else [2]):
        y = C.fp8_stream_gemm(xq.view(torch.uint8), xs, wk.view(torch.uint8), ws, rw, split, shuffled, depth)
        assert y.shape == (M, N)
        err = ((y.float() - want).norm() / want.norm()).item()
        assert err < 1e-2, err


def test_attention_head_dim_64_runs_sdpa_with_a_warning(gpu):
    """Llama-3.2 1B/3B shapes (head_dim 64) are not tiled by the HIP flash kernels: the op runs
    PyTorch's SDPA for them (warned once per shape) and matches the fp32 reference, forward and
    backward."""
    import warnings as _w

    torch.manual_seed(0)
    H, KVH, D, S = 8, 2, 64, 256
    qkv = _rand(1, S, (H + 2 * KVH) * D, device=gpu).requires_grad_()
    ops.functional._ATTN_FALLBACK_WARNED.discard((D, True))
    with _w.catch_warnings(record=True) as rec:
        _w.simplefilter("always")
        o = ops.attention(qkv, H, KVH)
    assert any("SDPA" in str(r.message) for r in rec)
    q, k, v = ops.functional.split_qkv(qkv.detach().float(), H, KVH)
    want = ref.attention(q, k, v, True).reshape(1, S, -1)
    assert ((o.float() - want).norm() / want.norm()).item() < 2e-2
    o.float().square().sum().backward()
    assert qkv.grad is not None and torch.isfinite(qkv.grad).all()


@pytest.mark.parametrize("mb,S", [(1, 8192), (2, 1023), (1, 64)])
def test_synthetic_tokens_kernel_matches_cpu_reference(gpu, mb, S):
    """The bench's data stream generated by the HIP kernel (csrc/data.hip) is bit-identical to the
    torch definition on the CPU (workloads/data.py), for several (seed, index) keys."""
    from dstack_amd.workloads.data import SyntheticLM

    V = 128256
    g, c = SyntheticLM(V, S, mb, gpu, seed=3), SyntheticLM(V, S, mb, "cpu", seed=3)
    for index in (0, 1, 17, 1 << 40):
        a, b = g.tokens(index).cpu(), c.tokens(index)
        assert a.shape == (mb, S + 1) and torch.equal(a, b), index


def _qkv_rope_ref(h, w, cos, sin, H, KV):
    """fp32 reference of rope(h W^T) on the q and k heads (head_dim 128)."""
    B, S, _ = h.shape
    x = (h.reshape(B * S, -1) @ w.t()).view(B, S, H + 2 * KV, 128)
    return torch.cat([ref.apply_rope(x[:, :, : H + KV], cos, sin), x[:, :, H + KV :]], 2).reshape(B, S, -1)


@pytest.mark.parametrize("B,S,K,H,KV", [(2, 256, 512, 4, 2), (1, 1024, 4096, 32, 8), (1, 8192, 256, 2, 1)])
def test_gemm_nt_rope_epilogue_matches_fp32(gpu, B, S, K, H, KV):
    """The qkv GEMM with RoPE in its epilogue (EPI_ROPE: b1 unit = dims 64-127 of the tile's two
    heads) against fp32 matmul + rotate-half; (1, 8192, ...) reaches the last positions."""
    C = _ext.require()
    N = (H + 2 * KV) * 128
    h = _rand(B, S, K, device=gpu)
    w = _rand(N, K, device=gpu, seed=1, scale=K ** -0.5)
    cos, sin = ref.rope_cos_sin(S, 128, 500000.0, gpu)
    assert C.gemm_nt_rope_supported(B * S, N, K, S, (H + KV) * 128)
    out = C.gemm_nt_rope(h.view(B * S, K), w, cos, sin, S, (H + KV) * 128).view(B, S, N)
    exp = _qkv_rope_ref(h.float(), w.float(), cos, sin, H, KV)
    _close(out, exp, 3e-2, 1e-2)
    # v heads are the plain product
    _close(out[..., (H + KV) * 128:], (h.float().view(B * S, K) @ w.float().t()).view(B, S, N)[..., (H + KV) * 128:],
           3e-2, 1e-2)


@pytest.mark.parametrize("B,S,D,H,KV", [(2, 256, 512, 4, 2), (1, 8192, 1024, 8, 2)])
def test_qkv_rope_attention_fused_matches_fp32(gpu, monkeypatch, B, S, D, H, KV):
    """attention(rope(h Wqkv^T)) with both RoPE passes fused (GEMM epilogue forward, dQ epilogue and
    dK reduction backward) against fp32 autograd, and against the separate-kernel path."""
    monkeypatch.delenv("DSTACK_AMD_QKV_ROPE", raising=False)
    N = (H + 2 * KV) * 128
    h = _rand(B, S, D, device=gpu).requires_grad_()
    w = _rand(N, D, device=gpu, seed=1, scale=D ** -0.5).requires_grad_()
    cos, sin = ref.rope_cos_sin(S, 128, 500000.0, gpu)
    assert ops.functional._qkv_rope_ok(h, w, cos, H, KV)
    o = ops.qkv_rope_attention(h, w, cos, sin, H, KV)
    do = _rand(B, S, H * 128, device=gpu, seed=3)
    o.backward(do)
    hr, wr = h.detach().float().requires_grad_(), w.detach().float().requires_grad_()
    q, k, v = ops.functional.split_qkv(_qkv_rope_ref(hr, wr, cos, sin, H, KV), H, KV)
    orf = ref.attention(q, k, v, True).reshape(B, S, -1)
    orf.backward(do.float())
    _close(o, orf, 2e-2, 2e-2)
    for name, a, b in (("dh", h.grad, hr.grad), ("dw", w.grad, wr.grad)):
        a = a.float()
        rel = ((a - b).norm() / (b.norm() + 1e-12)).item()
        assert rel < 2e-2, f"{name}: rel {rel}"
    # the unfused path (GEMM, rope_qkv, attention, inverse rope_qkv) agrees closely
    monkeypatch.setenv("DSTACK_AMD_QKV_ROPE", "0")
    h2, w2 = h.detach().clone().requires_grad_(), w.detach().clone().requires_grad_()
    o2 = ops.qkv_rope_attention(h2, w2, cos, sin, H, KV)
    o2.backward(do)
    for name, a, b in (("o", o, o2), ("dh", h.grad, h2.grad), ("dw", w.grad, w2.grad)):
        a, b = a.float(), b.float()
        rel = ((a - b).norm() / (b.norm() + 1e-12)).item()
        assert rel < 1e-2, f"fused vs unfused {name}: rel {rel}"


@pytest.mark.parametrize("M,N,K", [(256, 256, 256), (512, 768, 1024), (256, 512, 8192), (768, 256, 28672 // 4)])
def test_gemm_nt_f8_matches_fp32(gpu, M, N, K):
    """The e4m3 form of the 256x256 GEMM (scaled 16x16x128 MFMA, raw product) against the fp32
    product of the same e4m3 values."""
    C = _ext.require()
    assert C.gemm_nt_f8_supported(M, N, K)
    g = torch.Generator(device=gpu).manual_seed(5)
    a = (torch.randn(M, K, device=gpu, generator=g) * 2).to(torch.float8_e4m3fn)
    w = (torch.randn(N, K, device=gpu, generator=g) * 2).to(torch.float8_e4m3fn)
    out = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    C.gemm_nt_f8(a.view(torch.uint8), w.view(torch.uint8), out)
    exp = a.float() @ w.float().t()
    rel = ((out.float() - exp).norm() / exp.norm()).item()
    assert rel < 5e-3, rel
    _close(out, exp, 0.0, 1e-2)


@pytest.mark.parametrize("kind,M,N,K", [("km", 6144, 4096, 8192), ("km", 4096, 14336, 8192), ("km", 1024, 4096, 8192),
                                        ("nt", 2048, 12288, 1024)])
def test_gemm_split_remainder_matches_fp32(gpu, kind, M, N, K):
    """Shapes whose persistent grid ends in a part-filled round (the qkv / down weight gradients:
    1.5 and 3.5 rounds): the last round's tiles run as two K halves plus the fixup kernel.  Every
    epilogue the fixup implements (bf16 store / accumulate, the fp32 accumulator modes) against fp32."""
    C = _ext.require()
    g = torch.Generator(device=gpu).manual_seed(11)
    if kind == "km":  # C[M][N] (+)= A[K][M]^T B[K][N], token-major operands
        a = (torch.randn(K, M, device=gpu, generator=g) * 0.05).bfloat16()
        b = (torch.randn(K, N, device=gpu, generator=g) * 0.05).bfloat16()
        exp = a.float().t() @ b.float()
        out = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
        C.gemm_km(a, b, out, 0)
        _close(out, exp, 0.0, 1e-2)
        base = (torch.randn(M, N, device=gpu, generator=g) * 0.1).bfloat16()
        out.copy_(base)
        C.gemm_km(a, b, out, 1)
        _close(out, exp + base.float(), 0.0, 1e-2)
        acc = torch.empty(M, N, device=gpu, dtype=torch.float32)
        C.gemm_km_f32(a, b, acc, None, 0)
        assert ((acc - exp).norm() / exp.norm()).item() < 1e-5
        C.gemm_km_f32(a, b, acc, None, 1)
        assert ((acc - 2 * exp).norm() / exp.norm()).item() < 2e-5
        C.gemm_km_f32(a, b, acc, out, 2)
        _close(out, 3 * exp, 0.0, 1e-2)
    else:
        a = (torch.randn(M, K, device=gpu, generator=g) * 0.05).bfloat16()
        b = (torch.randn(N, K, device=gpu, generator=g) * 0.05).bfloat16()
        exp = a.float() @ b.float().t()
        out = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
        C.gemm_nt(a, b, out, False)
        _close(out, exp, 0.0, 1e-2)
        base = (torch.randn(M, N, device=gpu, generator=g) * 0.1).bfloat16()
        out.copy_(base)
        C.gemm_nt(a, b, out, True)
        _close(out, exp + base.float(), 0.0, 1e-2)
