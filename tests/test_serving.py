"""Serving engine: HF-Llama parity of the paged prefill/decode path, the native scheduler (pages,
admission, preemption), sampling, top-k/top-p and the OpenAI-compatible HTTP API (CPU), plus the
HIP kernels against their fp32 references and the hipGraph decode path (GPU).

Parity source: ``transformers.LlamaForCausalLM`` (installed) with random weights written by
``save_pretrained`` to a temp dir — the reference orchestrator ships no model code (its services
run vLLM/TGI containers), so HF's Llama is the oracle for the model math."""

import json
import math
import time

import pytest
import torch

from dstack_amd.ops import serving as sops
from dstack_amd.serving._native import Scheduler
from dstack_amd.serving.engine import LLMEngine, SamplingParams, _filter_top_k_top_p
from dstack_amd.serving.model import ServingLlama, load_spec


def _hf_tiny(tmp_path, rope_scaling=None, tie=False, vocab=512):
    transformers = pytest.importorskip("transformers")
    cfg = transformers.LlamaConfig(
        hidden_size=256, intermediate_size=512, num_hidden_layers=2, num_attention_heads=2, num_key_value_heads=1,
        vocab_size=vocab, max_position_embeddings=1024, rope_theta=500000.0, head_dim=128,
        rope_scaling=rope_scaling, tie_word_embeddings=tie, eos_token_id=2, bos_token_id=1)
    torch.manual_seed(0)
    m = transformers.LlamaForCausalLM(cfg).eval()
    with torch.no_grad():  # HF inits norms to 1 and uses std 0.02; widen so logits are not flat
        for p in m.parameters():
            if p.dim() == 2:
                p.normal_(0, 0.08)
    path = tmp_path / "hf"
    m.save_pretrained(str(path))
    return m, str(path)


@pytest.mark.parametrize("variant", ["plain", "llama3_rope", "tied"])
def test_hf_parity_prefill_and_greedy_decode(tmp_path, variant):
    rope = {"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
            "original_max_position_embeddings": 64} if variant == "llama3_rope" else None
    hf, path = _hf_tiny(tmp_path, rope_scaling=rope, tie=variant == "tied")
    eng = LLMEngine.from_model(path, device="cpu", max_model_len=512, max_batch=4, num_pages=32)
    prompts = [[1, 5, 9, 33, 7, 100, 2, 45, 61], [1, 300, 301, 302]]
    # prefill logits == HF logits of the last prompt token
    m = eng.model
    toks = torch.zeros(256, dtype=torch.int64)
    toks[:9] = torch.tensor(prompts[0])
    toks[128:132] = torch.tensor(prompts[1])
    pos = torch.cat([torch.arange(128), torch.arange(128)]).int()
    pos[9:128] = 0
    pos[132:] = 0
    slots = torch.full((256,), -1, dtype=torch.int32)
    slots[:9] = torch.arange(9)
    slots[128:132] = torch.arange(4) + 64
    logits = m.prefill(toks, pos, slots, [0, 128], [9, 4])
    with torch.no_grad():
        for i, p in enumerate(prompts):
            want = hf(torch.tensor([p])).logits[0, -1]
            torch.testing.assert_close(logits[i], want, atol=2e-4, rtol=2e-4)
    # greedy generation through paged decode == HF greedy generate
    outs = eng.generate(prompts, SamplingParams(max_tokens=12, temperature=0, ignore_eos=True))
    for p, r in zip(prompts, outs):
        with torch.no_grad():
            ref = hf.generate(torch.tensor([p]), max_new_tokens=12, do_sample=False, eos_token_id=None,
                              pad_token_id=0)[0, len(p):].tolist()
        assert r.output_ids == ref
        assert r.finish_reason == "length"


def test_checkpoint_loader_rejects_incomplete(tmp_path):
    from safetensors.torch import load_file, save_file

    _, path = _hf_tiny(tmp_path)
    sd = load_file(f"{path}/model.safetensors")
    sd.pop("model.layers.1.mlp.up_proj.weight")
    save_file(sd, f"{path}/model.safetensors")
    m = ServingLlama(load_spec(path), "cpu")
    with pytest.raises(ValueError, match="missing 1 tensors"):
        m.load_hf()


def _hf_family_tiny(tmp_path, family):
    transformers = pytest.importorskip("transformers")
    common = dict(hidden_size=256, intermediate_size=512, num_hidden_layers=2, num_attention_heads=2,
                  num_key_value_heads=1, vocab_size=512, max_position_embeddings=1024, rope_theta=1000000.0,
                  eos_token_id=2, bos_token_id=1)
    if family == "mistral":
        cfg = transformers.MistralConfig(head_dim=128, sliding_window=512, **common)
        cls = transformers.MistralForCausalLM
    else:
        cfg = transformers.Qwen2Config(use_sliding_window=False, **common)
        cls = transformers.Qwen2ForCausalLM
    torch.manual_seed(0)
    m = cls(cfg).eval()
    with torch.no_grad():
        for name, p in m.named_parameters():
            if p.dim() == 2:
                p.normal_(0, 0.08)
            elif name.endswith("bias"):
                p.normal_(0, 0.5)  # Qwen2's q/k/v biases: make them matter
    path = tmp_path / family
    m.save_pretrained(str(path))
    return m, str(path)


@pytest.mark.parametrize("family", ["mistral", "qwen2"])
def test_hf_parity_other_llama_block_families(tmp_path, family):
    """Mistral and Qwen2 (q/k/v biases) checkpoints: greedy decode through the paged engine equals
    the transformers model; a sliding-window Mistral is capped at its window."""
    hf, path = _hf_family_tiny(tmp_path, family)
    spec = load_spec(path)
    assert spec.family == family and spec.qkv_bias == (family == "qwen2")
    if family == "mistral":
        assert spec.cfg.max_seq_len == 512
    eng = LLMEngine.from_model(path, device="cpu", max_model_len=256, max_batch=4, num_pages=32)
    prompts = [[1, 5, 9, 33, 7, 100, 2, 45, 61], [1, 300, 301, 302]]
    outs = eng.generate(prompts, SamplingParams(max_tokens=10, temperature=0, ignore_eos=True))
    for p, r in zip(prompts, outs):
        with torch.no_grad():
            ref = hf.generate(torch.tensor([p]), max_new_tokens=10, do_sample=False, eos_token_id=None,
                              pad_token_id=0)[0, len(p):].tolist()
        assert r.output_ids == ref, (family, r.output_ids, ref)


def test_qwen2_checkpoint_needs_its_biases(tmp_path):
    from safetensors.torch import load_file, save_file

    _, path = _hf_family_tiny(tmp_path, "qwen2")
    sd = load_file(f"{path}/model.safetensors")
    sd.pop("model.layers.0.self_attn.k_proj.bias")
    save_file(sd, f"{path}/model.safetensors")
    with pytest.raises(ValueError, match="missing 1 tensors"):
        ServingLlama(load_spec(path), "cpu").load_hf()


def test_spec_rejects_non_llama(tmp_path):
    (tmp_path / "config.json").write_text(json.dumps({"model_type": "gpt2", "architectures": ["GPT2LMHeadModel"],
                                                      "num_attention_heads": 2, "hidden_size": 256}))
    with pytest.raises(ValueError, match="Llama family"):
        load_spec(str(tmp_path))


# ------------------------------------------------------------------------------------------------
# native scheduler
# ------------------------------------------------------------------------------------------------
def test_scheduler_prefill_then_decode_pages():
    s = Scheduler(num_pages=8, page_size=64, max_batch=4, max_prefill_tokens=512, max_model_len=1024)
    s.add(1, 100, 300)
    s.add(2, 64, 300)
    p = s.schedule()
    assert p["kind"] == "prefill" and list(p["seq_ids"]) == [1, 2]
    assert p["rows"] == 256 and list(p["offsets"]) == [0, 128] and list(p["lens"]) == [100, 64]
    # 100 tokens + 1 -> 2 pages; 64 + 1 -> 2 pages
    assert s.free_pages == 4
    slots = p["slots"]
    pages1 = s.pages(1)
    assert slots[0] == pages1[0] * 64 and slots[99] == pages1[1] * 64 + 35 and slots[100] == -1
    for sid in (1, 2):
        s.mark_computed(sid)
        s.append(sid)
    d = s.schedule()
    assert d["kind"] == "decode"
    assert list(d["positions"]) == [100, 64] and list(d["ctx_lens"]) == [101, 65]
    assert d["block_tables"].shape == (2, 16)
    assert list(d["block_tables"][1][:2]) == s.pages(2)
    s.finish(1)
    assert s.free_pages == 6


def test_scheduler_prefill_budget_and_batch_cap():
    s = Scheduler(num_pages=64, page_size=64, max_batch=3, max_prefill_tokens=256, max_model_len=2048)
    for i in range(5):
        s.add(i, 100, 200)
    p = s.schedule()
    assert list(p["seq_ids"]) == [0, 1]  # 2 x 128 padded rows fill the budget
    p = s.schedule()
    assert list(p["seq_ids"]) == [2]  # max_batch 3
    assert s.num_waiting == 2
    d = s.schedule()
    assert d["kind"] == "decode" and len(d["seq_ids"]) == 3


def test_scheduler_preempts_newest_when_out_of_pages():
    s = Scheduler(num_pages=4, page_size=64, max_batch=4, max_prefill_tokens=4096, max_model_len=1024)
    s.add(1, 63, 1000)
    s.add(2, 63, 1000)
    p = s.schedule()
    assert list(p["seq_ids"]) == [1, 2] and s.free_pages == 2  # 63 prompt tokens + 1 -> one page each
    for sid in (1, 2):
        s.mark_computed(sid)
        s.append(sid)
    for _ in range(200):  # grow both until the pool runs dry
        d = s.schedule()
        if d["preempted"]:
            break
        for sid in d["seq_ids"]:
            s.mark_computed(sid)
            s.append(sid)
    assert list(d["preempted"]) == [2]
    assert list(d["seq_ids"]) == [1] and s.num_waiting == 1
    s.finish(1)
    p = s.schedule()  # the preempted sequence comes back with all its tokens as the prompt
    assert p["kind"] == "prefill" and list(p["seq_ids"]) == [2] and p["lens"][0] == s.num_tokens(2) > 63


def test_scheduler_rejects_bad_requests():
    s = Scheduler(num_pages=2, page_size=64, max_batch=4, max_prefill_tokens=4096, max_model_len=1024)
    with pytest.raises(ValueError):
        s.add(1, 0, 10)
    with pytest.raises(ValueError):
        s.add(1, 200, 300)  # needs 4 pages, pool has 2
    s.add(1, 10, 20)
    with pytest.raises(ValueError):
        s.add(1, 10, 20)


def test_engine_preemption_keeps_greedy_outputs():
    torch.manual_seed(0)
    kw = dict(device="cpu", max_model_len=256, max_batch=8)
    prompts = [[1 + i, 2, 3, 4 + i] * (5 + i) for i in range(4)]
    sp = SamplingParams(max_tokens=60, temperature=0, ignore_eos=True)
    big = LLMEngine.from_model("llama-tiny", num_pages=64, **kw).generate(prompts, sp)
    small_eng = LLMEngine.from_model("llama-tiny", num_pages=5, **kw)
    small = small_eng.generate(prompts, sp)
    assert small_eng.stats["preemptions"] > 0
    assert [r.output_ids for r in small] == [r.output_ids for r in big]


# ------------------------------------------------------------------------------------------------
# tensor parallel (gloo, 2 ranks on the CPU): same tokens as the single-process engine
# ------------------------------------------------------------------------------------------------
def _tp_worker(rank, world, port, model, q):
    import os

    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        eng = LLMEngine.from_model(model, device="cpu", max_model_len=256, max_batch=4, num_pages=24,
                                   tp_group=dist.group.WORLD)
        if rank == 0:
            prompts = [[1, 5, 9, 33, 7, 100, 2, 45, 61], [1, 300, 301, 302], list(range(3, 140))]
            outs = eng.generate(prompts, SamplingParams(max_tokens=10, temperature=0, ignore_eos=True))
            seeded = eng.generate([[4, 5, 6]], SamplingParams(max_tokens=6, temperature=0.9, seed=3, ignore_eos=True))
            eng.shutdown()
            q.put([r.output_ids for r in outs] + [seeded[0].output_ids])
        else:
            eng.follow()
    finally:
        dist.destroy_process_group()


def _hf_tiny_tp(tmp_path, family="llama"):
    transformers = pytest.importorskip("transformers")
    common = dict(hidden_size=512, intermediate_size=1024, num_hidden_layers=2, num_attention_heads=4,
                  num_key_value_heads=2, vocab_size=512, max_position_embeddings=1024, rope_theta=500000.0)
    if family == "qwen2":
        m_cls, cfg = transformers.Qwen2ForCausalLM, transformers.Qwen2Config(use_sliding_window=False, **common)
    else:
        m_cls, cfg = transformers.LlamaForCausalLM, transformers.LlamaConfig(head_dim=128, **common)
    torch.manual_seed(1)
    m = m_cls(cfg)
    with torch.no_grad():
        for name, p in m.named_parameters():
            if p.dim() == 2:
                p.normal_(0, 0.06)
            elif name.endswith("bias"):
                p.normal_(0, 0.5)
    m.save_pretrained(str(tmp_path / "hftp"))
    return str(tmp_path / "hftp")


@pytest.mark.parametrize("source", ["random", "hf", "hf-qwen2"])
def test_tensor_parallel_matches_single_process(tmp_path, source):
    import torch.multiprocessing as mp

    from dstack_amd.server.testing import free_port

    model = "llama-tiny" if source == "random" else _hf_tiny_tp(tmp_path, "qwen2" if source == "hf-qwen2" else "llama")
    single = LLMEngine.from_model(model, device="cpu", max_model_len=256, max_batch=4, num_pages=24)
    prompts = [[1, 5, 9, 33, 7, 100, 2, 45, 61], [1, 300, 301, 302], list(range(3, 140))]
    want = [r.output_ids for r in single.generate(prompts, SamplingParams(max_tokens=10, temperature=0,
                                                                          ignore_eos=True))]
    want.append(single.generate([[4, 5, 6]], SamplingParams(max_tokens=6, temperature=0.9, seed=3,
                                                            ignore_eos=True))[0].output_ids)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_tp_worker, args=(r, 2, port, model, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == want


# ------------------------------------------------------------------------------------------------
# ops references
# ------------------------------------------------------------------------------------------------
def test_paged_decode_ref_matches_dense_attention():
    torch.manual_seed(0)
    H, KVH, B = 8, 2, 3
    k_cache, v_cache = sops.alloc_cache(12, KVH, torch.float32)
    k_cache.normal_()
    v_cache.normal_()
    tables = torch.tensor([[3, 7, 1, 0], [5, 0, 0, 0], [11, 2, 9, 4]], dtype=torch.int32)
    ctx = torch.tensor([150, 1, 256], dtype=torch.int32)
    q = torch.randn(B, (H + 2 * KVH) * 128)
    out = sops.paged_decode(q, k_cache, v_cache, tables, ctx, H, KVH)
    for b in range(B):
        n = int(ctx[b])
        idx = torch.arange(n)
        pages = tables[b][idx // 64].long()
        k = k_cache[pages, :, idx % 64]  # [n, KVH, D]
        v = v_cache[pages, :, :, idx % 64]
        qb = q[b, : H * 128].view(H, 128)
        kk = k.repeat_interleave(H // KVH, dim=1).transpose(0, 1)
        vv = v.repeat_interleave(H // KVH, dim=1).transpose(0, 1)
        p = torch.softmax(torch.einsum("hd,hnd->hn", qb, kk) / math.sqrt(128), -1)
        torch.testing.assert_close(out[b].view(H, 128), torch.einsum("hn,hnd->hd", p, vv))


def test_split_plan_covers_table():
    for B in (1, 4, 64, 256):
        for W in (1, 16, 128, 2048):
            n, pps = sops.split_plan(B, 8, W)
            assert n * pps >= W and (n - 1) * pps < W


def test_sample_ref_greedy_and_logprob():
    logits = torch.randn(4, 100)
    tok, lp = sops.sample(logits, torch.zeros(4), torch.zeros(4, dtype=torch.int64), torch.zeros(4, dtype=torch.int32))
    assert tok.tolist() == logits.argmax(-1).tolist()
    torch.testing.assert_close(lp, torch.log_softmax(logits, -1).max(-1).values)


def test_top_k_top_p_filter():
    class R:
        def __init__(self, k, p):
            self.params = SamplingParams(top_k=k, top_p=p, temperature=1.0)

    logits = torch.log(torch.tensor([[0.5, 0.3, 0.15, 0.05], [0.5, 0.3, 0.15, 0.05], [0.1, 0.2, 0.3, 0.4]]))
    out = _filter_top_k_top_p(logits, [R(2, 1.0), R(0, 0.7), R(0, 1.0)])
    assert torch.isinf(out[0]).tolist() == [False, False, True, True]
    assert torch.isinf(out[1]).tolist() == [False, False, True, True]  # 0.5 + 0.3 >= 0.7
    assert not torch.isinf(out[2]).any()


# ------------------------------------------------------------------------------------------------
# OpenAI-compatible HTTP API
# ------------------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def api():
    from fastapi.testclient import TestClient

    from dstack_amd.serving.server import create_app

    eng = LLMEngine.from_model("llama-tiny", device="cpu", max_model_len=256, max_batch=8, num_pages=32)
    app = create_app(eng, served_model_name="llama-tiny")
    with TestClient(app) as c:
        yield c


def test_api_models_and_health(api):
    assert api.get("/health").status_code == 200
    data = api.get("/v1/models").json()
    assert data["object"] == "list" and data["data"][0]["id"] == "llama-tiny"


def test_api_completion(api):
    r = api.post("/v1/completions", json={"model": "llama-tiny", "prompt": "hello", "max_tokens": 5,
                                          "temperature": 0, "ignore_eos": True})
    assert r.status_code == 200, r.text
    body = r.json()
    assert body["object"] == "text_completion" and body["choices"][0]["finish_reason"] == "length"
    assert body["usage"] == {"prompt_tokens": 6, "completion_tokens": 5, "total_tokens": 11}
    # deterministic for temperature 0
    again = api.post("/v1/completions", json={"model": "llama-tiny", "prompt": "hello", "max_tokens": 5,
                                              "temperature": 0, "ignore_eos": True}).json()
    assert again["choices"][0]["text"] == body["choices"][0]["text"]


def test_api_completion_stream_and_seeded_sampling(api):
    payload = {"model": "llama-tiny", "prompt": [1, 2, 3], "max_tokens": 4, "temperature": 0.8, "seed": 7,
               "stream": True, "ignore_eos": True}
    with api.stream("POST", "/v1/completions", json=payload) as r:
        assert r.status_code == 200
        lines = [ln for ln in r.iter_lines() if ln.startswith("data: ")]
    assert lines[-1] == "data: [DONE]"
    chunks = [json.loads(ln[6:]) for ln in lines[:-1]]
    assert chunks[-1]["choices"][0]["finish_reason"] == "length"
    text = "".join(c["choices"][0]["text"] for c in chunks)
    same = api.post("/v1/completions", json=dict(payload, stream=False)).json()
    assert same["choices"][0]["text"] == text  # same seed -> same draw


def test_api_chat(api):
    r = api.post("/v1/chat/completions", json={"model": "llama-tiny", "max_tokens": 3, "temperature": 0,
                                               "messages": [{"role": "user", "content": "hi"}]})
    assert r.status_code == 200, r.text
    body = r.json()
    assert body["object"] == "chat.completion"
    assert body["choices"][0]["message"]["role"] == "assistant"
    assert body["usage"]["completion_tokens"] <= 3
    with api.stream("POST", "/v1/chat/completions", json={"model": "llama-tiny", "max_tokens": 3, "stream": True,
                                                          "messages": [{"role": "user", "content": "hi"}]}) as r:
        lines = [ln for ln in r.iter_lines() if ln.startswith("data: ")]
    first = json.loads(lines[0][6:])
    assert first["object"] == "chat.completion.chunk" and first["choices"][0]["delta"].get("role") == "assistant"


def test_api_errors(api):
    r = api.post("/v1/completions", json={"model": "other", "prompt": "x"})
    assert r.status_code == 404
    r = api.post("/v1/completions", json={"model": "llama-tiny", "prompt": "x" * 400, "max_tokens": 2})
    assert r.status_code == 400
    m = api.get("/metrics").text
    assert "dstack_serving_running" in m and "dstack_serving_kv_usage" in m


# ------------------------------------------------------------------------------------------------
# GPU: HIP kernels vs fp32 references, engine on the HIP path with hipGraphs
# ------------------------------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("H,KVH", [(32, 8), (64, 8), (8, 8)])
def test_gpu_paged_decode_kernel(gpu, H, KVH):
    torch.manual_seed(0)
    dev = "cuda"
    pages = 80
    k_cache, v_cache = sops.alloc_cache(pages, KVH, torch.bfloat16, dev)
    k_cache.normal_()
    v_cache.normal_()
    B, W = 5, 40
    perm = torch.randperm(pages, device=dev)[: B * W].view(B, W).int() if pages >= B * W else \
        torch.randint(0, pages, (B, W), device=dev, dtype=torch.int32)
    ctx = torch.tensor([1, 63, 64, 1000, 2560], dtype=torch.int32, device=dev)
    qkv = torch.randn(B, (H + 2 * KVH) * 128, device=dev).to(torch.bfloat16)
    want = sops.paged_decode_ref(qkv, k_cache, v_cache, perm, ctx, H, KVH)
    for nsplit_target in (None, "one"):
        ws = sops.DecodeWorkspace(B, H, KVH, W, dev)
        if nsplit_target == "one":
            ws.nsplit, ws.pps = 1, W
        got = sops.paged_decode(qkv, k_cache, v_cache, perm, ctx, H, KVH, ws=ws)
        torch.testing.assert_close(got.float(), want, atol=2e-2, rtol=2e-2)


@pytest.mark.gpu
def test_gpu_rope_cache_write_kernel(gpu):
    torch.manual_seed(0)
    dev, H, KVH, T = "cuda", 32, 8, 70
    cos, sin = sops_rope(dev)
    qkv = torch.randn(T, (H + 2 * KVH) * 128, device=dev).to(torch.bfloat16)
    pos = torch.randint(0, 4000, (T,), device=dev, dtype=torch.int32)
    slots = torch.randperm(10 * 64, device=dev)[:T].int()
    slots[5] = -1
    kc, vc = sops.alloc_cache(10, KVH, torch.bfloat16, dev)
    kr, vr = sops.alloc_cache(10, KVH, torch.float32, dev)
    got = sops.rope_cache_write(qkv.clone(), pos, slots, cos, sin, kc, vc, H, KVH)
    want = sops.rope_cache_write_ref(qkv.float().clone(), pos, slots, cos, sin, kr, vr, H, KVH)
    torch.testing.assert_close(got.float(), want, atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(kc.float(), kr, atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(vc.float(), vr, atol=1e-6, rtol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("cache_dtype", [torch.bfloat16, torch.float8_e4m3fn])
def test_gpu_rope_cache_write_scaled_raw_product(gpu, cache_dtype):
    """A raw fp8 GEMM product with its row-wise scales handed to the RoPE / cache-write kernel gives
    bit-for-bit the qkv (every head, v included) and the cache of the pre-scaled product."""
    torch.manual_seed(1)
    dev, H, KVH, T = "cuda", 8, 2, 40
    cos, sin = sops_rope(dev)
    W = (H + 2 * KVH) * 128
    raw = (torch.randn(T, W, device=dev) * 300).to(torch.bfloat16)
    rs, cs = torch.rand(T, device=dev) * 1e-2, torch.rand(W, device=dev) * 1e-2
    scaled = (raw.float() * rs[:, None] * cs[None, :]).to(torch.bfloat16)
    pos = torch.randint(0, 4000, (T,), device=dev, dtype=torch.int32)
    slots = torch.randperm(4 * 64, device=dev)[:T].int()
    slots[3] = -1
    ka, va = sops.alloc_cache(4, KVH, cache_dtype, dev)
    kb, vb = sops.alloc_cache(4, KVH, cache_dtype, dev)
    a = sops.rope_cache_write(raw.clone(), pos, slots, cos, sin, ka, va, H, KVH, 0.5, 0.5, rs=rs, cs=cs)
    b = sops.rope_cache_write(scaled.clone(), pos, slots, cos, sin, kb, vb, H, KVH, 0.5, 0.5)
    assert torch.equal(a, b)
    assert torch.equal(ka.view(torch.uint8), kb.view(torch.uint8)) if cache_dtype != torch.bfloat16 else torch.equal(ka, kb)
    assert torch.equal(va.view(torch.uint8), vb.view(torch.uint8)) if cache_dtype != torch.bfloat16 else torch.equal(va, vb)


def sops_rope(dev):
    from dstack_amd.serving.model import rope_tables

    return rope_tables(4096, 128, 500000.0, None, dev)


@pytest.mark.gpu
def test_gpu_sample_kernel(gpu):
    torch.manual_seed(0)
    dev = "cuda"
    V = 128256
    logits = (torch.randn(6, V, device=dev) * 3).to(torch.bfloat16)
    temps = torch.zeros(6, device=dev)
    seeds = torch.arange(6, device=dev, dtype=torch.int64)
    steps = torch.zeros(6, device=dev, dtype=torch.int32)
    tok, lp = sops.sample(logits, temps, seeds, steps)
    assert tok.tolist() == logits.float().argmax(-1).int().tolist()
    torch.testing.assert_close(lp, torch.log_softmax(logits.float(), -1).max(-1).values, atol=1e-3, rtol=1e-3)
    # temperature sampling follows softmax(logits / T): frequencies over many seeds on a small vocab
    small = torch.tensor([[0.0, 1.0, 2.0, -1.0] + [-30.0] * 12], device=dev).to(torch.bfloat16).repeat(4096, 1)
    t = torch.full((4096,), 0.7, device=dev)
    toks, lps = sops.sample(small, t, torch.arange(4096, device=dev, dtype=torch.int64),
                            torch.zeros(4096, device=dev, dtype=torch.int32))
    freq = torch.bincount(toks.long(), minlength=16)[:4].float() / 4096
    want = torch.softmax(torch.tensor([0.0, 1.0, 2.0, -1.0]) / 0.7, -1).to(dev)
    assert (freq - want).abs().max() < 0.03, (freq, want)
    torch.testing.assert_close(lps.exp(), want[toks.long()], atol=1e-3, rtol=1e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("family", ["llama", "qwen2", "mistral"])
def test_gpu_engine_matches_cpu_and_graphs(gpu, tmp_path, family):
    """Tiny HF Llama / Qwen2 (biases) / Mistral on the HIP path: greedy tokens with and without
    hipGraphs identical, first token = the fp32 HF argmax up to bf16 near-ties."""
    hf, path = _hf_tiny(tmp_path) if family == "llama" else _hf_family_tiny(tmp_path, family)
    prompts = [[1, 5, 9, 33, 7, 100, 2, 45, 61], [1, 300, 301, 302], list(range(1, 200))]
    sp = SamplingParams(max_tokens=20, temperature=0, ignore_eos=True)
    g = LLMEngine.from_model(path, device="cuda", max_model_len=512, max_batch=8, num_pages=64)
    g.capture_graphs()
    assert g._graphs
    out_g = [r.output_ids for r in g.generate(prompts, sp)]
    ng = LLMEngine.from_model(path, device="cuda", max_model_len=512, max_batch=8, num_pages=64, use_graphs=False)
    out_ng = [r.output_ids for r in ng.generate(prompts, sp)]
    assert out_g == out_ng
    # the first generated token is HF's (fp32) argmax, up to bf16 near-ties
    with torch.no_grad():
        for p, o in zip(prompts, out_g):
            ref = hf(torch.tensor([p])).logits[0, -1]
            assert ref[o[0]] >= ref.max() - 0.02 * (ref.max() - ref.min())


@pytest.mark.gpu
@pytest.mark.parametrize("M", [1, 2, 3, 4])
@pytest.mark.parametrize("N,K", [(1024, 4096), (4100, 14336), (257, 3584)])
def test_gemv_matches_fp32(gpu, M, N, K):
    """Decode-projection GEMV kernel vs an fp32 matmul (row counts not divisible by 4, a K that
    is not a multiple of the 4-step unroll, x with a padded row stride)."""
    from dstack_amd.ops import _ext

    C = _ext.require()
    g = torch.Generator(device=gpu).manual_seed(M * 7 + N)
    xs = torch.randn(M, K + 64, device=gpu, generator=g).to(torch.bfloat16)
    x = xs[:, :K]
    w = (torch.randn(N, K, device=gpu, generator=g) * 0.02).to(torch.bfloat16)
    y = C.gemv(x, w)
    ref = x.float() @ w.float().t()
    err = ((y.float() - ref).norm() / ref.norm()).item()
    assert y.shape == (M, N) and err < 5e-3, err


# ------------------------------------------------------------------------------------------------
# fp8 (e4m3) projection weights
# ------------------------------------------------------------------------------------------------
def test_fp8_reference_quantization_roundtrip():
    from dstack_amd.ops import reference as ref

    torch.manual_seed(0)
    x = torch.randn(5, 256) * torch.tensor([0.01, 1.0, 30.0, 1e3, 1e-3])[:, None]
    q, s = ref.quant_fp8_rows(x)
    assert q.dtype == torch.float8_e4m3fn and s.shape == (5,)
    assert (q.float().abs().amax(dim=1) == 448).all()  # every row uses the full e4m3 range
    back = q.float() * s[:, None]
    assert ((back - x).norm(dim=1) / x.norm(dim=1)).max() < 0.04  # 3 mantissa bits


def test_fp8_engine_close_to_bf16_engine():
    """The fp8 model's prefill logits track the unquantized model's (per-channel weight scales,
    per-token activation scales), and it frees about half of the projection bytes."""
    kw = dict(device="cpu", max_model_len=256, max_batch=4, num_pages=16)
    base = LLMEngine.from_model("llama-tiny", **kw)
    q8 = LLMEngine.from_model("llama-tiny", quantization="fp8", **kw)
    assert q8.model.weight_bytes() < 0.75 * base.model.weight_bytes()
    assert all(type(L["wgu"]).__name__ == "Fp8Weight" for L in q8.model.layers)
    prompt = torch.tensor(list(range(1, 129)))
    pos = torch.arange(128, dtype=torch.int32)
    slots = torch.arange(128, dtype=torch.int32)
    a = base.model.prefill(prompt, pos, slots, [0], [128])
    b = q8.model.prefill(prompt, pos, slots, [0], [128])
    cos = torch.nn.functional.cosine_similarity(a.float(), b.float(), dim=-1).item()
    assert cos > 0.99, cos
    sp = SamplingParams(max_tokens=8, temperature=0, ignore_eos=True)
    out = q8.generate([[1, 2, 3, 4, 5]], sp)
    assert len(out[0].output_ids) == 8


def test_fp8_rejects_unknown_quantization():
    from dstack_amd.serving.model import ServingLlama, load_spec

    with pytest.raises(ValueError, match="quantization"):
        ServingLlama(load_spec("llama-tiny"), "cpu", quantization="int3")


@pytest.mark.gpu
@pytest.mark.parametrize("M,K", [(1, 4096), (7, 8192), (256, 4096), (5, 28672), (4, 32768), (2, 1000)])
def test_gpu_quant_fp8_rows_matches_torch(gpu, M, K):
    """HIP per-row e4m3 quantization: scales equal max|x|/448 and the bytes decode to the same
    values as torch's float8_e4m3fn cast (round to nearest even) up to ties."""
    from dstack_amd.ops import _ext, reference as ref

    C = _ext.require()
    g = torch.Generator(device=gpu).manual_seed(M)
    x = (torch.randn(M, K, device=gpu, generator=g) * torch.rand(M, 1, device=gpu, generator=g) * 10).bfloat16()
    q, s = C.quant_fp8_rows(x)
    qr, sr = ref.quant_fp8_rows(x)
    torch.testing.assert_close(s, sr, rtol=1e-6, atol=0)
    got = q.view(torch.float8_e4m3fn).float()
    want = qr.float()
    assert (got != want).float().mean().item() < 1e-3
    assert ((got * s[:, None] - x.float()).norm() / x.float().norm()).item() < 0.04


@pytest.mark.gpu
@pytest.mark.parametrize("M", [1, 2, 4])
@pytest.mark.parametrize("N,K", [(1024, 4096), (4101, 14336)])
def test_gpu_gemv_fp8_matches_fp32(gpu, M, N, K):
    """fp8-weight GEMV vs the fp32 product of the dequantized weights (rows not divisible by 4,
    padded x rows)."""
    from dstack_amd.ops import _ext

    C = _ext.require()
    g = torch.Generator(device=gpu).manual_seed(M * 11 + N)
    xs = torch.randn(M, K + 64, device=gpu, generator=g).to(torch.bfloat16)
    x = xs[:, :K]
    w = (torch.randn(N, K, device=gpu, generator=g) * 0.02).to(torch.bfloat16)
    q, s = C.quant_fp8_rows(w)
    y = C.gemv_fp8(x, q, s)
    ref = x.float() @ (q.view(torch.float8_e4m3fn).float() * s[:, None]).t()
    err = ((y.float() - ref).norm() / ref.norm()).item()
    assert y.shape == (M, N) and err < 5e-3, err


@pytest.mark.gpu
def test_gpu_fp8_engine_tracks_bf16(gpu):
    """fp8 serving model on the HIP path (GEMV for batch 1, hipBLASLt fp8 GEMM with row-wise scales
    for prefill and larger batches): prefill logits close to the bf16 model's, generation runs
    with hipGraphs."""
    kw = dict(device="cuda", max_model_len=512, max_batch=8, num_pages=64)
    base = LLMEngine.from_model("llama-tiny", **kw)
    q8 = LLMEngine.from_model("llama-tiny", quantization="fp8", **kw)
    prompt = torch.arange(1, 257, device=gpu)
    pos = torch.arange(256, dtype=torch.int32, device=gpu)
    slots = torch.arange(256, dtype=torch.int32, device=gpu)
    a = base.model.prefill(prompt, pos, slots, [0], [256])
    b = q8.model.prefill(prompt, pos, slots, [0], [256])
    cos = torch.nn.functional.cosine_similarity(a.float(), b.float(), dim=-1).item()
    assert cos > 0.99, cos
    q8.capture_graphs()
    sp = SamplingParams(max_tokens=16, temperature=0, ignore_eos=True)
    outs = q8.generate([[1, 2, 3, 4, 5], list(range(7, 90))], sp)
    assert all(len(o.output_ids) == 16 for o in outs)


@pytest.mark.gpu
def test_gpu_fp8_deferred_row_scales_match_rowwise(gpu):
    """Prefill-sized fp8 GEMMs run with scalar scales on the raw e4m3 operands and apply the
    row-wise scales afterwards (SwiGLU-quant kernel for gate/up, the fused add + RMSNorm -> e4m3
    kernel for o / down, or an in-place pass).
    Kernels: bit-identical to scaling in fp32 then rounding.  Model: the extra bf16 rounding of the
    raw product keeps the prefill logits as close to the bf16 model's as the row-wise path's."""
    from dstack_amd.ops import _ext

    C = _ext.require()
    torch.manual_seed(0)
    for M, F in ((128, 1024), (256, 3584), (64, 28672)):
        raw = torch.randn(M, 2 * F, device=gpu, dtype=torch.bfloat16) * 300
        rs = torch.rand(M, device=gpu) * 1e-2
        cs = torch.rand(2 * F, device=gpu) * 1e-2
        scaled = (raw.float() * rs[:, None] * cs[None, :]).bfloat16()
        q, s = C.swiglu_quant_fp8_rows(raw, rs, cs)
        q2, s2 = C.swiglu_quant_fp8_rows(scaled)
        assert torch.equal(s, s2)
        assert torch.equal(q.view(torch.uint8), q2.view(torch.uint8))
        y = raw.clone()
        C.scale_rows_cols_(y, rs, cs)
        assert torch.equal(y, scaled)
    for M, D in ((64, 1024), (2048, 8192)):  # the fused add + RMSNorm -> e4m3 with a raw delta
        raw = torch.randn(M, D, device=gpu, dtype=torch.bfloat16) * 300
        rs, cs = torch.rand(M, device=gpu) * 1e-2, torch.rand(D, device=gpu) * 1e-2
        x = torch.randn(M, D, device=gpu, dtype=torch.bfloat16)
        w = torch.rand(D, device=gpu, dtype=torch.bfloat16) + 0.5
        scaled = (raw.float() * rs[:, None] * cs[None, :]).bfloat16()
        h1, q1, s1 = C.rms_norm_fp8(x, raw, w, 1e-5, rs, cs)
        h2, q2, s2 = C.rms_norm_fp8(x, scaled, w, 1e-5)
        assert torch.equal(h1, h2) and torch.equal(s1, s2)
        assert torch.equal(q1.view(torch.uint8), q2.view(torch.uint8))
    kw = dict(device="cuda", max_model_len=512, max_batch=8, num_pages=64)
    base = LLMEngine.from_model("llama-tiny", **kw)
    q8 = LLMEngine.from_model("llama-tiny", quantization="fp8", **kw)
    n = 384  # past the in-tree decode fp8 GEMM's 256 rows: the hipBLASLt path
    prompt = torch.arange(1, n + 1, device=gpu)
    pos = torch.arange(n, dtype=torch.int32, device=gpu)
    slots = torch.arange(n, dtype=torch.int32, device=gpu)
    ref_logits = base.model.prefill(prompt, pos, slots, [0], [n]).float()
    q8.model.fp8_defer_rows = 1 << 62
    a = q8.model.prefill(prompt, pos, slots, [0], [n]).float()
    q8.model.fp8_defer_rows = 128
    b = q8.model.prefill(prompt, pos, slots, [0], [n]).float()
    cs = torch.nn.functional.cosine_similarity
    cos_rowwise, cos_deferred = cs(a, ref_logits, dim=-1).item(), cs(b, ref_logits, dim=-1).item()
    assert cos_deferred > 0.99 and cos_deferred > cos_rowwise - 0.003, (cos_rowwise, cos_deferred)
    assert cs(a, b, dim=-1).item() > 0.995


@pytest.mark.gpu
def test_gpu_fp8_stream_gemm_in_the_engine(gpu, monkeypatch):
    """The weight-streaming decode fp8 GEMM in the model (``_mm_fp8`` for 129..256 rows, pre-shuffled
    second copy ``Fp8Weight.qs``), forced onto llama-tiny's MLP (the default rule only takes the
    70B-sized gate/up and down weights): a 256-token forward's logits match the hipBLASLt path's."""
    from dstack_amd.ops import _ext
    from dstack_amd.ops.serving import fp8_stream_shuffle

    kw = dict(device="cuda", max_model_len=512, max_batch=8, num_pages=64)
    q8 = LLMEngine.from_model("llama-tiny", quantization="fp8", **kw)
    m = q8.model
    assert all(L[k].qs is None for L in m.layers for k in m.FP8_KEYS)  # tiny shapes: no second copy
    n = 256  # (prefill segments are 128-row aligned)
    prompt = torch.arange(1, n + 1, device=gpu)
    pos = torch.arange(n, dtype=torch.int32, device=gpu)
    slots = torch.arange(n, dtype=torch.int32, device=gpu)
    a = m.prefill(prompt, pos, slots, [0], [n]).float()
    m._stream_cfg = lambda N, K: (32, 1)
    m._add_stream_copies(reserve_bytes=1 << 62)  # no room left: no copies, hipBLASLt stays
    assert all(L[k].qs is None for L in m.layers for k in m.FP8_KEYS)
    m._add_stream_copies(reserve_bytes=0)
    for L in m.layers:
        for k in ("wgu", "wdown"):
            group = 16 if m.fp8_stream_layout == 1 else 256
            assert torch.equal(L[k].qs.view(torch.uint8), fp8_stream_shuffle(L[k].q, group).view(torch.uint8))
    C = _ext.require()
    calls, orig = [], C.fp8_stream_gemm
    monkeypatch.setattr(C, "fp8_stream_gemm", lambda *a_, **k_: calls.append(a_[0].shape) or orig(*a_, **k_))
    b = m.prefill(prompt, pos, slots, [0], [n]).float()
    assert len(calls) == 2 * len(m.layers) and all(128 < c[0] <= 256 for c in calls), calls
    cos = torch.nn.functional.cosine_similarity(a, b, dim=-1).item()
    assert cos > 0.999, cos


@pytest.mark.gpu
def test_gpu_fp8_swiglu_gemm_matches_deferred_kernels(gpu):
    """The fp8 gate/up GEMM with the SwiGLU and the row-wise scales in its epilogue plus the
    one-pass row quantizer (csrc/gemm_nt.hip EPI_SWIGLU_F8, fp8.hip quant_rows_pmax) against
    hipBLASLt's raw product fed to the deferred-scale SwiGLU-quant kernel; and the fp8 engine's
    prefill logits with the fused path on and off."""
    from dstack_amd.ops import _ext
    from dstack_amd.ops import reference as ref

    C = _ext.require()
    torch.manual_seed(0)
    one = torch.ones((), device=gpu)
    for M, F, K in ((256, 1024, 512), (512, 3584, 8192)):
        assert C.gemm_nt_f8_swiglu_supported(M, F, K)
        x = torch.randn(M, K, device=gpu, dtype=torch.bfloat16)
        w = torch.randn(2 * F, K, device=gpu, dtype=torch.bfloat16) * 0.02
        xq, xs = C.quant_fp8_rows(x)
        wq, ws = ref.quant_fp8_rows(w)
        xs = xs.reshape(-1).contiguous()
        raw = torch._scaled_mm(xq.view(torch.float8_e4m3fn), wq.t(), scale_a=one, scale_b=one,
                               out_dtype=torch.bfloat16)
        q_ref, s_ref = C.swiglu_quant_fp8_rows(raw, xs, ws)
        q, s, a = C.gemm_nt_f8_swiglu_quant(xq.view(torch.uint8), wq.view(torch.uint8), xs, ws)
        assert torch.allclose(s, s_ref, rtol=1e-3, atol=0), (s - s_ref).abs().max().item()
        same = (q.view(torch.uint8) == q_ref.view(torch.uint8)).float().mean().item()
        assert same > 0.999, same
        deq, deq_ref = q.view(torch.float8_e4m3fn).float() * s[:, None], q_ref.view(torch.float8_e4m3fn).float() * s_ref[:, None]
        assert ((deq - deq_ref).norm() / deq_ref.norm()).item() < 1e-2
        exp = ref.swiglu((raw.float() * xs[:, None] * ws[None, :]).bfloat16().float())
        assert ((a.float() - exp).norm() / exp.norm()).item() < 1e-2
    kw = dict(device="cuda", max_model_len=1024, max_batch=8, num_pages=64)
    q8 = LLMEngine.from_model("llama-tiny", quantization="fp8", **kw)
    n = 512  # a multiple of 256 rows: the fused gate/up path
    prompt = torch.arange(1, n + 1, device=gpu)
    pos = torch.arange(n, dtype=torch.int32, device=gpu)
    slots = torch.arange(n, dtype=torch.int32, device=gpu)
    q8.model.fp8_swiglu_gemm = False
    a = q8.model.prefill(prompt, pos, slots, [0], [n]).float()
    q8.model.fp8_swiglu_gemm = True
    b = q8.model.prefill(prompt, pos, slots, [0], [n]).float()
    assert torch.nn.functional.cosine_similarity(a, b, dim=-1).item() > 0.999


# ------------------------------------------------------------------------------------------------
# fp8 (e4m3) KV cache
# ------------------------------------------------------------------------------------------------
def test_fp8_kv_cache_engine_close_to_bf16():
    """An fp8 KV cache holds twice the tokens per byte; greedy decoding on it tracks the bf16
    cache (first decode logits close; the CPU path dequantizes in the fp32 reference)."""
    kw = dict(device="cpu", max_model_len=256, max_batch=4, num_pages=16)
    base = LLMEngine.from_model("llama-tiny", **kw)
    f8 = LLMEngine.from_model("llama-tiny", kv_cache_dtype="fp8", **kw)
    assert f8.model.k_cache[0].dtype == torch.float8_e4m3fn
    assert f8.model.kv_bytes_per_page() * 4 == base.model.kv_bytes_per_page()  # fp32 CPU cache vs 1 byte
    sp = SamplingParams(max_tokens=12, temperature=0, ignore_eos=True)
    prompts = [[1, 5, 9, 33, 7, 100, 2, 45, 61], list(range(3, 90))]
    a = [r.output_ids for r in base.generate(prompts, sp)]
    b = [r.output_ids for r in f8.generate(prompts, sp)]
    agree = sum(x == y for p, q in zip(a, b) for x, y in zip(p, q)) / sum(len(p) for p in a)
    assert agree > 0.8, (a, b)
    with pytest.raises(ValueError, match="kv_cache_dtype"):
        LLMEngine.from_model("llama-tiny", kv_cache_dtype="int4", **kw)


@pytest.mark.gpu
def test_gpu_paged_decode_empty_splits_ignore_workspace(gpu):
    """Splits past a sequence's context write only their -inf lse; the combine must not read their
    (uninitialised) partial rows: a NaN-filled workspace leaves the output finite and exact."""
    torch.manual_seed(0)
    dev, H, KVH, B, W = "cuda", 8, 2, 1, 8
    k_cache, v_cache = sops.alloc_cache(16, KVH, torch.bfloat16, dev)
    k_cache.normal_()
    v_cache.normal_()
    table = torch.arange(W, dtype=torch.int32, device=dev).view(1, W)
    ctx = torch.tensor([201], dtype=torch.int32, device=dev)  # 4 of 8 single-page splits populated
    qkv = torch.randn(B, (H + 2 * KVH) * 128, device=dev).to(torch.bfloat16)
    ws = sops.DecodeWorkspace(B, H, KVH, W, dev)
    assert ws.nsplit == 8
    ws.o_part.fill_(float("nan"))
    got = sops.paged_decode(qkv, k_cache, v_cache, table, ctx, H, KVH, ws=ws)
    want = sops.paged_decode_ref(qkv, k_cache, v_cache, table, ctx, H, KVH)
    assert torch.isfinite(got).all()
    torch.testing.assert_close(got.float(), want, atol=2e-2, rtol=2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("H,KVH", [(32, 8), (64, 8)])
def test_gpu_paged_decode_fp8_cache(gpu, H, KVH):
    """Paged decode over an e4m3 cache (with non-unit k/v scales folded into the kernel) vs the
    fp32 reference over the dequantized cache, split and single-split."""
    torch.manual_seed(0)
    dev = "cuda"
    pages, B, W = 80, 5, 40
    k_cache, v_cache = sops.alloc_cache(pages, KVH, torch.float8_e4m3fn, dev)
    k_cache.copy_(torch.randn(k_cache.shape, device=dev).clamp(-4, 4).to(torch.float8_e4m3fn))
    v_cache.copy_(torch.randn(v_cache.shape, device=dev).clamp(-4, 4).to(torch.float8_e4m3fn))
    perm = torch.randint(0, pages, (B, W), device=dev, dtype=torch.int32)
    ctx = torch.tensor([1, 63, 64, 1000, 2560], dtype=torch.int32, device=dev)
    qkv = torch.randn(B, (H + 2 * KVH) * 128, device=dev).to(torch.bfloat16)
    ks, vs = 0.5, 2.0
    want = sops.paged_decode_ref(qkv, k_cache, v_cache, perm, ctx, H, KVH, ks, vs)
    for one in (False, True):
        ws = sops.DecodeWorkspace(B, H, KVH, W, dev)
        if one:
            ws.nsplit, ws.pps = 1, W
        got = sops.paged_decode(qkv, k_cache, v_cache, perm, ctx, H, KVH, ws=ws, k_scale=ks, v_scale=vs)
        torch.testing.assert_close(got.float(), want, atol=4e-2, rtol=2e-2)


@pytest.mark.gpu
def test_gpu_rope_cache_write_fp8(gpu):
    """RoPE + scatter into an e4m3 cache: the bytes equal the reference's cast of k / k_scale and
    v / v_scale (up to rounding ties of the bf16-rotated k)."""
    torch.manual_seed(0)
    dev, H, KVH, T = "cuda", 32, 8, 70
    cos, sin = sops_rope(dev)
    qkv = torch.randn(T, (H + 2 * KVH) * 128, device=dev).to(torch.bfloat16)
    pos = torch.randint(0, 4000, (T,), device=dev, dtype=torch.int32)
    slots = torch.randperm(10 * 64, device=dev)[:T].int()
    slots[5] = -1
    kc, vc = sops.alloc_cache(10, KVH, torch.float8_e4m3fn, dev)
    kr, vr = sops.alloc_cache(10, KVH, torch.float8_e4m3fn, dev)
    got = sops.rope_cache_write(qkv.clone(), pos, slots, cos, sin, kc, vc, H, KVH, 0.5, 2.0)
    want = sops.rope_cache_write_ref(qkv.clone(), pos, slots, cos, sin, kr, vr, H, KVH, 0.5, 2.0)
    torch.testing.assert_close(got, want)  # q / k rotation is unchanged
    assert (kc.float() != kr.float()).float().mean().item() < 1e-3
    assert torch.equal(vc.float(), vr.float())


@pytest.mark.gpu
def test_gpu_fp8_kv_decode_logits_track_bf16(gpu):
    """One decode step over a 200-token context held in an fp8 cache gives logits close to the
    same step over the bf16 cache (same weights), on the HIP path."""
    kw = dict(device="cuda", max_model_len=512, max_batch=8, num_pages=64)
    outs = []
    for kv in ("auto", "fp8"):
        m = LLMEngine.from_model("llama-tiny", kv_cache_dtype=kv, **kw).model
        n = 256  # prefill rows (128-aligned); the first 200 are the prompt
        toks = torch.arange(1, n + 1, device=gpu) % 500
        pos = torch.arange(n, dtype=torch.int32, device=gpu)
        slots = torch.where(pos < 200, pos, torch.full_like(pos, -1))
        m.prefill(toks, pos, slots, [0], [200])
        table = torch.arange(8, dtype=torch.int32, device=gpu).view(1, 8)
        logits = m.decode(torch.tensor([7], device=gpu), torch.tensor([200], dtype=torch.int32, device=gpu),
                          torch.tensor([200], dtype=torch.int32, device=gpu), table,
                          torch.tensor([201], dtype=torch.int32, device=gpu))
        outs.append(logits.float())
    cos = torch.nn.functional.cosine_similarity(outs[0], outs[1], dim=-1).item()
    assert cos > 0.99, cos


@pytest.mark.gpu
@pytest.mark.parametrize("rows", [37, 2048])
@pytest.mark.parametrize("with_delta", [False, True])
def test_gpu_rms_norm_fp8_matches_unfused(gpu, with_delta, rows):
    """The fused (add +) RMSNorm -> e4m3 kernel equals RMSNorm followed by the row quantizer
    (decode batches and, past 1024 rows, prefill, where the unfused norm is the wave-per-row one)."""
    from dstack_amd.ops import _ext

    C = _ext.require()
    g = torch.Generator(device=gpu).manual_seed(3)
    x = torch.randn(rows, 8192, device=gpu, generator=g).bfloat16()
    d = torch.randn(rows, 8192, device=gpu, generator=g).bfloat16()
    w = (torch.rand(8192, device=gpu, generator=g) + 0.5).bfloat16()
    if with_delta:
        h_ref, y_ref, _ = C.add_rms_norm_fwd(x, d, w, 1e-5)
        h, q, s = C.rms_norm_fp8(x, d, w, 1e-5)
        assert torch.equal(h, h_ref)
    else:
        y_ref = C.rms_norm_fwd(x, w, 1e-5)[0]
        _, q, s = C.rms_norm_fp8(x, None, w, 1e-5)
    q_ref, s_ref = C.quant_fp8_rows(y_ref)
    torch.testing.assert_close(s, s_ref, rtol=1e-6, atol=0)
    assert (q != q_ref).float().mean().item() < 1e-3


def test_api_client_disconnect_aborts_request():
    """A client that leaves mid-stream aborts its request: decoding stops and the KV pages are
    freed instead of running to max_tokens with no consumer."""
    import asyncio

    from dstack_amd.serving.server import create_app

    eng = LLMEngine.from_model("llama-tiny", device="cpu", max_model_len=512, max_batch=4, num_pages=32)
    app = create_app(eng, served_model_name="llama-tiny")
    seen = []
    orig = eng.add_request

    def add_request(*a, **k):
        r = orig(*a, **k)
        seen.append(r)
        return r

    eng.add_request = add_request
    payload = json.dumps({"model": "llama-tiny", "prompt": [1, 2, 3], "max_tokens": 500, "temperature": 0,
                          "ignore_eos": True, "stream": True}).encode()

    async def run():
        got_body = asyncio.Event()
        state = {"sent_request": False}

        async def receive():
            if not state["sent_request"]:
                state["sent_request"] = True
                return {"type": "http.request", "body": payload, "more_body": False}
            await got_body.wait()
            return {"type": "http.disconnect"}

        async def send(msg):
            if msg["type"] == "http.response.body" and msg.get("body"):
                got_body.set()

        scope = {"type": "http", "asgi": {"version": "3.0"}, "http_version": "1.1", "method": "POST",
                 "scheme": "http", "path": "/v1/completions", "raw_path": b"/v1/completions", "query_string": b"",
                 "headers": [(b"content-type", b"application/json")], "client": ("127.0.0.1", 1),
                 "server": ("127.0.0.1", 80), "root_path": ""}
        await asyncio.wait_for(app(scope, receive, send), 60)

    eng.start()
    try:
        asyncio.run(run())
        deadline = time.time() + 10
        while time.time() < deadline and (not seen[0].finished or eng.metrics()["running"]):
            time.sleep(0.02)
    finally:
        eng.stop()
    req = seen[0]
    assert req.finished and req.finish_reason == "abort"
    assert len(req.output_ids) < 500
    assert eng.metrics()["running"] == 0


def test_api_completions_rejects_before_submitting_any_prompt(api):
    """Prompt 2 of 2 too long: a 400, and prompt 1 was never submitted (no orphaned decode)."""
    before = api.get("/metrics").text
    r = api.post("/v1/completions", json={"model": "llama-tiny", "prompt": [[1, 2], list(range(1, 300))],
                                          "max_tokens": 2})
    assert r.status_code == 400
    after = api.get("/metrics").text

    def reqs(m):
        return [ln for ln in m.splitlines() if ln.startswith("dstack_serving_requests_total")][0]

    assert reqs(before) == reqs(after)


@pytest.mark.gpu
def test_gpu_swiglu_quant_fp8_rows_matches_separate_kernels(gpu):
    """The fused SwiGLU + per-row e4m3 quantization equals swiglu_fwd followed by quant_fp8_rows
    (same bf16-rounded product, same scales, same bytes)."""
    from dstack_amd.ops import _ext

    C = _ext.require()
    torch.manual_seed(0)
    for M, F in ((1, 512), (37, 1024), (256, 3584), (16, 14336), (8, 28672), (3, 40960)):
        gu = torch.randn(M, 2 * F, device=gpu, dtype=torch.bfloat16) * 2
        q, s = C.swiglu_quant_fp8_rows(gu)
        q2, s2 = C.quant_fp8_rows(C.swiglu_fwd(gu))
        assert torch.equal(s, s2)
        assert torch.equal(q.view(torch.uint8), q2.view(torch.uint8))


def test_fp8_stream_shuffle_layout_matches_the_kernel_addressing():
    """ops.serving.fp8_stream_shuffle (the pre-shuffled weight layouts of fp8_stream_gemm(...,
    shuffled=1 | 2)): lane r + 16 g of 16-row block nb at K-step t reads bytes [32 g + 16 h, +16) of row
    16 nb + r at the offset the kernel computes (csrc/fp8_gemm.hip fp8_stream_gemm_kernel) for 16-row
    blocks and for 256-row groups; unshuffle inverts it."""
    N, K = 1792, 384
    w = torch.randint(0, 256, (N, K), dtype=torch.uint8)
    ks = K // 128
    for group in (16, 256, 224):
        sh = sops.fp8_stream_shuffle(w, group)
        assert sh.shape == (N, K) and sh.is_contiguous()
        assert torch.equal(sops.fp8_stream_unshuffle(sh, group), w)
        flat = sh.flatten()
        for nb in range(0, N // 16, 5):
            for t in range(ks):
                for lane in range(0, 64, 3):
                    r, g = lane % 16, lane // 16
                    for h in range(2):
                        if group == 16:
                            off = ((nb * ks + t) * 2 + h) * 1024 + lane * 16
                        else:  # the gb blocks of a workgroup's rows side by side per K-step
                            gb = group // 16
                            off = (((nb // gb) * ks + t) * gb + nb % gb) * 2048 + h * 1024 + lane * 16
                        k = t * 128 + 32 * g + 16 * h
                        assert torch.equal(flat[off:off + 16], w[16 * nb + r, k:k + 16])
    f8 = sops.fp8_stream_shuffle(w.view(torch.float8_e4m3fn), 224)
    assert f8.dtype == torch.float8_e4m3fn and torch.equal(f8.view(torch.uint8), sh)


def test_fp8_rows_shuffle_layout_is_the_kernels_lds_image():
    """ops.serving.fp8_rows_shuffle (fp8_rows_gemm(..., wimg=True)): per 128-row tile and K-step the
    1 KiB DMA piece p holds, at lane * 16, row 8 p + lane // 8's chunk (lane % 8) ^ f8_swz(row % 16) --
    what the kernel's row-major DMA writes to LDS (csrc/fp8_gemm.hip fp8_rows_gemm_kernel)."""
    N, K = 256, 384
    w = torch.randint(0, 256, (N, K), dtype=torch.uint8)
    img = sops.fp8_rows_shuffle(w).flatten()
    swz = lambda r: ((r >> 1) & 1) | (((r >> 3) & 1) << 2)  # noqa: E731
    ks = K // 128
    for nb in range(N // 128):
        for t in range(ks):
            for piece in range(16):
                for lane in range(0, 64, 5):
                    row, off = 8 * piece + (lane >> 3), (nb * ks + t) * 16384 + piece * 1024 + lane * 16
                    ch = (lane & 7) ^ swz(row & 15)
                    assert torch.equal(img[off:off + 16], w[nb * 128 + row, t * 128 + ch * 16:t * 128 + ch * 16 + 16])
