"""The bench's synthetic token stream (workloads/data.py): deterministic per (seed, index), fresh
every micro-step, the advertised chain structure and entropy floor."""

import math

import torch

from dstack_amd.workloads.data import SyntheticLM, _A, _B


def test_stream_is_deterministic_and_fresh():
    s = SyntheticLM(32000, 512, 2, "cpu", seed=7)
    a, b = s.batch(3)
    assert a.shape == (2, 512) and b.shape == (2, 512)
    assert torch.equal(a[:, 1:], b[:, :-1])  # targets are the inputs shifted by one
    assert torch.equal(s.tokens(3), SyntheticLM(32000, 512, 2, "cpu", seed=7).tokens(3))
    assert not torch.equal(s.tokens(3), s.tokens(4))
    assert not torch.equal(s.tokens(3), SyntheticLM(32000, 512, 2, "cpu", seed=8).tokens(3))
    x = s.tokens(0)
    assert int(x.min()) >= 0 and int(x.max()) < 32000


def test_chain_structure_matches_closed_form():
    V = 128256
    s = SyntheticLM(V, 4096, 1, "cpu", seed=1, copy_p=0.5)
    x = s.tokens(0)[0]
    chained = x[1:] == (_A * x[:-1] + _B) % V
    assert 0.45 < chained.float().mean().item() < 0.55
    # tokens that are not chained follow the Zipf head: few distinct ids, far below uniform
    assert x.unique().numel() < 0.5 * x.numel()


def test_loss_floor_and_row_starts():
    s = SyntheticLM(1000, 64, 4, "cpu", seed=0, zipf_s=1.0, copy_p=0.25)
    ranks = torch.arange(1, 1001, dtype=torch.float64)
    q = ranks.reciprocal() / ranks.reciprocal().sum()
    h = float(-(q * q.log()).sum())
    assert math.isclose(s.unigram_entropy, h, rel_tol=1e-9)
    hp = -(0.25 * math.log(0.25) + 0.75 * math.log(0.75))
    assert math.isclose(s.loss_floor, hp + 0.75 * h, rel_tol=1e-9)
    assert s.loss_floor < math.log(1000)
    # every row starts from a fresh sample (no chain crosses rows)
    assert not bool(s.row_start[1:65].any()) and bool(s.row_start[65])


def test_zero_output_head_starts_at_ln_vocab():
    """``init_weights(lm_head_std=0)``: uniform logits, so the first loss is exactly ln(vocab)."""
    import math

    import torch

    from dstack_amd.models.llama import CONFIGS, Llama

    cfg = CONFIGS["llama-tiny"]
    m = Llama(cfg)
    m.init_weights(seed=1, lm_head_std=0.0)
    tok = torch.randint(0, cfg.vocab_size, (2, 65), generator=torch.Generator().manual_seed(0))
    with torch.no_grad():
        loss = m.loss(tok[:, :-1], tok[:, 1:]).item()
    assert abs(loss - math.log(cfg.vocab_size)) < 1e-4


def test_splitmix64_matches_uint64_arithmetic():
    """The int64 torch form of splitmix64 (wrap-around multiply, logical shifts) equals the uint64
    definition that ops/csrc/data.hip computes."""
    from dstack_amd.workloads.data import _splitmix64

    def ref(z):
        m = (1 << 64) - 1
        z = (z + 0x9E3779B97F4A7C15) & m
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
        return z ^ (z >> 31)

    xs = [0, 1, 2, 12345, (1 << 40) + 7, (1 << 62) + 3, (1 << 63) - 1]
    got = _splitmix64(torch.tensor(xs, dtype=torch.int64)).tolist()
    assert [g & ((1 << 64) - 1) for g in got] == [ref(x) for x in xs]
