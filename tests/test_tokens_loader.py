"""Token-shard input (native loader, workloads/tokens.py): windows are contiguous slices of the
shards, every window once per epoch, data-parallel ranks disjoint, batch i reproducible (resume),
headerless and llm.c shards, and the Trainer on real-data input."""

import numpy as np
import pytest
import torch

from dstack_amd.workloads.tokens import TokenShards, write_shard


@pytest.fixture
def shards(tmp_path):
    write_shard(str(tmp_path / "a.bin"), np.arange(0, 4001), np.uint16)  # 40 windows of seq 100
    write_shard(str(tmp_path / "b.bin"), np.arange(50000, 52001), np.uint32)  # 20 windows
    np.arange(60000, 61001, dtype=np.uint16).tofile(str(tmp_path / "c.raw"))  # headerless: 10 windows
    return tmp_path


def _windows(ts, n):
    out = []
    for i in range(n):
        x, y = ts.batch(i)
        assert torch.equal(x[:, 1:], y[:, :-1])
        for row in torch.cat([x, y[:, -1:]], dim=1):
            assert torch.equal(row, row[0] + torch.arange(row.numel()))  # one contiguous slice
            out.append(int(row[0]))
    return out


def test_epoch_coverage_ranks_and_resume(shards):
    glob = f"{shards}/*.bin"
    r0 = TokenShards(glob, 100, 3, "cpu", seed=11, rank=0, world=2)
    r1 = TokenShards(glob, 100, 3, "cpu", seed=11, rank=1, world=2)
    assert r0.num_tokens == 6002 and r0.batches_per_epoch == 10  # 60 windows / (3 x 2)
    seen = _windows(r0, 10) + _windows(r1, 10)
    assert len(seen) == 60 and len(set(seen)) == 60  # every window once, ranks disjoint
    # batch 10 opens epoch 1 in a new order; a fresh loader seeking to it agrees (resume)
    e1 = r0.tokens(10)
    again = TokenShards(glob, 100, 3, "cpu", seed=11, rank=0, world=2).tokens(10)
    assert torch.equal(e1, again)
    assert not torch.equal(e1, r0.tokens(0))  # seeking back works too
    other_seed = TokenShards(glob, 100, 3, "cpu", seed=12, rank=0, world=2)
    assert not torch.equal(other_seed.tokens(0), r0.tokens(0))


def test_headerless_shards_need_token_width(shards):
    with pytest.raises(ValueError, match="token_bytes"):
        TokenShards(f"{shards}/c.raw", 100, 1, "cpu")
    ts = TokenShards(f"{shards}/c.raw", 100, 1, "cpu", token_bytes=2)
    assert ts.batches_per_epoch == 10 and 60000 <= int(ts.tokens(0)[0, 0]) < 61000


def test_vocab_guard_and_missing_files(shards):
    with pytest.raises(FileNotFoundError):
        TokenShards(f"{shards}/nope*.bin", 100, 1, "cpu")
    ts = TokenShards(f"{shards}/b.bin", 100, 1, "cpu", vocab_size=1000)
    with pytest.raises(ValueError, match="vocab size"):
        ts.tokens(0)


def test_trainer_on_token_shards_and_resume_index(shards, tmp_path):
    from dstack_amd.workloads.train_llama import Trainer

    write_shard(str(tmp_path / "tiny.bin"), np.random.default_rng(0).integers(0, 1000, 40000), np.uint16)
    spec = f"tokens:{tmp_path}/tiny.bin"
    tr = Trainer("llama-tiny", 32, 2, torch.device("cpu"), data=spec, lr_warmup=2)
    first = [tr.batch()[0].clone() for _ in range(3)]
    loss = tr.step()
    assert torch.isfinite(loss)
    tr2 = Trainer("llama-tiny", 32, 2, torch.device("cpu"), data=spec)
    tr2._i = 2  # what a checkpoint restores
    assert torch.equal(tr2.batch()[0], first[2])


@pytest.mark.gpu
def test_token_shards_to_gpu_and_train_step(gpu, tmp_path):
    """Pinned ring buffers + async H2D: consecutive batches on the GPU equal the CPU loader's, and
    a training step runs on token-shard input."""
    from dstack_amd.workloads.train_llama import Trainer

    write_shard(str(tmp_path / "t.bin"), np.random.default_rng(1).integers(0, 1000, 200000), np.uint16)
    spec = str(tmp_path / "t.bin")
    g = TokenShards(spec, 256, 4, gpu, seed=3)
    c = TokenShards(spec, 256, 4, "cpu", seed=3)
    for i in range(8):  # more batches than ring slots
        assert torch.equal(g.tokens(i).cpu(), c.tokens(i))
    tr = Trainer("llama-tiny", 256, 2, gpu, data=f"tokens:{spec}", lr_warmup=2)
    losses = [tr.step().item() for _ in range(3)]
    assert all(np.isfinite(losses))


def test_tokenize_text_to_shards(tmp_path):
    """Text -> tokenizer.json ids -> shards the loader reads back in order."""
    from tokenizers import Tokenizer, models, pre_tokenizers

    from dstack_amd.workloads.tokens import main, tokenize_to_shards

    vocab = {w: i for i, w in enumerate(["[UNK]", "<eos>", "the", "mi355x", "trains", "fast", "model"])}
    tok = Tokenizer(models.WordLevel(vocab, unk_token="[UNK]"))
    tok.pre_tokenizer = pre_tokenizers.Whitespace()
    tok.save(str(tmp_path / "tokenizer.json"))
    (tmp_path / "corpus.txt").write_text("the mi355x trains fast\n\nthe model trains\n" * 50)
    paths = tokenize_to_shards(str(tmp_path / "tokenizer.json"), [str(tmp_path / "corpus.txt")],
                               str(tmp_path / "shards"), shard_tokens=120, eos_id=1)
    assert len(paths) == 4  # 50 * (5 + 4) = 450 tokens
    data = np.concatenate([np.fromfile(p, dtype=np.uint16, offset=1024) for p in paths])
    assert data[:9].tolist() == [2, 3, 4, 5, 1, 2, 6, 4, 1]
    main(["info", str(tmp_path / "shards" / "*.bin"), "--seq-len", "16"])
