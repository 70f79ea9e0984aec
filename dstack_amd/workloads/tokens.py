"""Real-data input for the training workload: token shards read by the native loader
(``native/dataloader/tokloader.cpp``, C ABI over ctypes).

Shards are flat binary token files -- uint16 / uint32 ids, optionally with the 1 KiB llm.c header
(``write_shard`` writes that format).  The loader memory-maps them, cuts the corpus into
non-overlapping ``seq_len + 1`` windows, visits every window once per epoch in a seeded order,
gives every data-parallel rank disjoint windows, and assembles batches on a background thread
ahead of the training step; batch ``i`` is a pure function of (shards, seed, rank, world, i), so a
job resumed from a checkpoint continues the exact stream (``Trainer`` stores the batch index).

    Trainer(..., data="tokens:/data/fineweb/*.bin")        # or: train_llama --data tokens:...
"""

from __future__ import annotations

import ctypes
import glob
import os
from typing import List, Sequence, Tuple

import numpy as np
import torch

from dstack_amd.native_bin import BUILD_DIR, build_native

_LIB = None


def _lib():
    global _LIB
    if _LIB is None:
        path = os.environ.get("DSTACK_TOKLOADER_LIB") or str(BUILD_DIR / "libdstack_tokloader.so")
        if not os.path.exists(path):
            build_native(("build/libdstack_tokloader.so",))
        lib = ctypes.CDLL(path)
        lib.tl_open.restype = ctypes.c_void_p
        lib.tl_open.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                ctypes.c_int, ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                ctypes.c_char_p, ctypes.c_int]
        lib.tl_next.restype = ctypes.c_int
        lib.tl_next.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]
        lib.tl_seek.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
        for fn in ("tl_num_windows", "tl_num_tokens", "tl_batches_per_epoch"):
            getattr(lib, fn).restype = ctypes.c_uint64
            getattr(lib, fn).argtypes = [ctypes.c_void_p]
        lib.tl_close.argtypes = [ctypes.c_void_p]
        _LIB = lib
    return _LIB


MAGIC = 20240520


def write_shard(path: str, tokens, dtype=np.uint16, header: bool = True) -> None:
    """Write token ids as a shard (llm.c header: magic, version 1 = uint16 / 2 = uint32, count)."""
    arr = np.asarray(tokens, dtype=dtype)
    with open(path, "wb") as f:
        if header:
            hdr = np.zeros(256, dtype=np.int32)
            hdr[0], hdr[1], hdr[2] = MAGIC, (2 if arr.dtype == np.uint32 else 1), arr.size
            f.write(hdr.tobytes())
        f.write(arr.tobytes())


def expand_paths(spec) -> List[str]:
    items = [spec] if isinstance(spec, str) else list(spec)
    out: List[str] = []
    for it in items:
        for part in str(it).split(","):
            hits = sorted(glob.glob(part))
            if not hits:
                raise FileNotFoundError(f"no token shards match {part!r}")
            out.extend(hits)
    return out


class TokenShards:
    def __init__(self, paths, seq_len: int, micro_batch: int, device, seed: int = 0, rank: int = 0, world: int = 1,
                 token_bytes: int = 0, prefetch: int = 4, vocab_size: int | None = None):
        self.paths = expand_paths(paths)
        self.S, self.mb = seq_len, micro_batch
        self.device = torch.device(device)
        self.vocab_size = vocab_size
        lib = _lib()
        arr = (ctypes.c_char_p * len(self.paths))(*[p.encode() for p in self.paths])
        err = ctypes.create_string_buffer(512)
        self._h = lib.tl_open(arr, len(self.paths), token_bytes, seq_len, micro_batch, seed, rank, world, prefetch,
                              err, len(err))
        if not self._h:
            raise ValueError(f"token loader: {err.value.decode()}")
        self._next = 0
        # a ring of pinned host buffers: the H2D copy of batch i is asynchronous, so its buffer is
        # reused only after the copy's event has completed
        cuda = self.device.type == "cuda"
        self._ring = [torch.empty(micro_batch * (seq_len + 1), dtype=torch.int32, pin_memory=cuda) for _ in range(3)]
        self._events = [None] * len(self._ring)
        self._slot = 0

    @property
    def num_tokens(self) -> int:
        return int(_lib().tl_num_tokens(self._h))

    @property
    def batches_per_epoch(self) -> int:
        return int(_lib().tl_batches_per_epoch(self._h))

    def tokens(self, index: int) -> torch.Tensor:
        """``micro_batch x (seq_len + 1)`` int64 tokens of batch ``index`` on the device."""
        lib = _lib()
        if index != self._next:
            lib.tl_seek(self._h, index)
        k = self._slot
        self._slot = (k + 1) % len(self._ring)
        if self._events[k] is not None:
            self._events[k].synchronize()
        host = self._ring[k]
        got = ctypes.c_uint64(0)
        if lib.tl_next(self._h, ctypes.c_void_p(host.data_ptr()), ctypes.byref(got)) != 0:
            raise RuntimeError("token loader stopped")
        assert got.value == index, (got.value, index)
        self._next = index + 1
        if self.vocab_size is not None:
            hi = int(host.max())
            if hi >= self.vocab_size:
                raise ValueError(f"token id {hi} >= vocab size {self.vocab_size}: shards of another tokenizer?")
        # (on the CPU the ring buffer itself would be handed out and overwritten two batches later)
        t = host.to(self.device, non_blocking=True) if self.device.type == "cuda" else host.clone()
        if self.device.type == "cuda":
            ev = torch.cuda.Event()
            ev.record()
            self._events[k] = ev
        return t.view(self.mb, self.S + 1).long()

    def batch(self, index: int) -> Tuple[torch.Tensor, torch.Tensor]:
        rows = self.tokens(index)
        return rows[:, :-1], rows[:, 1:]

    def close(self) -> None:
        if getattr(self, "_h", None):
            _lib().tl_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 -- interpreter teardown
            pass


def shard_paths_of(spec: str) -> Sequence[str]:
    """``tokens:<glob>[,<glob>...]`` -> shard paths."""
    return expand_paths(spec.split(":", 1)[1] if spec.startswith("tokens:") else spec)


def tokenize_to_shards(tokenizer_path: str, inputs: Sequence[str], out_dir: str, shard_tokens: int = 100_000_000,
                       eos_id: int | None = None, prefix: str = "shard") -> List[str]:
    """Tokenize text files (one document per line, or whole files with ``--whole-files``) with an
    HF ``tokenizer.json`` into shards of ``shard_tokens`` tokens (uint16 ids when the vocabulary
    fits, uint32 otherwise), an end-of-text id between documents.  Returns the shard paths."""
    from tokenizers import Tokenizer

    tok = Tokenizer.from_file(tokenizer_path)
    vocab = tok.get_vocab_size()
    dtype = np.uint16 if vocab <= 65536 else np.uint32
    os.makedirs(out_dir, exist_ok=True)
    paths: List[str] = []
    buf: List[int] = []

    def flush(final=False):
        while len(buf) >= shard_tokens or (final and buf):
            chunk, buf[:] = buf[:shard_tokens], buf[shard_tokens:]
            path = os.path.join(out_dir, f"{prefix}_{len(paths):05d}.bin")
            write_shard(path, chunk, dtype)
            paths.append(path)

    for fn in inputs:
        with open(fn, encoding="utf-8") as f:
            for line in f:
                line = line.rstrip("\n")
                if not line:
                    continue
                buf.extend(tok.encode(line).ids)
                if eos_id is not None:
                    buf.append(eos_id)
                if len(buf) >= shard_tokens:
                    flush()
    flush(final=True)
    return paths


def main(argv=None):
    import argparse

    ap = argparse.ArgumentParser(description="token shards for train_llama --data tokens:<glob>")
    sub = ap.add_subparsers(dest="cmd", required=True)
    t = sub.add_parser("tokenize", help="text files -> token shards")
    t.add_argument("--tokenizer", required=True, help="HF tokenizer.json")
    t.add_argument("--out", required=True)
    t.add_argument("--shard-tokens", type=int, default=100_000_000)
    t.add_argument("--eos-id", type=int, default=None)
    t.add_argument("inputs", nargs="+")
    i = sub.add_parser("info", help="token and window counts of shards")
    i.add_argument("glob")
    i.add_argument("--seq-len", type=int, default=8192)
    a = ap.parse_args(argv)
    if a.cmd == "tokenize":
        for p in tokenize_to_shards(a.tokenizer, a.inputs, a.out, a.shard_tokens, a.eos_id):
            print(p)
    else:
        ts = TokenShards(a.glob, a.seq_len, 1, "cpu")
        print(f"{len(ts.paths)} shards, {ts.num_tokens} tokens, {ts.batches_per_epoch} windows of {a.seq_len}")


if __name__ == "__main__":
    main()
