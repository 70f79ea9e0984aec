"""Synthetic token streams for the training workload (no dataset downloads in this environment).

``SyntheticLM`` is the bench's data: a fresh batch for every micro-step (nothing is revisited, so
the model cannot memorise rows), with structure a language model can learn, and a known entropy
floor so a loss curve can be read against it:

* unigram: token ranks follow a Zipf(s) law over the whole vocabulary, mapped to token ids by a
  fixed random permutation (frequent tokens are not simply the low ids);
* bigram chains: with probability ``copy_p`` the next token is ``f(previous)`` for a fixed affine
  map ``f(x) = (A x + B) mod V`` -- an arbitrary permutation from the model's point of view, so it
  has to be learnt per token through the embeddings.

Generation has no sequential loop over positions: for position ``t`` with ``k`` copies since the
last fresh sample ``z_s``, ``x_t = f^k(z_s) = A^k z_s + B (1 + A + ... + A^(k-1)) mod V``, with
``s`` found by a prefix max over the fresh-sample indices.  The random numbers are counter-based
(splitmix64 of the batch key and the position), so every batch is a pure function of
``(seed, index)`` -- a resumed job continues the exact stream -- and the same on every device: on
a GPU one HIP kernel of the extension generates it (``ops/csrc/data.hip``; with PyTorch ops the
first batch of a fresh process paid ~0.37 s for the first use of PyTorch's elementwise kernels,
``profiles/first_step_split_r9j.json``), on the CPU :func:`_tokens_reference` does it in torch ops.
"""

from __future__ import annotations

import math
from typing import Tuple

import torch

_A = 48271  # odd, not a multiple of 3 or 167: a unit mod 128256 (= 2^8 * 3 * 167)
_B = 12345


def _i64(x: int) -> int:
    return x - (1 << 64) if x >= (1 << 63) else x


_C1, _C2, _C3 = _i64(0x9E3779B97F4A7C15), _i64(0xBF58476D1CE4E5B9), _i64(0x94D049BB133111EB)


def _srl(z: torch.Tensor, s: int) -> torch.Tensor:
    """Logical right shift of int64 lanes holding uint64 bit patterns."""
    return (z >> s) & ((1 << (64 - s)) - 1)


def _splitmix64(z: torch.Tensor) -> torch.Tensor:
    """splitmix64 on int64 tensors (two's-complement wrap-around = uint64 arithmetic mod 2^64)."""
    z = z + _C1
    z = (z ^ _srl(z, 30)) * _C2
    z = (z ^ _srl(z, 27)) * _C3
    return z ^ _srl(z, 31)


def _tokens_reference(key: int, n: int, row_len: int, cdf, perm, pow_a, geo_b, copy_p: float, V: int):
    """The stream in torch ops (CPU tensors): the definition ``csrc/data.hip`` implements."""
    i = torch.arange(n, dtype=torch.int64)
    k64 = torch.tensor(_i64(key), dtype=torch.int64)
    x0 = _splitmix64(k64 ^ _splitmix64(2 * i))
    x1 = _splitmix64(k64 ^ _splitmix64(2 * i + 1))
    u = _srl(x0, 11).double() * (2.0 ** -53)
    z = perm[torch.searchsorted(cdf, u).clamp_max_(V - 1)]
    c = _srl(x1, 40).float() * (2.0 ** -24)
    copy = (c < torch.tensor(copy_p, dtype=torch.float32)) & ((i % row_len) != 0)
    last = torch.cummax(torch.where(copy, torch.zeros_like(i), i), 0).values
    k = i - last
    return (pow_a[k] * z[last] + geo_b[k]) % V


class SyntheticLM:
    def __init__(self, vocab_size: int, seq_len: int, micro_batch: int, device, seed: int = 0,
                 zipf_s: float = 1.1, copy_p: float = 0.5):
        self.V, self.S, self.mb = vocab_size, seq_len, micro_batch
        self.device = torch.device(device)
        self.seed = seed
        self.copy_p = copy_p
        if math.gcd(_A, vocab_size) != 1:
            raise ValueError(f"vocab size {vocab_size} shares a factor with the chain multiplier {_A}")
        ranks = torch.arange(1, vocab_size + 1, dtype=torch.float64)
        w = ranks.pow(-zipf_s)
        q = w / w.sum()
        self.unigram_entropy = float(-(q * q.log()).sum())
        self.cdf = torch.cumsum(q, 0).to(self.device)
        g = torch.Generator().manual_seed(seed ^ 0x5EED)
        self.perm = torch.randperm(vocab_size, generator=g).to(self.device)
        n = micro_batch * (seq_len + 1)
        pw, geo = [1], [0]
        for _ in range(n):  # A^k and sum_{j<k} A^j (mod V) for every run length k <= n
            geo.append((geo[-1] + pw[-1]) % vocab_size)
            pw.append(pw[-1] * _A % vocab_size)
        # built on the CPU and copied (no device kernels at construction: the first use of a
        # PyTorch kernel in a process costs tens of milliseconds)
        self.pow_a = torch.tensor(pw, dtype=torch.int64).to(self.device)
        self.geo_b = (torch.tensor(geo, dtype=torch.int64) * _B % vocab_size).to(self.device)
        self.row_start = (torch.arange(n) % (seq_len + 1)) == 0  # (CPU; documents the row layout)
        self._ws = None  # the HIP kernel's workspace, allocated at the first GPU batch

    @property
    def loss_floor(self) -> float:
        """Entropy (nats/token) of the stream given the previous token: the best achievable loss
        (up to the small chance that a fresh sample equals ``f(previous)``)."""
        p = self.copy_p
        h = -(p * math.log(p) + (1 - p) * math.log(1 - p)) if 0 < p < 1 else 0.0
        return h + (1 - p) * self.unigram_entropy

    def key(self, index: int) -> int:
        return (self.seed * 1_000_003 + index) & 0x7FFF_FFFF_FFFF_FFFF

    def tokens(self, index: int) -> torch.Tensor:
        """``micro_batch x (seq_len + 1)`` token ids of micro-batch ``index``."""
        n = self.mb * (self.S + 1)
        if self.device.type == "cuda":
            from dstack_amd.ops import _ext

            C = _ext.require()
            if self._ws is None:
                self._ws = torch.empty(n, dtype=torch.int64, device=self.device)
            out = torch.empty(n, dtype=torch.int64, device=self.device)
            C.synthetic_tokens(self.cdf, self.perm, self.pow_a, self.geo_b, out, self._ws, self.key(index),
                               float(self.copy_p), self.S + 1)
            return out.view(self.mb, self.S + 1)
        x = _tokens_reference(self.key(index), n, self.S + 1, self.cdf, self.perm, self.pow_a, self.geo_b,
                              self.copy_p, self.V)
        return x.view(self.mb, self.S + 1)

    def batch(self, index: int) -> Tuple[torch.Tensor, torch.Tensor]:
        rows = self.tokens(index)
        return rows[:, :-1], rows[:, 1:]
