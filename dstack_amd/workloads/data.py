"""Synthetic token streams for the training workload (no dataset downloads in this environment).

``SyntheticLM`` is the bench's data: a fresh batch for every micro-step (nothing is revisited, so
the model cannot memorise rows), with structure a language model can learn, and a known entropy
floor so a loss curve can be read against it:

* unigram: token ranks follow a Zipf(s) law over the whole vocabulary, mapped to token ids by a
  fixed random permutation (frequent tokens are not simply the low ids);
* bigram chains: with probability ``copy_p`` the next token is ``f(previous)`` for a fixed affine
  map ``f(x) = (A x + B) mod V`` -- an arbitrary permutation from the model's point of view, so it
  has to be learnt per token through the embeddings.

Generation is vectorised on the device (no sequential loop over positions): for position ``t``
with ``k`` copies since the last fresh sample ``z_s``, ``x_t = f^k(z_s) = A^k z_s + B (1 + A + ...
+ A^(k-1)) mod V``, with ``s`` found by a cumulative max over the fresh-sample indices.  Every batch
is a pure function of ``(seed, index)``, so a resumed job continues the exact stream.
"""

from __future__ import annotations

import math
from typing import Tuple

import torch

_A = 48271  # odd, not a multiple of 3 or 167: a unit mod 128256 (= 2^8 * 3 * 167)
_B = 12345


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
        self.pow_a = torch.tensor(pw, dtype=torch.int64, device=self.device)
        self.geo_b = torch.tensor(geo, dtype=torch.int64, device=self.device) * _B % vocab_size
        self.idx = torch.arange(n, device=self.device)
        self.row_start = (self.idx % (seq_len + 1)) == 0
        self.gen = torch.Generator(device=self.device)

    @property
    def loss_floor(self) -> float:
        """Entropy (nats/token) of the stream given the previous token: the best achievable loss
        (up to the small chance that a fresh sample equals ``f(previous)``)."""
        p = self.copy_p
        h = -(p * math.log(p) + (1 - p) * math.log(1 - p)) if 0 < p < 1 else 0.0
        return h + (1 - p) * self.unigram_entropy

    def tokens(self, index: int) -> torch.Tensor:
        """``micro_batch x (seq_len + 1)`` token ids of micro-batch ``index``."""
        self.gen.manual_seed((self.seed * 1_000_003 + index) & 0x7FFF_FFFF_FFFF)
        n = self.idx.numel()
        u = torch.rand(n, generator=self.gen, device=self.device, dtype=torch.float64)
        z = self.perm[torch.searchsorted(self.cdf, u).clamp_max_(self.V - 1)]
        copy = torch.rand(n, generator=self.gen, device=self.device) < self.copy_p
        copy &= ~self.row_start  # every row starts from a fresh sample
        last = torch.cummax(torch.where(copy, torch.zeros_like(self.idx), self.idx), 0).values
        k = self.idx - last
        x = (self.pow_a[k] * z[last] + self.geo_b[k]) % self.V
        return x.view(self.mb, self.S + 1)

    def batch(self, index: int) -> Tuple[torch.Tensor, torch.Tensor]:
        rows = self.tokens(index)
        return rows[:, :-1], rows[:, 1:]
