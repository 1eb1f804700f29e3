"""Token streams for the char-LM: a text file as bytes, or a synthetic corpus
with learnable structure (no network: no dataset download).

Batching is the classic TBPTT layout: the token stream is cut into
``global_batch`` parallel streams; rank r of W owns streams
[r*B/W, (r+1)*B/W) (data parallel), and consecutive ``seq_len`` windows of
each stream are consecutive training segments, so the hidden state carried
from one segment to the next is the true continuation.
"""
from __future__ import annotations

from pathlib import Path
from typing import Iterator, Optional, Tuple

import numpy as np
import torch
from torch import Tensor


class CharCorpus:
    def __init__(self, tokens: Tensor, vocab_size: int = 256):
        assert tokens.dtype == torch.int64 and tokens.dim() == 1
        self.tokens = tokens
        self.vocab_size = vocab_size

    def __len__(self) -> int:
        return self.tokens.numel()

    @classmethod
    def from_text(cls, path: Path) -> "CharCorpus":
        data = np.frombuffer(Path(path).read_bytes(), dtype=np.uint8).astype(np.int64)
        return cls(torch.from_numpy(data.copy()), 256)

    @classmethod
    def synthetic(cls, n_tokens: int, vocab_size: int = 256, n_words: int = 2000, seed: int = 0) -> "CharCorpus":
        """Zipf-distributed 'words' (random letter strings) separated by a space
        token: enough structure that the LM's loss falls well below log(V)."""
        rng = np.random.default_rng(seed)
        letters = np.arange(1, min(vocab_size, 96))
        lens = rng.integers(2, 10, size=n_words)
        table = rng.choice(letters, size=int(lens.sum()))
        starts = np.concatenate([[0], np.cumsum(lens)[:-1]])
        p = 1.0 / np.arange(1, n_words + 1)
        p /= p.sum()
        n_est = int(n_tokens / (lens.mean() + 1)) + 16
        out = np.empty(0, dtype=np.int64)
        while out.size < n_tokens:
            ids = rng.choice(n_words, size=n_est, p=p)
            wl = lens[ids] + 1                                  # word + separator
            pos = np.repeat(np.cumsum(wl) - wl, wl)
            off = np.arange(wl.sum()) - pos
            src = np.repeat(starts[ids], wl) + off
            tok = np.where(off == np.repeat(lens[ids], wl), 0, table[np.minimum(src, table.size - 1)])
            out = np.concatenate([out, tok.astype(np.int64)])
        return cls(torch.from_numpy(out[:n_tokens].copy()), vocab_size)

    def to(self, device) -> "CharCorpus":
        return CharCorpus(self.tokens.to(device), self.vocab_size)

    def streams(self, global_batch: int, rank: int = 0, world: int = 1) -> Tensor:
        """[global_batch / world, L] token streams owned by this rank."""
        if global_batch % world:
            raise ValueError(f"global batch {global_batch} not divisible by world size {world}")
        L = self.tokens.numel() // global_batch
        data = self.tokens[: L * global_batch].view(global_batch, L)
        per = global_batch // world
        return data[rank * per:(rank + 1) * per]

    @staticmethod
    def segments(streams: Tensor, seq_len: int, limit: Optional[int] = None) -> Iterator[Tuple[Tensor, Tensor]]:
        """Consecutive (input, target) windows [b, seq_len] for truncated BPTT."""
        L = streams.shape[1]
        n = (L - 1) // seq_len
        if limit is not None:
            n = min(n, limit)
        for i in range(n):
            s = i * seq_len
            yield streams[:, s:s + seq_len], streams[:, s + 1:s + 1 + seq_len]
