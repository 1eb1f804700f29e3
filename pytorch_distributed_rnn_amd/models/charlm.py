"""Character-level LSTM language model (BASELINE config 4: 2-layer LSTM,
hidden 1024, seq_len 512, DDP) and the stacked bidirectional LSTM encoder
(BASELINE config 5: hidden 4096, fp16).

Neither model exists in the reference (no GRU / embedding /
char-LM there); they reuse its building blocks -- ``nn.LSTM``-compatible
layers whose forward runs on the framework's kernels -- and make
``_reset_hidden_state`` real (the reference's is dead code,
reference: src/motion/trainer/base.py:161-162) for truncated BPTT.

Precision: parameters are fp32 masters; the recurrent stack, the embedding
output and the vocabulary projection run in ``compute_dtype`` (bf16 / fp16 on
MI355X), the loss in fp32.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
from torch import Tensor, nn
from torch.nn import functional as F

from ..ops.embedding import embedding
from ..ops.gemm import linear
from .rnn import LSTM


class CharLM(nn.Module):
    def __init__(self, vocab_size: int = 256, embed_dim: int = 256, hidden_dim: int = 1024,
                 num_layers: int = 2, dropout: float = 0.0, compute_dtype: torch.dtype = torch.bfloat16):
        super().__init__()
        self.vocab_size = vocab_size
        self.hidden_dim = hidden_dim
        self.num_layers = num_layers
        self.compute_dtype = compute_dtype
        self.embedding = nn.Embedding(vocab_size, embed_dim)
        self.lstm = LSTM(embed_dim, hidden_dim, num_layers, batch_first=False, dropout=dropout)
        self.fc = nn.Linear(hidden_dim, vocab_size)
        self._state: Optional[Tuple[Tensor, Tensor]] = None

    def reset_hidden_state(self) -> None:
        """Start a new TBPTT stream (called at every epoch start)."""
        self._state = None

    def _cdt(self, device) -> torch.dtype:
        return self.compute_dtype if device.type == "cuda" else torch.float32

    def forward(self, tokens: Tensor, state: Optional[Tuple[Tensor, Tensor]] = None,
                carry: bool = False) -> Tensor:
        """tokens [B, T] -> logits [T, B, V] (sequence-first, compute dtype).

        ``carry=True`` continues from (and updates) the detached state of the
        previous segment -- truncated BPTT over a long stream."""
        cdt = self._cdt(tokens.device)
        x = embedding(tokens.t(), self.embedding.weight, out_dtype=cdt)      # [T, B, E]
        if state is None and carry:
            state = self._state
        out, (hn, cn) = self.lstm(x, state)
        if carry:
            self._state = (hn.detach(), cn.detach())
        return linear(out, self.fc.weight, self.fc.bias)  # in-tree GEMM head (ops/gemm.py)


class BiLSTMEncoder(nn.Module):
    """Stacked bidirectional LSTM with a per-timestep linear head."""

    def __init__(self, input_dim: int, hidden_dim: int, num_layers: int, output_dim: int,
                 compute_dtype: torch.dtype = torch.float16):
        super().__init__()
        self.compute_dtype = compute_dtype
        self.lstm = LSTM(input_dim, hidden_dim, num_layers, batch_first=False, bidirectional=True)
        self.fc = nn.Linear(2 * hidden_dim, output_dim)

    def forward(self, x: Tensor) -> Tensor:
        """x [T, B, I] -> [T, B, output_dim]."""
        cdt = self.compute_dtype if x.is_cuda else torch.float32
        out, _ = self.lstm(x.to(cdt))
        return linear(out, self.fc.weight, self.fc.bias)
