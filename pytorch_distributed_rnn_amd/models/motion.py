"""Motion (UCI-HAR activity) classifier: stacked LSTM + linear head.

Same architecture, constructor signature and ``state_dict`` keys as the
reference ``MotionModel`` (reference: src/motion/model.py:4-17):
``lstm.weight_ih_l{k}``, ``lstm.weight_hh_l{k}``, ``lstm.bias_ih_l{k}``,
``lstm.bias_hh_l{k}``, ``fc.weight``, ``fc.bias``; logits come from the
top layer's hidden state at the last timestep.

MI355X specifics: the LSTM stack runs as one fused HIP launch per direction of
the pass, and the classifier reads the top layer's final hidden state ``h_n``
directly (identical to ``out[:, -1, :]`` for a unidirectional LSTM) so that
neither the forward nor the backward materialises the [B, T, H] output stream
(its gradient is zero everywhere except the last step).
"""
from __future__ import annotations

from typing import Optional

import torch
from torch import Tensor, nn

from .rnn import GRU, LSTM
from ..ops.gemm import linear


class MotionModel(nn.Module):
    # forward(features, idx=...) gathers the batch rows inside the fused kernel
    supports_index_batches = True

    def __init__(self, input_dim: int, hidden_dim: int, layer_dim: int, output_dim: int,
                 cell: str = "lstm", dropout: float = 0.0, compute_dtype: torch.dtype = torch.float32,
                 bidirectional: bool = False):
        super().__init__()
        self.bidirectional = bidirectional
        # bf16: inputs and recurrent weights in bf16 storage, fp32 accumulation,
        # cell state and master weights (BASELINE config 2)
        self.compute_dtype = compute_dtype
        self.hidden_dim = hidden_dim
        self.layer_dim = layer_dim
        self.cell = cell
        rnn_cls = {"lstm": LSTM, "gru": GRU}[cell]
        # attribute name kept as `lstm` for checkpoint compatibility
        self.lstm = rnn_cls(input_dim, hidden_dim, layer_dim, batch_first=True, dropout=dropout,
                            bidirectional=bidirectional)
        # bidirectional (extension): the head reads out[:, -1, :] = [h_fwd(T-1), h_bwd(T-1)]
        self.fc = nn.Linear(hidden_dim * (2 if bidirectional else 1), output_dim)

    def forward(self, x: Tensor, idx: Optional[Tensor] = None) -> Tensor:
        if self.compute_dtype != torch.float32 and x.dtype != self.compute_dtype:
            x = x.to(self.compute_dtype)
        if self.bidirectional:
            if idx is not None:
                x = x.index_select(0, idx)
            out, _ = self.lstm(x)
            return self._head(out[:, -1, :])
        if self.cell == "lstm":
            _, (hn, _) = self.lstm(x, need_out=False, idx=idx)
        else:
            if idx is not None:
                x = x.index_select(0, idx)
            _, hn = self.lstm(x)
        return self._head(hn[-1])

    def _head(self, h: Tensor) -> Tensor:
        """The linear head; on the GPU on the in-tree narrow fp32 GEMM
        (ops/gemm.linear: forward, dX, dW with db as its row sums)."""
        h = h if h.dtype == self.fc.weight.dtype else h.to(self.fc.weight.dtype)
        if h.is_cuda:
            return linear(h, self.fc.weight, self.fc.bias)
        return self.fc(h)
