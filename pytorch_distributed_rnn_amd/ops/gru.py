"""GRU stack operator: fused HIP kernels for small hidden sizes (fp32), the MFMA
step kernels for 16-bit inputs with H % 64 == 0 (ops/gru_large.py), ATen otherwise.

New capability (BASELINE.json names an "LSTM/GRU cell"; the reference itself
only uses nn.LSTM).  Gate order and parameters follow nn.GRU
(r, z, n; n = tanh(W_in x + b_in + r * (W_hn h + b_hn))).
"""
from __future__ import annotations

from typing import Optional, Sequence, Tuple

import torch
from torch import Tensor

from .. import _ext


def gru_reference(x: Tensor, weights: Sequence[Optional[Tensor]], h0: Optional[Tensor], hidden: int,
                  num_layers: int, batch_first: bool, dropout: float = 0.0,
                  training: bool = False) -> Tuple[Tensor, Tensor]:
    has_bias = weights[2] is not None
    flat = [w for w in weights if w is not None]
    if h0 is None:
        b = x.shape[0] if batch_first else x.shape[1]
        h0 = x.new_zeros(num_layers, b, hidden)
    out, hn = torch._VF.gru(x, h0, flat, has_bias, num_layers, dropout, training, False, batch_first)
    return out, hn


def fused_small_supported(x: Tensor, hidden: int, num_layers: int) -> bool:
    from . import gru_fused
    return gru_fused.supported(x, hidden, num_layers)


def gru_forward(x: Tensor, weights: Sequence[Optional[Tensor]], h0: Optional[Tensor] = None, *,
                hidden: int, num_layers: int, batch_first: bool = False, dropout: float = 0.0,
                training: bool = False) -> Tuple[Tensor, Tensor]:
    if dropout == 0.0 and fused_small_supported(x, hidden, num_layers):
        from .gru_fused import fused_gru
        return fused_gru(x, weights, h0, hidden=hidden, num_layers=num_layers, batch_first=batch_first)
    from . import gru_large
    if gru_large.supported(x, hidden):
        return gru_large.gru_large_forward(x, weights, h0, hidden=hidden, num_layers=num_layers,
                                           batch_first=batch_first, dropout=dropout, training=training)
    return gru_reference(x, weights, h0, hidden, num_layers, batch_first, dropout, training)
