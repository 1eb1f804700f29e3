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
    drop = dropout if training else 0.0
    if x.dtype == torch.float32:
        from .gru_fused import fused_gru
        from .lstm import _pad_state, pad_gate_rows, small_plan
        plan = small_plan(x, hidden, num_layers, cell="gru", per_layer=drop > 0, batch_first=batch_first)
        if plan is not None:
            hp, chunks = plan
            if hp == hidden and len(chunks) == 1:
                return fused_gru(x, weights, h0, hidden=hidden, num_layers=num_layers, batch_first=batch_first)
            # zero-padded units: r = z = 1/2, n = tanh(0) = 0 -> h stays exactly 0
            h, hns = x, []
            for k, (l0, n) in enumerate(chunks):
                ws = list(weights[4 * l0:4 * (l0 + n)])
                if hp != hidden:
                    for j in range(n):
                        in_pad = None if l0 + j == 0 else hp
                        ws[4 * j:4 * j + 4] = [pad_gate_rows(ws[4 * j], hidden, hp, 3, in_pad),
                                               pad_gate_rows(ws[4 * j + 1], hidden, hp, 3, hp),
                                               pad_gate_rows(ws[4 * j + 2], hidden, hp, 3),
                                               pad_gate_rows(ws[4 * j + 3], hidden, hp, 3)]
                hh = _pad_state(h0[l0:l0 + n], hidden, hp) if h0 is not None else None
                out, hn = fused_gru(h, ws, hh, hidden=hp, num_layers=n, batch_first=batch_first)
                hns.append(hn)
                if k < len(chunks) - 1 and drop > 0:
                    out = torch.nn.functional.dropout(out, drop, True)
                h = out
            hn = torch.cat(hns)
            if hp != hidden:
                h, hn = h[..., :hidden], hn[..., :hidden]
            return h, hn
    from . import gru_large
    if gru_large.supported(x, hidden):
        return gru_large.gru_large_forward(x, weights, h0, hidden=hidden, num_layers=num_layers,
                                           batch_first=batch_first, dropout=dropout, training=training)
    _ext.fallback(f"GRU(H={hidden}, I={x.shape[-1]}, layers={num_layers}, {x.dtype})", x.device)
    return gru_reference(x, weights, h0, hidden, num_layers, batch_first, dropout, training)
