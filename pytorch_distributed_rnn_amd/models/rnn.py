"""Recurrent layers with nn.LSTM / nn.GRU compatible parameters and state_dicts.

These subclass the stock torch modules so that parameter names
(``weight_ih_l0``, ``weight_hh_l0``, ``bias_ih_l0``, ``bias_hh_l0``, ...),
initialisation and ``state_dict`` layout are byte-for-byte those of
``torch.nn.LSTM`` -- the reference builds its model from ``nn.LSTM``
(reference: src/motion/model.py:9) and its checkpoints must stay loadable.
Only ``forward`` is replaced: on MI355X it dispatches to the fused HIP kernels
(``ops.lstm`` / ``ops.gru``), elsewhere to the ATen reference.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
from torch import Tensor, nn

from ..ops import gru as gru_ops
from ..ops import lstm as lstm_ops


class LSTM(nn.LSTM):
    """``nn.LSTM`` whose forward runs on the fused MI355X kernels.

    Extra keyword ``need_out`` (forward) lets callers that only consume
    ``h_n`` (e.g. a last-timestep classifier) skip the per-timestep output
    stream at inference."""

    def _weights(self):
        ws = []
        for l in range(self.num_layers):
            sfx = f"_l{l}"
            ws += [getattr(self, "weight_ih" + sfx), getattr(self, "weight_hh" + sfx),
                   getattr(self, "bias_ih" + sfx) if self.bias else None,
                   getattr(self, "bias_hh" + sfx) if self.bias else None]
        return ws

    def forward(self, input, hx: Optional[Tuple[Tensor, Tensor]] = None, *, need_out: bool = True,
                idx: Optional[Tensor] = None):  # type: ignore[override]
        if isinstance(input, nn.utils.rnn.PackedSequence) or self.proj_size > 0:
            return super().forward(input, hx)
        unbatched = input.dim() == 2
        if unbatched:
            input = input.unsqueeze(0 if self.batch_first else 1)
            if hx is not None:
                hx = (hx[0].unsqueeze(1), hx[1].unsqueeze(1))
        h0, c0 = (hx if hx is not None else (None, None))
        if self.bidirectional:
            out, hn, cn = lstm_ops.lstm_bidirectional_forward(
                input, self._all_weights_tensors(), h0, c0, hidden=self.hidden_size,
                num_layers=self.num_layers, batch_first=self.batch_first,
                dropout=self.dropout if self.training else 0.0, training=self.training)
        else:
            out, hn, cn = lstm_ops.lstm_forward(
                input, self._weights(), h0, c0, hidden=self.hidden_size,
                num_layers=self.num_layers, batch_first=self.batch_first, need_out=need_out,
                idx=idx, dropout=self.dropout if self.training else 0.0, training=self.training)
        if unbatched:
            out = out.squeeze(0 if self.batch_first else 1) if out is not None else None
            hn, cn = hn.squeeze(1), cn.squeeze(1)
        return out, (hn, cn)

    def _all_weights_tensors(self):
        return [getattr(self, n) for names in self._all_weights for n in names]


class GRU(nn.GRU):
    """``nn.GRU`` whose forward runs on the fused MI355X GRU kernels (small H,
    fp32) or the MFMA step kernels (16-bit, H % 64 == 0, also bidirectional)."""

    def _weights(self):
        ws = []
        for l in range(self.num_layers):
            sfx = f"_l{l}"
            ws += [getattr(self, "weight_ih" + sfx), getattr(self, "weight_hh" + sfx),
                   getattr(self, "bias_ih" + sfx) if self.bias else None,
                   getattr(self, "bias_hh" + sfx) if self.bias else None]
        return ws

    def forward(self, input, hx: Optional[Tensor] = None):  # type: ignore[override]
        if isinstance(input, nn.utils.rnn.PackedSequence):
            return super().forward(input, hx)
        if self.bidirectional:
            from ..ops import gru_large
            if not gru_large.supported(input if input.dim() == 3 else input.unsqueeze(1), self.hidden_size):
                return super().forward(input, hx)
        unbatched = input.dim() == 2
        if unbatched:
            input = input.unsqueeze(0 if self.batch_first else 1)
            if hx is not None:
                hx = hx.unsqueeze(1)
        if self.bidirectional:
            out, hn = gru_large.gru_large_forward(
                input, [getattr(self, n) for names in self._all_weights for n in names], hx,
                hidden=self.hidden_size, num_layers=self.num_layers, batch_first=self.batch_first,
                bidirectional=True, dropout=self.dropout if self.training else 0.0, training=self.training)
        else:
            out, hn = gru_ops.gru_forward(input, self._weights(), hx, hidden=self.hidden_size,
                                          num_layers=self.num_layers, batch_first=self.batch_first,
                                          dropout=self.dropout if self.training else 0.0,
                                          training=self.training)
        if unbatched:
            out, hn = out.squeeze(0 if self.batch_first else 1), hn.squeeze(1)
        return out, hn
