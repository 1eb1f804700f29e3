"""Fused small-H GRU stack on the gate-split / unit-group kernels of
csrc/kernels/lstm_small.hip (CELL = GRU).

The GRU's three gates are laid out on the LSTM kernels' four-lane quad as
[r | z | n_x | n_h] -- n_x = W_in x + b_in and n_h = W_hn h + b_hn stay
separate because n = tanh(n_x + r * n_h).  The host packs nn.GRU's
parameters into 4-block stacks with zero blocks:

    W_ih4 = [W_ir; W_iz; W_in; 0]      W_hh4 = [W_hr; W_hz; 0; W_hn]
    b_ih4 = [b_ir; b_iz; b_in; 0]      b_hh4 = [b_hr; b_hz; 0; b_hn]

so the forward dot products, the BPTT column phase (W^T g and the dW outer
products) and the deterministic slab reduction are shared with the LSTM
kernels; only the cell math differs.  Gradients come back in the packed
layout and are unpacked here to nn.GRU's.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch
from torch import Tensor

from .. import _ext


def supported(x: Tensor, hidden: int, num_layers: int) -> bool:
    if x.dtype != torch.float32 or x.dim() != 3 or x.device.type != "cuda":
        return False
    mod = _ext.native(x.device)
    if mod is None or not mod.lstm_small_supported(hidden, x.shape[-1], num_layers):
        return False
    lanes = 8 if hidden >= 64 else 4
    return num_layers * 4 * hidden <= 512 and num_layers * hidden * lanes <= 512


def _pack(weights: Sequence[Optional[Tensor]], num_layers: int, hidden: int, like: Tensor) -> List[Tensor]:
    H = hidden
    out = []
    with torch.no_grad():
        for l in range(num_layers):
            w_ih, w_hh, b_ih, b_hh = weights[4 * l:4 * l + 4]
            I = w_ih.shape[1]
            z_ih = like.new_zeros(H, I)
            z_hh = like.new_zeros(H, H)
            zb = like.new_zeros(H)
            b_ih = b_ih if b_ih is not None else like.new_zeros(3 * H)
            b_hh = b_hh if b_hh is not None else like.new_zeros(3 * H)
            out += [torch.cat([w_ih, z_ih]).contiguous(),
                    torch.cat([w_hh[:2 * H], z_hh, w_hh[2 * H:]]).contiguous(),
                    torch.cat([b_ih, zb]).contiguous(),
                    torch.cat([b_hh[:2 * H], zb, b_hh[2 * H:]]).contiguous()]
    return out


class _FusedSmallGRU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, h0, cfg, *weights):
        hidden, num_layers, batch_first = cfg
        mod = _ext.native(x.device)
        packed = _pack(weights, num_layers, hidden, x)
        h0c = h0.contiguous() if h0 is not None else None
        out, hn, _, act = mod.lstm_small_fwd(x, None, packed, h0c, None, hidden, num_layers, batch_first,
                                             True, True, 1, 1, cell=1)
        ctx.set_materialize_grads(False)
        ctx.cfg = (hidden, num_layers, batch_first, [w is not None for w in weights])
        ctx.save_for_backward(x, h0c, out, act, *packed)
        top = out[num_layers - 1]
        if not batch_first:
            top = top.transpose(0, 1)
        return top, hn

    @staticmethod
    def backward(ctx, dout, dhn):
        x, h0, hseq, act, *packed = ctx.saved_tensors
        hidden, num_layers, batch_first, present = ctx.cfg
        H = hidden
        mod = _ext.native(x.device)
        need_dx = ctx.needs_input_grad[0]
        need_dh0 = ctx.needs_input_grad[1]
        if dout is not None and dout.stride(-1) != 1:
            dout = dout.contiguous()
        dhn = dhn.contiguous() if dhn is not None else None
        dparams, dx, dh0, _ = mod.lstm_small_bwd(x, None, packed, h0, None, hseq, act, dout, dhn, None, H,
                                                 num_layers, batch_first, need_dx, need_dh0, 1, 1, None, cell=1)
        grads: List[Optional[Tensor]] = []
        off = 0
        for l in range(num_layers):
            views = []
            for w in packed[4 * l:4 * l + 4]:
                views.append(dparams[off:off + w.numel()].view_as(w))
                off += w.numel()
            dwih4, dwhh4, dbih4, dbhh4 = views
            gl = [dwih4[:3 * H],
                  torch.cat([dwhh4[:2 * H], dwhh4[3 * H:]]),
                  dbih4[:3 * H],
                  torch.cat([dbhh4[:2 * H], dbhh4[3 * H:]])]
            grads += [g if present[4 * l + k] else None for k, g in enumerate(gl)]
        return (dx if need_dx else None, dh0 if need_dh0 else None, None, *grads)


def fused_gru(x: Tensor, weights: Sequence[Optional[Tensor]], h0: Optional[Tensor], *, hidden: int,
              num_layers: int, batch_first: bool) -> Tuple[Tensor, Tensor]:
    return _FusedSmallGRU.apply(x, h0, (hidden, num_layers, batch_first), *weights)
