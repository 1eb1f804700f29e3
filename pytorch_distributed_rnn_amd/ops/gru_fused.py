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

from typing import Dict, List, Optional, Sequence, Tuple

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


_ZEROS: Dict[Tuple[torch.device, torch.dtype], Tensor] = {}
# superseded zero vectors stay referenced: a cat on another stream may still
# be reading one (they are never written, so sharing is safe; a few KB each)
_RETIRED: List[Tensor] = []
_UNPACK: Dict[Tuple[int, Tuple[int, ...], torch.device], Tensor] = {}


def _zeros(like: Tensor, n: int) -> Tensor:
    """Slice of a cached zero vector (the packed layout's empty blocks)."""
    key = (like.device, like.dtype)
    z = _ZEROS.get(key)
    if z is None or z.numel() < n:
        if z is not None:
            _RETIRED.append(z)
        z = like.new_zeros(max(n, 1024))
        _ZEROS[key] = z
    return z[:n]


def packed_numel(weights: Sequence[Optional[Tensor]], num_layers: int, hidden: int) -> int:
    """Elements of the 4-block stacks of all layers (the ``out`` buffer of _pack)."""
    H = hidden
    return sum(4 * H * int(weights[4 * l].shape[1]) + 4 * H * H + 8 * H for l in range(num_layers))


def _pack(weights: Sequence[Optional[Tensor]], num_layers: int, hidden: int, like: Tensor,
          out: Optional[Tensor] = None) -> List[Tensor]:
    """All layers' 4-block stacks as views of ONE buffer built by a single
    batched cat launch (the zero blocks are slices of a cached zero vector),
    instead of a cat + zero fill per tensor per step.  ``out``: a persistent
    buffer of ``packed_numel`` elements the cat writes into -- no allocation,
    so the fused step can capture it in a HIP graph and every replay re-packs
    the current parameters."""
    H = hidden
    pieces: List[Tensor] = []
    shapes: List[Tuple[int, ...]] = []
    with torch.no_grad():
        for l in range(num_layers):
            w_ih, w_hh, b_ih, b_hh = weights[4 * l:4 * l + 4]
            I = w_ih.shape[1]
            zb = _zeros(like, H)
            b_ih = b_ih.reshape(-1) if b_ih is not None else _zeros(like, 3 * H)
            b_hh = b_hh.reshape(-1) if b_hh is not None else _zeros(like, 3 * H)
            pieces += [w_ih.reshape(-1), _zeros(like, H * I),
                       w_hh[:2 * H].reshape(-1), _zeros(like, H * H), w_hh[2 * H:].reshape(-1),
                       b_ih, zb, b_hh[:2 * H], zb, b_hh[2 * H:]]
            shapes += [(4 * H, I), (4 * H, H), (4 * H,), (4 * H,)]
        flat = torch.cat(pieces) if out is None else torch.cat(pieces, out=out)
    views, off = [], 0
    for s in shapes:
        n = 1
        for d in s:
            n *= d
        views.append(flat[off:off + n].view(s))
        off += n
    return views


def _unpack_index(hidden: int, in_dims: Tuple[int, ...], device: torch.device) -> Tensor:
    """Gather map from the packed gradient vector to nn.GRU's parameter order
    (per layer: dW_ih = rows [0, 3H) of its block, dW_hh / db_hh = rows
    [0, 2H) and [3H, 4H), db_ih = [0, 3H)); one index_select per step."""
    key = (hidden, in_dims, device)
    idx = _UNPACK.get(key)
    if idx is None:
        H, parts, off = hidden, [], 0
        for I in in_dims:
            parts.append(torch.arange(off, off + 3 * H * I)); off += 4 * H * I
            parts += [torch.arange(off, off + 2 * H * H), torch.arange(off + 3 * H * H, off + 4 * H * H)]
            off += 4 * H * H
            parts.append(torch.arange(off, off + 3 * H)); off += 4 * H
            parts += [torch.arange(off, off + 2 * H), torch.arange(off + 3 * H, off + 4 * H)]
            off += 4 * H
        idx = torch.cat(parts).to(device)
        _UNPACK[key] = idx
    return idx


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
        in_dims = tuple(int(packed[4 * l].shape[1]) for l in range(num_layers))
        g = dparams.index_select(0, _unpack_index(H, in_dims, dparams.device))
        grads: List[Optional[Tensor]] = []
        off = 0
        for l, I in enumerate(in_dims):
            for k, s in enumerate(((3 * H, I), (3 * H, H), (3 * H,), (3 * H,))):
                n = s[0] * (s[1] if len(s) > 1 else 1)
                grads.append(g[off:off + n].view(s) if present[4 * l + k] else None)
                off += n
        return (dx if need_dx else None, dh0 if need_dh0 else None, None, *grads)


def fused_gru(x: Tensor, weights: Sequence[Optional[Tensor]], h0: Optional[Tensor], *, hidden: int,
              num_layers: int, batch_first: bool) -> Tuple[Tensor, Tensor]:
    return _FusedSmallGRU.apply(x, h0, (hidden, num_layers, batch_first), *weights)
