"""LSTM stack operator: fused HIP kernels on MI355X, torch reference elsewhere.

The reference framework runs ``nn.LSTM`` (ATen CPU kernels) inside
``MotionModel`` (reference: src/motion/model.py:9,14).  Here the whole stack
(all layers, all timesteps, forward and BPTT) is one HIP launch each way for
small hidden sizes (H in {16, 32, 64}, input <= H) -- see
``csrc/kernels/lstm_small.hip`` -- and a per-timestep MFMA path for large
hidden sizes (``ops/lstm_large.py``).

Gate order and parameter layout are exactly nn.LSTM's (i, f, g, o; weight_ih_l*,
weight_hh_l*, bias_ih_l*, bias_hh_l*), so checkpoints interoperate with stock
PyTorch.
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence, Tuple

import torch
from torch import Tensor

from .. import _ext
from ..utils.tune import tune_int


def small_launch_config(batch: int, hidden: int, num_layers: int = 2) -> Tuple[int, int, int, int]:
    """(nb_fwd, split_fwd, nb_bwd, split_bwd) for the fused small-H kernels.

    ``nb``: sequences per workgroup (weights in VGPRs are shared by them);
    ``split``: lanes per hidden unit (more lanes = shorter per-timestep
    critical path).  Small batches are latency-bound -> widest split, one
    sequence per workgroup.  Overrides (for sweeps, PDRNN_TUNE): nb_fwd,
    split_fwd, nb_bwd, split_bwd."""
    nb_fwd = tune_int("nb_fwd", 0)
    nb_bwd = tune_int("nb_bwd", 0)
    sp_fwd = tune_int("split_fwd", 0)
    sp_bwd = tune_int("split_bwd", 0)
    if nb_fwd not in (1, 2):
        # Large batches are LDS-bandwidth bound in the gate-split forward
        # (every lane reads the whole [x | h] operand vector): above one
        # resident round of single-sequence workgroups the 2-lane K-split map
        # (each lane reads half the vector) is faster -- B=1440: 164 us vs
        # 178 us for gate-split with 2 sequences per workgroup, 204 us with 1
        # (bench/fwd_split.py, profiles/r2_fwd_split.log); B<=1024 stays on
        # the latency-optimal gate-split map with one sequence per workgroup
        nb_fwd = 1
        if batch > 1024 and hidden == 32 and sp_fwd == 0:
            sp_fwd = 2
    if nb_bwd not in (1, 2, 3):
        nb_bwd = 1
    return nb_fwd, sp_fwd, nb_bwd, sp_bwd  # split 0 = widest valid (chosen natively)


def gru_fwd_nb(batch: int, hidden: int, device=None) -> int:
    """Sequences per workgroup of the fused GRU step's gate-split forward: one
    sequence per 4-wave workgroup holds ~150 VGPRs at H = 32, three
    workgroups per CU; above that residency round two sequences share a
    workgroup (one round instead of two, like the LSTM's K-split choice at
    B > 1024).  PDRNN_TUNE nb_fwd overrides."""
    env = tune_int("nb_fwd", 0)
    if env in (1, 2):
        return env
    if hidden != 32 or not torch.cuda.is_available():
        return 1
    dev = device if device is not None else torch.cuda.current_device()
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    return 2 if batch > 3 * cus else 1


def fused_bwd_nb(batch: int, hidden: int, num_layers: int) -> int:
    """Sequences per workgroup of the fused training step's backward.

    1 = one sequence per workgroup (the default: above one residency round
    the deferred-dW backward, lstm_small.hip DWOUT + lstm_small_dw.hip).
    2..3 interleave sequences in one workgroup of the register-dW backward
    (sweeps via PDRNN_TUNE nb_bwd); a multi-sequence variant with LDS-DMA
    staged operands was measured slower at every motion batch and removed
    (profiles/r2_tp_backward_tried.md)."""
    env = tune_int("nb_bwd", 0)
    if env in (1, 2, 3):
        return env
    return 1


def fused_small_supported(x: Tensor, hidden: int, num_layers: int, bidirectional: bool,
                          proj_size: int = 0, batch_first: bool = True) -> bool:
    if bidirectional or proj_size:
        return False
    if x.dtype not in (torch.float32, torch.bfloat16) or x.dim() != 3:
        return False
    if x.dtype == torch.bfloat16:
        if x.shape[1 if batch_first else 0] * hidden * 4 > 48 * 1024:
            return False  # bf16 x is widened while staging into LDS: sequence must fit there
        if hidden >= 128:
            return False  # the MFMA large-H path serves 16-bit models from H = 128 up
    mod = _ext.native(x.device)
    if mod is None:
        return False
    return bool(mod.lstm_small_supported(hidden, x.shape[-1], num_layers))


class _FusedSmallLSTM(torch.autograd.Function):
    """Autograd node for the fused small-H LSTM stack.

    forward inputs: x, idx, h0, c0, config tuple, *weights (4 per layer)."""

    @staticmethod
    def forward(ctx, x, idx, h0, c0, cfg, *weights):
        hidden, num_layers, batch_first, need_out = cfg
        mod = _ext.native(x.device)
        if x.dtype == torch.bfloat16:
            # bf16 model: recurrent weights rounded to bf16 (fp32 masters keep
            # the update; gradients pass straight through), fp32 accumulation
            weights = tuple(w.to(torch.bfloat16).float() for w in weights)
        batch = idx.numel() if idx is not None else (x.shape[0] if batch_first else x.shape[1])
        nb_fwd, sp_fwd, nb_bwd, sp_bwd = small_launch_config(batch, hidden, num_layers)
        h0c = h0.float().contiguous() if h0 is not None else None
        c0c = c0.float().contiguous() if c0 is not None else None
        ctx.state_dtypes = (h0.dtype if h0 is not None else None, c0.dtype if c0 is not None else None)
        out, hn, cn, act = mod.lstm_small_fwd(
            x, idx, list(weights), h0c, c0c, hidden, num_layers, batch_first, True, need_out, nb_fwd,
            sp_fwd)
        ctx.set_materialize_grads(False)
        ctx.cfg = (hidden, num_layers, batch_first, nb_bwd, sp_bwd)
        ctx.save_for_backward(x, idx, h0c, c0c, out, act, *weights)
        top = out[num_layers - 1]  # [B, T, H]
        if not batch_first:
            top = top.transpose(0, 1)
        return top, hn, cn

    @staticmethod
    def backward(ctx, dout, dhn, dcn):
        x, idx, h0, c0, hseq, act, *weights = ctx.saved_tensors
        hidden, num_layers, batch_first, nb_bwd, sp_bwd = ctx.cfg
        mod = _ext.native(x.device)
        need_dx = ctx.needs_input_grad[0]
        need_dh0 = ctx.needs_input_grad[2] or ctx.needs_input_grad[3]
        if dout is not None and dout.stride(-1) != 1:
            dout = dout.contiguous()
        dhn = dhn.contiguous() if dhn is not None else None
        dcn = dcn.contiguous() if dcn is not None else None
        dparams, dx, dh0, dc0 = mod.lstm_small_bwd(
            x, idx, list(weights), h0, c0, hseq, act, dout, dhn, dcn, hidden, num_layers,
            batch_first, need_dx, need_dh0, nb_bwd, sp_bwd, None)
        grads = []
        off = 0
        for w in weights:
            n = w.numel()
            grads.append(dparams[off:off + n].view_as(w))
            off += n
        hdt, cdt = ctx.state_dtypes
        if dx is not None and dx.dtype != x.dtype:
            dx = dx.to(x.dtype)
        return (dx if need_dx else None, None,
                dh0.to(hdt) if ctx.needs_input_grad[2] else None,
                dc0.to(cdt) if ctx.needs_input_grad[3] else None, None, *grads)


def _flat_weights(weights: Sequence[Optional[Tensor]], num_layers: int, hidden: int,
                  like: Tensor) -> List[Tensor]:
    out = []
    for l in range(num_layers):
        w_ih, w_hh, b_ih, b_hh = weights[4 * l:4 * l + 4]
        if b_ih is None:
            b_ih = like.new_zeros(4 * hidden)
        if b_hh is None:
            b_hh = like.new_zeros(4 * hidden)
        out += [w_ih.contiguous(), w_hh.contiguous(), b_ih.contiguous(), b_hh.contiguous()]
    return out


def lstm_reference(x: Tensor, weights: Sequence[Optional[Tensor]], h0: Optional[Tensor],
                   c0: Optional[Tensor], hidden: int, num_layers: int, batch_first: bool,
                   dropout: float = 0.0, training: bool = False,
                   bidirectional: bool = False) -> Tuple[Tensor, Tensor, Tensor]:
    """Stock ATen LSTM (CPU / MIOpen) -- the torch reference path for tests."""
    dirs = 2 if bidirectional else 1
    has_bias = weights[2] is not None
    # mixed precision (16-bit activations, fp32 master weights): compute in the
    # activation dtype, like torch.autocast does for nn.LSTM
    flat = [w if w.dtype == x.dtype else w.to(x.dtype) for w in weights if w is not None]
    if h0 is not None and h0.dtype != x.dtype:
        h0, c0 = h0.to(x.dtype), c0.to(x.dtype)
    if h0 is None:
        b = x.shape[0] if batch_first else x.shape[1]
        h0 = x.new_zeros(num_layers * dirs, b, hidden)
        c0 = x.new_zeros(num_layers * dirs, b, hidden)
    out, hn, cn = torch._VF.lstm(x, (h0, c0), flat, has_bias, num_layers, dropout, training,
                                 bidirectional, batch_first)
    return out, hn, cn


_SMALL_H = (16, 32, 64)


def small_plan(x: Tensor, hidden: int, num_layers: int, *, cell: str = "lstm", per_layer: bool = False,
               batch_first: bool = True) -> Optional[Tuple[int, List[Tuple[int, int]]]]:
    """How the fused small-H kernels cover an arbitrary unidirectional stack:
    ``(H_pad, [(first_layer, n_layers), ...])`` or None.

    * hidden sizes the kernels are not instantiated for (8, 24, 48, ...) run
      zero-padded to the next of 16/32/64: padded units have zero weights and
      bias, so i=f=o=1/2, g=0 -> c and h stay exactly 0 and never touch a real
      unit (their W columns are zero); padded gradients are dropped;
    * stacks deeper than one launch holds (4 layers, 512 lanes) run as chunks
      of layers, each chunk's top output feeding the next (``per_layer``: one
      layer per launch, e.g. nn.LSTM dropout between layers)."""
    if x.dim() != 3 or x.dtype not in (torch.float32, torch.bfloat16):
        return None
    mod = _ext.native(x.device)
    if mod is None:
        return None
    I = x.shape[-1]
    T = x.shape[1 if batch_first else 0]
    for hp in _SMALL_H:
        if hp < hidden or hp < I:
            continue
        if x.dtype == torch.bfloat16 and T * hp * 4 > 48 * 1024:
            continue  # bf16 x is widened while staging into LDS: the sequence must fit there
        chunks, l = [], 0
        while l < num_layers:
            n = 1 if per_layer else min(4, num_layers - l)
            while n > 0 and not _chunk_ok(mod, cell, hp, I if l == 0 else hp, n):
                n -= 1
            if n == 0:
                break
            chunks.append((l, n))
            l += n
        if l == num_layers:
            return hp, chunks
    return None


def _chunk_ok(mod, cell: str, hp: int, in_dim: int, n: int) -> bool:
    if not mod.lstm_small_supported(hp, in_dim, n):
        return False
    if cell == "gru":  # GRU: gate-split forward and unit-group backward maps only
        return n * 4 * hp <= 512 and n * hp * (8 if hp >= 64 else 4) <= 512
    return True


def pad_gate_rows(w: Optional[Tensor], hidden: int, hp: int, gates: int, in_pad: Optional[int] = None):
    """[gates*H, I] -> [gates*hp, in_pad] (or [gates*H] -> [gates*hp]) with zero
    rows/columns; differentiable (the gradient of the real block flows back)."""
    if w is None:
        return None
    if w.dim() == 1:
        return torch.nn.functional.pad(w.view(gates, hidden), (0, hp - hidden)).reshape(gates * hp)
    i = w.shape[1]
    ip = i if in_pad is None else in_pad
    return torch.nn.functional.pad(w.view(gates, hidden, i), (0, ip - i, 0, hp - hidden)).reshape(gates * hp, ip)


def _pad_state(s: Optional[Tensor], hidden: int, hp: int) -> Optional[Tensor]:
    if s is None or hp == hidden:
        return s
    return torch.nn.functional.pad(s, (0, hp - hidden))


def _run_small_chunk(x, idx, h0, c0, ws, hidden, n, batch_first, need_out):
    flat = _flat_weights(ws, n, hidden, x)
    needs_grad = torch.is_grad_enabled() and (
        x.requires_grad or any(w.requires_grad for w in flat)
        or (h0 is not None and h0.requires_grad) or (c0 is not None and c0.requires_grad))
    if needs_grad:
        return _FusedSmallLSTM.apply(x, idx, h0, c0, (hidden, n, batch_first, need_out), *flat)
    mod = _ext.native(x.device)
    nb_fwd, sp_fwd, _, _ = small_launch_config(
        idx.numel() if idx is not None else (x.shape[0] if batch_first else x.shape[1]), hidden, n)
    out, hn, cn, _ = mod.lstm_small_fwd(
        x, idx, flat, h0.contiguous() if h0 is not None else None,
        c0.contiguous() if c0 is not None else None, hidden, n, batch_first, False, need_out, nb_fwd, sp_fwd)
    return out, hn, cn


def lstm_forward(x: Tensor, weights: Sequence[Optional[Tensor]], h0: Optional[Tensor] = None,
                 c0: Optional[Tensor] = None, *, hidden: int, num_layers: int,
                 batch_first: bool = False, need_out: bool = True, idx: Optional[Tensor] = None,
                 dropout: float = 0.0, training: bool = False,
                 bidirectional: bool = False) -> Tuple[Optional[Tensor], Tensor, Tensor]:
    """LSTM stack forward.  Returns (out, h_n, c_n) like nn.LSTM.

    ``idx`` (optional) gathers batch rows from ``x`` (a device-resident dataset)
    inside the kernel; ``need_out=False`` lets inference skip the per-timestep
    output stream when only h_n is consumed."""
    drop = dropout if training else 0.0
    plan = None if bidirectional else small_plan(x, hidden, num_layers, per_layer=drop > 0,
                                                 batch_first=batch_first)
    if plan is not None:
        hp, chunks = plan
        if hp == hidden and len(chunks) == 1:
            return _run_small_chunk(x, idx, h0, c0, list(weights), hidden, num_layers, batch_first, need_out)
        h, hns, cns = x, [], []
        for k, (l0, n) in enumerate(chunks):
            ws = list(weights[4 * l0:4 * (l0 + n)])
            if hp != hidden:
                for j in range(n):
                    in_pad = None if l0 + j == 0 else hp
                    ws[4 * j:4 * j + 4] = [pad_gate_rows(ws[4 * j], hidden, hp, 4, in_pad),
                                           pad_gate_rows(ws[4 * j + 1], hidden, hp, 4, hp),
                                           pad_gate_rows(ws[4 * j + 2], hidden, hp, 4),
                                           pad_gate_rows(ws[4 * j + 3], hidden, hp, 4)]
            last = k == len(chunks) - 1
            out, hn, cn = _run_small_chunk(
                h, idx if l0 == 0 else None,
                _pad_state(h0[l0:l0 + n], hidden, hp) if h0 is not None else None,
                _pad_state(c0[l0:l0 + n], hidden, hp) if c0 is not None else None,
                ws, hp, n, batch_first, need_out or not last)
            hns.append(hn)
            cns.append(cn)
            if not last and drop > 0:
                out = torch.nn.functional.dropout(out, drop, True)
            h = out
        hn, cn = torch.cat(hns), torch.cat(cns)
        if hp != hidden:
            hn, cn = hn[..., :hidden], cn[..., :hidden]
            h = h[..., :hidden] if h is not None else None
        return h, hn, cn
    from . import lstm_large
    if lstm_large.supported(x, hidden, num_layers):
        if idx is not None:
            if batch_first:  # gather the batch straight into the time-major layout: one launch
                x = x.transpose(0, 1).index_select(1, idx)
                batch_first = False
                out, hn, cn = lstm_large.lstm_large_forward(x, weights, h0, c0, hidden=hidden,
                                                            num_layers=num_layers, batch_first=False,
                                                            bidirectional=bidirectional, dropout=dropout,
                                                            training=training)
                return (out.transpose(0, 1) if out is not None else None), hn, cn
            x = x.index_select(1, idx)
        return lstm_large.lstm_large_forward(x, weights, h0, c0, hidden=hidden,
                                             num_layers=num_layers, batch_first=batch_first,
                                             bidirectional=bidirectional, dropout=dropout,
                                             training=training)
    hp = -(-hidden // 64) * 64  # large-H kernels: H % 64 == 0 -> zero-pad the hidden size
    if not bidirectional and hidden > 64 and lstm_large.supported(x, hp, num_layers):
        if idx is not None:
            x = x.index_select(0 if batch_first else 1, idx)
        per = len(weights) // num_layers
        ws: List[Optional[Tensor]] = []
        for l in range(num_layers):
            w = list(weights[l * per:(l + 1) * per]) + ([None, None] if per == 2 else [])
            in_pad = None if l == 0 else hp
            ws += [pad_gate_rows(w[0], hidden, hp, 4, in_pad), pad_gate_rows(w[1], hidden, hp, 4, hp),
                   pad_gate_rows(w[2], hidden, hp, 4), pad_gate_rows(w[3], hidden, hp, 4)]
        out, hn, cn = lstm_large.lstm_large_forward(
            x, ws, _pad_state(h0, hidden, hp), _pad_state(c0, hidden, hp), hidden=hp,
            num_layers=num_layers, batch_first=batch_first, dropout=dropout, training=training)
        return out[..., :hidden], hn[..., :hidden], cn[..., :hidden]
    _ext.fallback(f"LSTM(H={hidden}, I={x.shape[-1]}, layers={num_layers}, {x.dtype}, "
                  f"bidirectional={bidirectional})", x.device)
    if idx is not None:
        x = x.index_select(0, idx)
    return lstm_reference(x, weights, h0, c0, hidden, num_layers, batch_first, dropout, training,
                          bidirectional)


def _bidir_small_hp(x: Tensor, hidden: int, num_layers: int, batch_first: bool) -> Optional[int]:
    """Padded hidden size for a bidirectional stack on the small-H kernels
    (layer >= 1 consumes [fwd | bwd] = 2H features, which must fit the
    kernel's input width <= H_pad), or None."""
    if x.dim() != 3 or x.dtype not in (torch.float32, torch.bfloat16):
        return None
    mod = _ext.native(x.device)
    if mod is None:
        return None
    I, T = x.shape[-1], x.shape[1 if batch_first else 0]
    for hp in _SMALL_H:
        if hp < hidden or hp < I or (num_layers > 1 and hp < 2 * hidden):
            continue
        if x.dtype == torch.bfloat16 and T * hp * 4 > 48 * 1024:
            continue
        if all(_chunk_ok(mod, "lstm", hp, I if l == 0 else hp, 1) for l in range(num_layers)):
            return hp
    return None


def _bidir_small(x, ws, h0, c0, hidden, hp, num_layers, batch_first, drop):
    """Stacked bidirectional LSTM on the fused kernels: per layer, the forward
    direction runs on x and the reverse direction on time-reversed x (one
    single-layer launch each), outputs concatenated [fwd | bwd] like nn.LSTM."""
    tdim = 1 if batch_first else 0
    h, hns, cns = x, [], []
    for l in range(num_layers):
        outs = []
        for d in range(2):
            k = 2 * l + d
            w = ws[4 * k:4 * k + 4]
            in_pad = None if l == 0 else hp
            w = [pad_gate_rows(w[0], hidden, hp, 4, in_pad if in_pad != w[0].shape[1] else None),
                 pad_gate_rows(w[1], hidden, hp, 4, hp),
                 pad_gate_rows(w[2], hidden, hp, 4), pad_gate_rows(w[3], hidden, hp, 4)]
            inp = h if d == 0 else h.flip(tdim)
            hh = _pad_state(h0[k:k + 1], hidden, hp) if h0 is not None else None
            cc = _pad_state(c0[k:k + 1], hidden, hp) if c0 is not None else None
            out, hn, cn = _run_small_chunk(inp, None, hh, cc, w, hp, 1, batch_first, True)
            out = out[..., :hidden]
            outs.append(out if d == 0 else out.flip(tdim))
            hns.append(hn[..., :hidden])
            cns.append(cn[..., :hidden])
        h = torch.cat(outs, dim=-1)
        if l < num_layers - 1:
            if h.shape[-1] < hp:  # next layer's input width: zero columns up to H_pad
                h = torch.nn.functional.pad(h, (0, hp - h.shape[-1]))
            if drop > 0:
                h = torch.nn.functional.dropout(h, drop, True)
    return h, torch.cat(hns), torch.cat(cns)


def lstm_bidirectional_forward(x: Tensor, all_weights: Sequence[Tensor], h0: Optional[Tensor],
                               c0: Optional[Tensor], *, hidden: int, num_layers: int,
                               batch_first: bool, dropout: float = 0.0,
                               training: bool = False) -> Tuple[Tensor, Tensor, Tensor]:
    """Stacked bidirectional LSTM (nn.LSTM(bidirectional=True) parameter order:
    per layer [fwd: w_ih, w_hh, b_ih, b_hh, bwd: w_ih, w_hh, b_ih, b_hh])."""
    from . import lstm_large
    if lstm_large.supported(x, hidden, num_layers, bidirectional=True):
        return lstm_large.lstm_large_forward(x, all_weights, h0, c0, hidden=hidden,
                                             num_layers=num_layers, batch_first=batch_first,
                                             bidirectional=True, dropout=dropout, training=training)
    has_bias = len(all_weights) == 8 * num_layers
    ws: List[Optional[Tensor]] = []
    per = 4 if has_bias else 2
    for l in range(num_layers * 2):
        chunk = list(all_weights[l * per:(l + 1) * per])
        if not has_bias:
            chunk += [None, None]
        ws += chunk
    hp = _bidir_small_hp(x, hidden, num_layers, batch_first)
    if hp is not None:
        return _bidir_small(x, ws, h0, c0, hidden, hp, num_layers, batch_first, dropout if training else 0.0)
    _ext.fallback(f"bidirectional LSTM(H={hidden}, I={x.shape[-1]}, layers={num_layers}, {x.dtype})", x.device)
    return lstm_reference(x, ws, h0, c0, hidden, num_layers, batch_first, dropout, training,
                          bidirectional=True)
