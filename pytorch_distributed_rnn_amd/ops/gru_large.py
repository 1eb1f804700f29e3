"""Large-hidden GRU stack on the MFMA step kernels (csrc/kernels/lstm_large.hip,
CELL = GRU).

New capability: the reference only builds ``nn.LSTM`` (reference:
src/motion/model.py:9), BASELINE.json names an "LSTM/GRU cell", and the
small-H GRU already runs on the fused kernels (ops/gru_fused.py).  This is the
16-bit, H % 64 == 0 counterpart for the shapes the large-H LSTM serves.

The GRU's gates ride on the LSTM step kernels' four-column quad as
``[r | z | n_x | n_h]`` (the layout of ops/gru_fused.py)::

    W_ih4 = [W_ir; W_iz; W_in; 0]      b4 = [b_ir + b_hr; b_iz + b_hz; b_in; b_hn]
    W_hh4 = [W_hr; W_hz; 0;    W_hn]

* forward: one library GEMM projects the input of all timesteps and both
  directions (``Xp = X W_ih4^T + b4``, gate-interleaved columns), then T
  launches of the MFMA step kernel whose epilogue applies
  ``r, z = sigma(.)``, ``n = tanh(n_x + r n_h)``, ``h = n + z (h_prev - n)``
  with ``h_prev`` kept in fp32;
* backward: T launches of the MFMA BPTT step (``dh_{t-1} = dgates_t W_hh4 +
  dh_t z_t``) emitting ``dgates = [dr r(1-r) | dz z(1-z) | dpre_n | dpre_n r]``
  in gate-blocked order, then ``dW_hh``, ``dW_ih``, the biases and ``dX`` as
  library GEMMs over all timesteps.

The zero blocks cost a quarter of the recurrent MFMA work; in exchange the GRU
shares every tile configuration, the split-K backward and the numerics tests
of the LSTM path.  Parameters stay in ``nn.GRU``'s layout (r, z, n).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch
from torch import Tensor

from .. import _ext
from . import shadow as _sh
from .lstm_large import (_tile, final_hidden, mark_ready, padded_cols, pipeline_backward, pipeline_chunks,
                         pipeline_forward, pipeline_join, pipeline_ok, pipeline_streams, run_recurrence, stack_layers)
from .gemm import col_sum, gemm_f32, linear16, mm_kk, mm_nk16


def supported(x: Tensor, hidden: int) -> bool:
    if x.dtype not in (torch.bfloat16, torch.float16, torch.float32) or x.device.type != "cuda" or x.dim() != 3:
        return False
    mod = _ext.native(x.device)
    return mod is not None and hasattr(mod, "lstm_large_fwd") and bool(mod.lstm_large_supported(hidden))


def _hprev(hseq_d: Tensor, h0d: Optional[Tensor], d: int) -> Tensor:
    """h_{t-1} in processing order for direction d ([T, B, H])."""
    T, B, H = hseq_d.shape
    h0d = h0d if h0d is not None else hseq_d.new_zeros(1, B, H)
    return torch.cat([h0d, hseq_d[:-1]], 0) if d == 0 else torch.cat([hseq_d[1:], h0d], 0)


def _gru_shadows(weights, ndir: int, H: int, I: int, cdt, device):
    """The packed compute-dtype copies the kernels read -- per direction W_ih
    (dX GEMM), the [r | z | n_x | 0] projection stack (gate-interleaved, both
    directions concatenated), the [r | z | 0 | n_h] recurrent stack, its
    gate-interleaved form (forward step) and its transpose (BPTT step) -- plus
    the folded projection bias.  Cached on the first weight and rebuilt only
    when a parameter's version counter or storage changes (an optimizer step),
    like the large LSTM's shadows (ops/lstm_large.py:_shadow_cat)."""
    masters = list(weights[:4 * ndir])
    box = []

    def alloc():
        # buffers allocated once: the zero blocks stay zero, a rebuild after an
        # optimizer step only converts the parameters into them
        z = dict(device=device, dtype=cdt)
        box.append(([torch.empty(3 * H, I, **z) for _ in range(ndir)], torch.zeros(ndir * 4 * H, I, **z),
                    [torch.zeros(4 * H, H, **z) for _ in range(ndir)], [torch.zeros(4 * H, H, **z) for _ in range(ndir)],
                    [torch.zeros(H, 4 * H, **z) for _ in range(ndir)],
                    torch.zeros(ndir * 4 * H, device=device, dtype=torch.float32)))
        return box[0]

    def build(*ms):
        # every job reads a master, never another output of the same launch
        wih, wih4_all, whh4, whh_p, wt, b4_all = box[0]
        jobs = []
        for d in range(ndir):
            w_ih, w_hh, b_ih, b_hh = ms[4 * d:4 * d + 4]
            wh = w_hh.view(3, H, H)
            jobs.append(_sh.job(wih[d], w_ih))
            # projection stack [r | z | n_x | 0], gate-interleaved: row 4u + q
            jobs.append(_sh.job(wih4_all[d * 4 * H:(d + 1) * 4 * H].view(H, 4, I)[:, :3],
                                w_ih.view(3, H, I).transpose(0, 1)))
            # recurrent stack [r | z | 0 | n_h] (gate-blocked), its interleaved
            # form and its transpose
            jobs.append(_sh.job(whh4[d][:2 * H], w_hh[:2 * H]))
            jobs.append(_sh.job(whh4[d][3 * H:], w_hh[2 * H:]))
            jobs.append(_sh.job(whh_p[d].view(H, 4, H)[:, :2], wh[:2].transpose(0, 1)))
            jobs.append(_sh.job(whh_p[d].view(H, 4, H)[:, 3], wh[2]))
            jobs.append(_sh.job(wt[d][:, :2 * H], w_hh[:2 * H].t()))
            jobs.append(_sh.job(wt[d][:, 3 * H:], w_hh[2 * H:].t()))
            # folded bias [b_ir + b_hr | b_iz + b_hz | b_in | b_hn], interleaved
            b = b4_all[d * 4 * H:(d + 1) * 4 * H].view(H, 4)
            bi = b_ih.view(3, H).t() if b_ih is not None else None
            bh = b_hh.view(3, H).t() if b_hh is not None else None
            if bi is not None and bh is not None:
                jobs.append(_sh.job(b[:, :2], bi[:, :2], bh[:, :2]))
            elif bi is not None or bh is not None:
                jobs.append(_sh.job(b[:, :2], (bi if bi is not None else bh)[:, :2]))
            if bi is not None:
                jobs.append(_sh.job(b[:, 2], bi[:, 2]))
            if bh is not None:
                jobs.append(_sh.job(b[:, 3], bh[:, 2]))
        return jobs

    return _sh.get(weights[0], ("gru", cdt, ndir, H, I), masters, alloc, build)


class _LargeGRULayer(torch.autograd.Function):
    """One layer, 1 or 2 directions.  x: [T, B, I] (compute dtype); weights per
    direction (w_ih, w_hh, b_ih, b_hh), fp32 masters (biases may be None)."""

    @staticmethod
    def forward(ctx, x, h0, cfg, *weights):
        ctx.set_materialize_grads(False)  # unused outputs: None, not a zero fill (lstm_large.run_recurrence)
        H, ndir, tile = cfg
        cdt = x.dtype
        T, B, I = x.shape
        mod = _ext.native(x.device)
        wih, wih4_all, whh4, whh_p, wt, b4_all = _gru_shadows(weights, ndir, H, I, cdt, x.device)
        if cdt == torch.float32:  # fp32-product MFMA GEMM (kernels/gemm_f32.hip), fp32 bias in the epilogue
            xp = gemm_f32(x.reshape(T * B, I), False, wih4_all, False, bias=b4_all)[0]
        else:  # in-tree MFMA GEMM (16-bit)
            xp = linear16(x.reshape(T * B, I), wih4_all, b4_all)
        xp = xp.view(T, B, ndir * 4 * H)
        h0c = h0.to(cdt).contiguous() if h0 is not None else None
        h0f = h0.float().contiguous() if h0 is not None else None
        rev_mask = 2 if ndir == 2 else 0
        hseq, hs32, acts = mod.lstm_large_fwd(xp, whh_p, h0c, h0f, H, rev_mask, tile, 1)
        last = [T - 1, 0][:ndir]
        hn = final_hidden(hseq, last, H)
        ctx.save_for_backward(x, hseq, hs32, acts, h0c, h0f, *wih, *wt)
        ctx.cfg = (H, ndir, tile, rev_mask, [w is not None for w in weights], h0 is not None,
                   h0.dtype if h0 is not None else None)
        return hseq, hn

    @staticmethod
    def backward(ctx, dhseq, dhn):
        H, ndir, tile, rev_mask, has_w, has_h0, h0_dtype = ctx.cfg
        x, hseq, hs32, acts, h0c, h0f, *ws = ctx.saved_tensors
        wih, wt = ws[:ndir], list(ws[ndir:])                        # wt: [H, 4H], gate-blocked
        cdt = x.dtype
        T, B, I = x.shape
        mod = _ext.native(x.device)

        def bptt():
            dout = dhseq.to(cdt).contiguous() if dhseq is not None else None
            dhn_f = dhn.float().contiguous() if dhn is not None else None
            return mod.lstm_large_bwd(dout, dhn_f, None, wt, hs32, acts, h0f, H, rev_mask, tile, 1)

        persistent = bool(getattr(mod, "lstm_large_bwd_persistent", lambda *a: True)(
            B, H, ndir, {torch.bfloat16: 0, torch.float16: 1}.get(cdt, 2), tile))
        dgates, dh0, _ = run_recurrence(dhseq, bptt, [dhseq, dhn, hs32, acts, h0f, *wt], persistent)
        grads: List[Optional[Tensor]] = []
        dx = None
        dx_pairs = []
        need_dx = ctx.needs_input_grad[0]
        x2 = x.reshape(T * B, I)
        if need_dx and cdt == torch.float32:
            # dX of both directions first (K segments): the layer below starts
            # its recurrence beside this layer's dW GEMMs (lstm_large.run_recurrence)
            Gx0 = dgates[0].view(T * B, 4 * H)[:, :3 * H]
            seg = (dgates[1].view(T * B, 4 * H)[:, :3 * H], wih[1]) if ndir > 1 else None
            dx = mark_ready(gemm_f32(Gx0, False, wih[0], True, pairs2=seg)[0].view(T, B, I))
        for d in range(ndir):
            G = dgates[d].view(T * B, 4 * H)                         # [r | z | dpre_n | dpre_n r]
            Gx = G[:, :3 * H]                                        # x side: [r | z | dpre_n]
            if cdt == torch.float32:
                # fp32-product MFMA GEMM (kernels/gemm_f32.hip) over shifted
                # views of the output sequence (no h_prev copy), the initial
                # state as a second K segment; db = the row sums of dgates^T of
                # the dW_ih pass (every row)
                # (the [r | z] and n_h gate blocks separately: nn.GRU's W_hh has
                # no n_x block, so neither product nor concatenation for it)
                hd = hseq[:, :, d * H:(d + 1) * H]
                g0 = G[:B] if d == 0 else G[(T - 1) * B:]
                Gs = G[B:] if d == 0 else G[:(T - 1) * B]
                hs = (hd[:-1] if d == 0 else hd[1:]).reshape((T - 1) * B, H)
                dwhh = torch.empty(3 * H, H, device=x.device, dtype=torch.float32)
                for cols, rows in ((slice(0, 2 * H), slice(0, 2 * H)), (slice(3 * H, 4 * H), slice(2 * H, 3 * H))):
                    seg2 = (g0[:, cols], h0c[d]) if h0c is not None else None
                    if T > 1:
                        gemm_f32(Gs[:, cols], True, hs, True, pairs2=seg2, out=dwhh[rows])
                    elif seg2 is not None:
                        gemm_f32(seg2[0], True, seg2[1], True, out=dwhh[rows])
                    else:
                        dwhh[rows].zero_()
                dwih, dbih = gemm_f32(Gx, True, x2, True, rowsum=True)
                dbhh = torch.empty(3 * H, device=x.device, dtype=torch.float32)
                dbhh[:2 * H].copy_(dbih[:2 * H])
                dbhh[2 * H:].copy_(col_sum(G[:, 3 * H:]))
            else:  # in-tree MFMA GEMM (ops/gemm.py)
                hprev = _hprev(hseq[:, :, d * H:(d + 1) * H], h0c[d:d + 1] if h0c is not None else None, d)
                dw4 = mm_kk([(G, hprev.reshape(T * B, H))])
                dwih = mm_kk([(Gx, x2)])
                cs = col_sum(G)
                dbih = cs[:3 * H]
                dwhh, dbhh = dw4.new_empty(3 * H, H), cs.new_empty(3 * H)  # nn.GRU has no n_x block in W_hh
                for dst, src in ((dwhh, dw4), (dbhh, cs)):
                    dst[:2 * H].copy_(src[:2 * H])
                    dst[2 * H:].copy_(src[3 * H:])
            if need_dx and cdt != torch.float32:
                dx_pairs.append((Gx, wih[d]))
            grads += [dwih, dwhh, dbih if has_w[4 * d + 2] else None, dbhh if has_w[4 * d + 3] else None]
        if dx_pairs:
            dx = mm_nk16(dx_pairs).view(T, B, I)  # 16-bit: both directions in one launch
        dh0_out = dh0.to(h0_dtype) if has_h0 else None
        # (the fp32 dx is returned as the very tensor mark_ready tagged: a view
        # would drop the ready event the layer below waits for)
        return (dx, dh0_out, None, *grads)


class _PipelinedGRUStack(torch.autograd.Function):
    """All layers of a unidirectional fp32 GRU stack (H = 128, row-owning
    kernels), chunk-pipelined like the LSTM's (ops/lstm_large.py, stacked-layer
    pipeline): layer l + 1 runs chunk c while layer l runs chunk c + 1.
    h0: [L, B, H] or None; weights: ``nn.GRU`` order, ``per`` per layer."""

    @staticmethod
    def forward(ctx, x, h0, cfg, *weights):
        ctx.set_materialize_grads(False)
        H, L, per, chunks = cfg
        T, B, I = x.shape
        dev = x.device
        mod = _ext.native(dev)
        lw = [list(weights[l * per:(l + 1) * per]) + ([None, None] if per == 2 else []) for l in range(L)]
        # per layer: (W_ih [3H, I_l], projection stack, W_hh4, its interleaved form, W_hh4^T, folded bias)
        sh = [_gru_shadows(lw[l], 1, H, I if l == 0 else H, torch.float32, dev) for l in range(L)]
        h0s = [h0[l].float().contiguous() if h0 is not None else None for l in range(L)]
        hseq = [x.new_empty(T, B, H) for _ in range(L)]
        hs32 = [x.new_empty(T, B, H) for _ in range(L)]
        acts = [x.new_empty(T, B, 4 * H) for _ in range(L)]
        xps = [gemm_f32(x.reshape(T * B, I), False, sh[0][1], False, bias=sh[0][5])[0].view(T, B, 4 * H)]
        xps += [x.new_empty(T, B, 4 * H) for _ in range(1, L)]
        rec = pipeline_streams(dev, L)

        def project(l, t0, t1):
            gemm_f32(hseq[l - 1][t0:t1].view(-1, H), False, sh[l][1], False, bias=sh[l][5],
                     out=xps[l][t0:t1].view(-1, 4 * H))

        def recur(l, t0, t1):  # (the GRU's fp32 hidden state rides in the c0 / cseq slot)
            mod.lstm_rows_fwd_range(xps[l][t0:t1], sh[l][3][0], h0s[l], h0s[l], hseq[l], hs32[l], acts[l], t0, t1, 1)

        pipeline_forward(rec, chunks, project, recur)
        pipeline_join(rec)
        hn = x.new_empty(L, B, H)
        for l in range(L):
            hn[l].copy_(hseq[l][T - 1])
        ctx.save_for_backward(x, *hseq, *hs32, *acts, *[t[0][0] for t in sh], *[t[4][0] for t in sh])
        ctx.states = h0s
        ctx.cfg = (H, L, per, chunks, [[w is not None for w in ws] for ws in lw], h0.dtype if h0 is not None else None)
        return hseq[L - 1], hn

    @staticmethod
    def backward(ctx, dhseq, dhn):
        H, L, per, chunks, has_w, h0_dtype = ctx.cfg
        h0s = ctx.states
        sv = ctx.saved_tensors
        x = sv[0]
        hseq, hs32, acts = sv[1:1 + L], sv[1 + L:1 + 2 * L], sv[1 + 2 * L:1 + 3 * L]
        wih, wt = sv[1 + 3 * L:1 + 4 * L], sv[1 + 4 * L:1 + 5 * L]
        T, B, I = x.shape
        dev = x.device
        mod = _ext.native(dev)
        dgates = [x.new_empty(T, B, 4 * H) for _ in range(L)]
        douts = [x.new_empty(T, B, H) for _ in range(L - 1)]
        douts.append(dhseq.float().contiguous() if dhseq is not None else None)
        dhb = [x.new_empty(B, H) for _ in range(L)]  # gradient leaving a chunk's first step
        dcb = [x.new_empty(B, H) for _ in range(L)]  # (unused by the GRU cell)
        carry = [x.new_empty(B, H) for _ in range(L)]
        dhn_l = [dhn[l].float().contiguous() if dhn is not None else None for l in range(L)]
        ins = [x] + list(hseq[:-1])
        dwih = [x.new_empty(3 * H, t.shape[2]) for t in ins]
        dwhh = [x.new_empty(3 * H, H) for _ in range(L)]
        dbih = [x.new_empty(3 * H) for _ in range(L)]
        dbhh = [x.new_empty(3 * H) for _ in range(L)]
        rec = pipeline_streams(dev, L)

        def project(l, t0, t1):  # dX of the layer above: its [r | z | dpre_n] block times W_ih
            gemm_f32(dgates[l + 1][t0:t1].view(-1, 4 * H)[:, :3 * H], False, wih[l + 1], True,
                     out=douts[l][t0:t1].view(-1, H), splitk=1)

        def recur(l, first, t0, t1):
            dout = douts[l][t0:t1] if douts[l] is not None else None
            mod.lstm_rows_bwd_range(dout, dhn_l[l] if first else dhb[l], None, wt[l], hs32[l], acts[l], h0s[l],
                                    dgates[l], dhb[l], dcb[l], carry[l], t0, t1, 1)

        def finish(l):
            _gru_weight_grads(dwih[l], dwhh[l], dbih[l], dbhh[l], dgates[l], hseq[l], h0s[l], ins[l])

        pipeline_backward(rec, chunks, project, recur, finish)
        dx = None
        if ctx.needs_input_grad[0]:  # (layer 0's stream is the caller's)
            dx = gemm_f32(dgates[0].view(T * B, 4 * H)[:, :3 * H], False, wih[0], True)[0].view(T, B, I)
        pipeline_join(rec)
        grads: List[Optional[Tensor]] = []
        for l in range(L):
            grads += [dwih[l], dwhh[l]]
            if per == 4:
                grads += [dbih[l] if has_w[l][2] else None, dbhh[l] if has_w[l][3] else None]
        dh0 = torch.stack(dhb).to(h0_dtype) if h0_dtype is not None else None
        return (dx, dh0, None, *grads)


def _gru_weight_grads(dwih: Tensor, dwhh: Tensor, dbih: Tensor, dbhh: Tensor, G3: Tensor, hd: Tensor,
                      h0: Optional[Tensor], xin: Tensor) -> None:
    """One unidirectional fp32 GRU layer's dW_ih, dW_hh, b_ih and b_hh
    gradients into the given fp32 tensors (the d = 0 case of
    _LargeGRULayer.backward): the [r | z] and n_h gate blocks of dW_hh over
    shifted views of the output sequence with h0 as a second K segment, db_ih
    as the row sums of the dW_ih pass."""
    T, B, H4 = G3.shape
    H = H4 // 4
    G = G3.view(T * B, H4)
    g0, Gs = G[:B], G[B:]
    hs = hd[:-1].reshape((T - 1) * B, H)
    for cols, rows in ((slice(0, 2 * H), slice(0, 2 * H)), (slice(3 * H, 4 * H), slice(2 * H, 3 * H))):
        seg2 = (g0[:, cols], h0) if h0 is not None else None
        if T > 1:
            gemm_f32(Gs[:, cols], True, hs, True, pairs2=seg2, out=dwhh[rows])
        elif seg2 is not None:
            gemm_f32(seg2[0], True, seg2[1], True, out=dwhh[rows])
        else:
            dwhh[rows].zero_()
    x2 = xin.reshape(T * B, -1)
    if x2.shape[1] % 32:  # narrow input: whole, aligned column tiles (lstm_large.padded_cols)
        c, rs = gemm_f32(G[:, :3 * H], True, padded_cols(x2), True, rowsum=True)
        dwih.copy_(c[:, :x2.shape[1]])
    else:
        _, rs = gemm_f32(G[:, :3 * H], True, x2, True, rowsum=True, out=dwih)
    dbih.copy_(rs)
    dbhh[:2 * H].copy_(rs[:2 * H])
    dbhh[2 * H:].copy_(col_sum(G[:, 3 * H:]))


def gru_large_forward(x: Tensor, weights: Sequence[Optional[Tensor]], h0: Optional[Tensor], *, hidden: int,
                      num_layers: int, batch_first: bool, bidirectional: bool = False, dropout: float = 0.0,
                      training: bool = False) -> Tuple[Tensor, Tensor]:
    """Stacked (bi)GRU on the MFMA step kernels; ``nn.GRU``-compatible outputs.

    ``weights``: ``nn.GRU`` ``_all_weights`` order (per layer and direction
    w_ih, w_hh[, b_ih, b_hh])."""
    ndir = 2 if bidirectional else 1
    per = len(weights) // (num_layers * ndir)
    seq = (x.transpose(0, 1) if batch_first else x).contiguous()
    if pipeline_ok(seq, hidden, num_layers, bidirectional, dropout, training):
        out, hn = _PipelinedGRUStack.apply(seq, h0, (hidden, num_layers, per, pipeline_chunks(seq.shape[0])), *weights)
        return (out.transpose(0, 1) if batch_first else out), hn
    tile = _tile()
    hns = []
    for l in range(num_layers):
        ws: List[Optional[Tensor]] = []
        for d in range(ndir):
            chunk = list(weights[(l * ndir + d) * per:(l * ndir + d + 1) * per])
            if per == 2:
                chunk += [None, None]
            ws += chunk
        h0l = h0[l * ndir:(l + 1) * ndir] if h0 is not None else None
        seq, hn = _LargeGRULayer.apply(seq, h0l, (hidden, ndir, tile), *ws)
        hns.append(hn)
        if dropout > 0 and training and l < num_layers - 1:
            seq = torch.nn.functional.dropout(seq, dropout, True)
    out = seq.transpose(0, 1) if batch_first else seq
    return out, stack_layers(hns)
