"""Large-hidden LSTM stack on the MFMA step kernels (csrc/kernels/lstm_large.hip).

Used when ``H % 64 == 0`` (other H >= 64 are zero-padded up by ops/lstm.py):
16-bit inputs (bf16 / fp16 compute on v_mfma_f32_16x16x32, fp32 master
weights, fp32 cell state and weight gradients) -- the char-LM (H = 1024) and
stacked bidirectional (H = 4096) configurations -- and fp32 inputs (exact fp32
products on v_mfma_f32_16x16x4_f32, e.g. the motion CLI with
``--hidden-units 128``).  Per layer:

* input projection for ALL timesteps and both directions in one library GEMM
  (``Xp = X [W_ih_fwd; W_ih_rev]^T + b``, gate-interleaved columns);
* T launches of the fused recurrent step (MFMA GEMM ``h_{t-1} W_hh^T`` + LSTM
  cell epilogue), both directions per launch;
* backward: one fused first-cell kernel + T launches of the fused BPTT step
  (MFMA ``dgates_t W_hh`` + cell backward of the previous step), then
  ``dW_hh``, ``dW_ih``, ``db`` and ``dX`` as library GEMMs over all
  timesteps with fp32 outputs.

Semantics are torch.nn.LSTM's (gate order i, f, g, o; reference:
src/motion/model.py:9 builds its model on nn.LSTM); parameters stay in the
stock nn.LSTM layout -- the gate interleave is a per-call permutation.
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence, Tuple

import torch
from torch import Tensor

from .. import _ext
from ..utils.tune import tune, tune_int
from . import gradsink
from . import shadow as _sh
from .gemm import col_sum, gemm_f32, linear16, mm_kk, mm_nk16


def _tile() -> int:
    """Forced step-kernel tile (PDRNN_TUNE large_tile; -1: the heuristic)."""
    return tune_int("large_tile", -1)


def supported(x: Tensor, hidden: int, num_layers: int, bidirectional: bool = False) -> bool:
    if x.dtype not in (torch.bfloat16, torch.float16, torch.float32) or x.device.type != "cuda" or x.dim() != 3:
        return False
    mod = _ext.native(x.device)
    return mod is not None and hasattr(mod, "lstm_large_fwd") and bool(mod.lstm_large_supported(hidden))


def _mm_f32(a: Tensor, b: Tensor) -> Tensor:
    """a @ b with fp32 output from 16-bit inputs (hipBLASLt fp32 accumulate)."""
    try:
        return torch.mm(a, b, out_dtype=torch.float32)
    except (RuntimeError, TypeError):
        return torch.mm(a.float(), b.float())


def _mm_tn_f32(g: Tensor, x: Tensor, steps: int) -> Tensor:
    """g^T x with fp32 output for g [K, M], x [K, N], K = steps * rows.

    Weight-gradient GEMMs of small layers have a tiny output and a huge K
    (fp32 motion model, H = 128, B = 1440, T = 128: 512 x 128 outputs, K =
    184k), so a single library GEMM has too few output tiles to fill the GPU
    (measured 632 us at 38 TF/s, `profiles/r2_fp32_large_h128.md`).  Those are
    split along K at step boundaries into one strided-batched GEMM plus a sum."""
    K, M = g.shape
    N = x.shape[1]
    c = 1
    if M * N <= (1 << 20) and K >= (1 << 14) and steps > 1:
        for d in range(min(steps, 128), 1, -1):
            if steps % d == 0 and K // d >= 1024:
                c = d
                break
    if c == 1:
        return _mm_f32(g.t(), x)
    gb = g.reshape(c, K // c, M).transpose(1, 2)
    xb = x.reshape(c, K // c, N)
    if g.dtype == torch.float32:
        return torch.bmm(gb, xb).sum(0)
    try:
        return torch.bmm(gb, xb, out_dtype=torch.float32).sum(0)
    except (RuntimeError, TypeError):
        return _mm_f32(g.t(), x)


def _addmm_f32_(c: Tensor, a: Tensor, b: Tensor) -> Tensor:
    """c += a @ b, fp32 c, 16-bit a / b."""
    try:
        return c.copy_(torch.addmm(c, a, b, out_dtype=torch.float32))
    except (RuntimeError, TypeError):
        return c.add_(torch.mm(a.float(), b.float()))


def shadow(w: Tensor, kind: str, cdt: torch.dtype, hidden: int) -> Tensor:
    """Compute-dtype copy of an fp32 master weight in the layout a kernel reads.

    The copy is 16-bit, or fp32 on the fp32 path. It is cached on the parameter
    and rebuilt only when the master changed: the version counter moves on every
    in-place update, and FusedAdam's native step bumps it explicitly. After an
    optimizer step, the first stale lookup rebuilds every stale shadow of the
    device in one pack launch (ops/shadow.py, kernels/shadow_pack.hip).

    kind: "i" gate-interleaved rows (forward step GEMM / input projection),
          "p" stored layout (dX GEMM), "t" transposed [I, 4H] (BPTT step GEMM)."""
    if kind == "p" and w.dtype == cdt:
        return w.detach()  # the master itself
    if kind not in ("i", "p", "t"):
        raise ValueError(kind)
    rows, cols = w.shape
    box = []  # the output buffer, for the builder (which must not hold the master)

    def alloc():
        box.append(torch.empty((cols, rows) if kind == "t" else (rows, cols), device=w.device, dtype=cdt))
        return box[0]

    def build(src):
        t = box[0]
        if kind == "i":
            return [_interleave_job(t, src, hidden)]
        if kind == "p":
            return [_sh.job(t, src)]
        return [_sh.job(t, src.t())]

    return _sh.get(w, (kind, cdt), [w], alloc, build)


def _interleave_job(dst: Tensor, src: Tensor, hidden: int):
    """dst[4u + q] = src[q*H + u]: gate-blocked -> gate-interleaved rows."""
    k = src.shape[1]
    return _sh.job(dst.view(hidden, 4, k), src.view(4, hidden, k).transpose(0, 1))


def _shadow_cat(ws: List[Tensor], cdt: torch.dtype, hidden: int) -> Tensor:
    """Both directions' interleaved input weights stacked [ndir*4H, I] (one
    input-projection GEMM for both), cached on the first weight."""
    if len(ws) == 1:
        return shadow(ws[0], "i", cdt, hidden)
    n4 = 4 * hidden
    key = ("icat", cdt, tuple(id(w) for w in ws))
    box = []

    def alloc():
        box.append(torch.empty(len(ws) * n4, ws[0].shape[1], device=ws[0].device, dtype=cdt))
        return box[0]

    def build(*srcs):
        t = box[0]
        return [_interleave_job(t[d * n4:(d + 1) * n4], src, hidden) for d, src in enumerate(srcs)]

    return _sh.get(ws[0], key, list(ws), alloc, build)


def _bias_cat(weights, ndir: int, hidden: int, device) -> Tensor:
    """b_ih + b_hh of every direction, gate-interleaved and concatenated (the
    projection GEMM's fp32 epilogue bias), cached like the shadow weights and
    rebuilt only after the biases change."""
    bs = [weights[4 * d + k] for d in range(ndir) for k in (2, 3)]
    n4 = 4 * hidden
    box = []

    def alloc():
        box.append(torch.zeros(ndir * n4, device=device, dtype=torch.float32))
        return box[0]

    def build(*srcs):
        t = box[0]
        jobs = []
        for d in range(ndir):
            b = t[d * n4:(d + 1) * n4].view(hidden, 4)  # interleaved: [u][q] = row q*H + u
            pair = [src.view(4, hidden).t() for src in srcs[2 * d:2 * d + 2] if src is not None]
            if len(pair) == 2:
                jobs.append(_sh.job(b, pair[0], pair[1]))
            elif pair:
                jobs.append(_sh.job(b, pair[0]))
            # no bias at all: the buffer stays zero
        return jobs

    return _sh.get(weights[0], ("bias", ndir, hidden), bs, alloc, build)


# ---------------------------------------------------------------------------
# Cross-layer overlap in the fp32 backward: layer l's recurrence (90 of 256
# CUs at the motion batch) needs only the layer above's dX, not its weight
# gradients.  The layer above records an event right after its dX GEMM and
# hangs it on the dX tensor; this layer's recurrence then runs on a
# high-priority side stream that waits for that event only, while the main
# stream is still busy with the layer above's dW GEMMs.  The main stream
# joins the side stream before this layer's own GEMMs (and every gradient is
# still returned through autograd on the main stream: DDP hooks unchanged).
_SIDE = {}


def _side_stream(device) -> "torch.cuda.Stream":
    s = _SIDE.get(device)
    if s is None:
        s = _SIDE[device] = torch.cuda.Stream(device=device, priority=-1)
    return s


def overlap_on() -> bool:
    return tune("large_overlap", "1") != "0"


def run_recurrence(dhseq: Optional[Tensor], fn, inputs: Sequence[Optional[Tensor]], persistent: bool = False):
    """fn() -> tensors: the layer's backward recurrence, on the side stream
    when the upstream gradient carries a ready event (see above), inline
    otherwise.  ``inputs``: the tensors fn reads, as autograd delivered them;
    fn converts them itself, so any conversion kernel runs on the side stream
    after the event.  The event covers the main stream up to the dX GEMM
    only, so the layer's Function must not let autograd materialise zero
    gradients (``ctx.set_materialize_grads(False)``): such a zero fill is
    queued on the main stream after the event, and the side stream read it
    before it ran (uninitialised dc carry: wrong gradients one run in a few,
    tools/pipe_determinism.py).  ``persistent``: the recurrence is one
    grid-synced persistent launch, whose co-residency is checked against an
    idle device only -- it runs inline, never beside the side-stream GEMMs."""
    if persistent:
        return fn()
    ev = getattr(dhseq, "_pdrnn_ready", None) if dhseq is not None else None
    if ev is not None and getattr(dhseq, "_pdrnn_ready_version", None) != dhseq._version:
        ev = None  # written after the event (e.g. an in-place gradient accumulation)
    if ev is None or not overlap_on():
        return fn()
    main = torch.cuda.current_stream(dhseq.device)
    side = _side_stream(dhseq.device)
    side.wait_event(ev)
    with torch.cuda.stream(side):
        out = fn()
    for t in inputs:  # main-stream tensors read on the side stream
        if t is not None:
            t.record_stream(side)
    for t in out:  # side-stream tensors read on the main stream
        if t is not None:
            t.record_stream(main)
    main.wait_stream(side)
    return out


def mark_ready(dx: Optional[Tensor]) -> Optional[Tensor]:
    """Record the event the layer below waits for (after this layer's dX)."""
    if dx is not None and dx.is_cuda and overlap_on():
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(dx.device))
        dx._pdrnn_ready = ev
        dx._pdrnn_ready_version = dx._version
    return dx


def final_hidden(hseq: Tensor, last: Sequence[int], H: int) -> Tensor:
    """[ndir, B, H] final hidden states out of hseq [T, B, ndir*H]: one copy
    per direction into a fresh tensor (no ATen concatenation kernel)."""
    hn = hseq.new_empty(len(last), hseq.shape[1], H)
    for d, t in enumerate(last):
        hn[d].copy_(hseq[t, :, d * H:(d + 1) * H])
    return hn


class _StackStates(torch.autograd.Function):
    """Per-layer final h and c ([ndir, B, H] each) stacked into nn.LSTM's
    [layers*ndir, B, H] pair by one pack launch (ops/shadow.py) instead of a
    slice copy per layer and state; the backward hands each layer its slices."""

    @staticmethod
    def forward(ctx, L, *states):
        ctx.set_materialize_grads(False)
        outs, jobs, ns = [], [], []
        for group in (states[:L], states[L:]):
            n = group[0].shape[0]
            out = group[0].new_empty(n * L, *group[0].shape[1:])
            jobs += [_sh.job(out[l * n:(l + 1) * n], s) for l, s in enumerate(group)]
            outs.append(out)
            ns.append(n)
        _sh.pack(jobs, states[0].device)
        ctx.L, ctx.ns = L, ns
        return tuple(outs)

    @staticmethod
    def backward(ctx, dh, dc):
        L = ctx.L
        grads = []
        for g, n in zip((dh, dc), ctx.ns):
            grads += [g[l * n:(l + 1) * n] if g is not None else None for l in range(L)]
        return (None, *grads)


def stack_layers(states: List[Tensor]) -> Tensor:
    """Per-layer [ndir, B, H] states -> [layers*ndir, B, H] (slice copies,
    autograd-tracked; a single layer is returned as is)."""
    if len(states) == 1:
        return states[0]
    n = states[0].shape[0]
    out = states[0].new_empty(n * len(states), *states[0].shape[1:])
    for l, s in enumerate(states):
        out[l * n:(l + 1) * n] = s
    return out


class _LargeLSTMLayer(torch.autograd.Function):
    """One layer, 1 or 2 directions.  x: [T, B, I] (compute dtype).

    weights: per direction (w_ih, w_hh, b_ih, b_hh), fp32 master parameters
    (biases may be None)."""

    @staticmethod
    def forward(ctx, x, h0, c0, cfg, *weights):
        ctx.set_materialize_grads(False)  # unused outputs: None, not a zero fill (run_recurrence)
        hidden, ndir, tile = cfg
        cdt = x.dtype
        T, B, I = x.shape
        H = hidden
        mod = _ext.native(x.device)
        w_ih = [weights[4 * d] for d in range(ndir)]
        w_hh = [weights[4 * d + 1] for d in range(ndir)]
        wih_p = _shadow_cat(w_ih, cdt, H)                                  # [ndir*4H, I]
        bias_all = _bias_cat(weights, ndir, H, x.device)                   # fp32 [ndir*4H], interleaved
        if cdt == torch.float32:  # fp32-product MFMA GEMM (kernels/gemm_f32.hip), fp32 bias in the epilogue
            xp = gemm_f32(x.reshape(T * B, I), False, wih_p, False, bias=bias_all)[0]
            xp = xp.view(T, B, ndir * 4 * H)
        else:  # in-tree MFMA GEMM, fp32 bias added before the 16-bit rounding (ops/gemm.py)
            xp = linear16(x.reshape(T * B, I), wih_p, bias_all).view(T, B, ndir * 4 * H)
        whh_p = [shadow(w, "i", cdt, H) for w in w_hh]
        h0c = h0.to(cdt).contiguous() if h0 is not None else None
        c0c = c0.float().contiguous() if c0 is not None else None
        rev_mask = 2 if ndir == 2 else 0
        hseq, cseq, acts = mod.lstm_large_fwd(xp, whh_p, h0c, c0c, H, rev_mask, tile, 0)
        last = [T - 1, 0][:ndir]
        # final h (out of hseq) and c (fp32 cseq -> compute dtype) of every
        # direction: one pack launch instead of a copy each
        hn = hseq.new_empty(ndir, B, H)
        cn = cseq.new_empty(ndir, B, H, dtype=cdt)
        _sh.pack([_sh.job(hn[d], hseq[last[d], :, d * H:(d + 1) * H]) for d in range(ndir)] +
                 [_sh.job(cn[d], cseq[d, last[d]]) for d in range(ndir)], x.device)
        # backward works in torch's gate-blocked order: W_ih as stored (dX GEMM),
        # W_hh transposed (BPTT step GEMM), both 16-bit shadows
        ctx.save_for_backward(x, hseq, cseq, acts, h0c, c0c, *[shadow(w, "p", cdt, H) for w in w_ih],
                              *[shadow(w, "t", cdt, H) for w in w_hh])
        ctx.cfg = (H, ndir, tile, rev_mask, [w is not None for w in weights], h0 is not None,
                   c0 is not None, h0.dtype if h0 is not None else None,
                   c0.dtype if c0 is not None else None)
        ctx.params = weights  # (gradsink: the 16-bit backward may accumulate into their .grad)
        ctx.direct = gradsink.enabled()
        return hseq, hn, cn

    @staticmethod
    def backward(ctx, dhseq, dhn, dcn):
        H, ndir, tile, rev_mask, has_w, has_h0, has_c0, h0_dtype, c0_dtype = ctx.cfg
        x, hseq, cseq, acts, h0c, c0c, *ws = ctx.saved_tensors
        wih, whh = ws[:ndir], ws[ndir:]
        cdt = x.dtype
        T, B, I = x.shape
        mod = _ext.native(x.device)
        wt = list(whh)                                              # [H, 4H], gate-blocked

        def bptt():
            dout = dhseq.to(cdt).contiguous() if dhseq is not None else None
            dhn_f = dhn.float().contiguous() if dhn is not None else None
            dcn_f = dcn.float().contiguous() if dcn is not None else None
            return mod.lstm_large_bwd(dout, dhn_f, dcn_f, wt, cseq, acts, c0c, H, rev_mask, tile, 0)

        persistent = bool(getattr(mod, "lstm_large_bwd_persistent", lambda *a: True)(
            B, H, ndir, {torch.bfloat16: 0, torch.float16: 1}.get(cdt, 2), tile))
        dgates, dh0, dc0 = run_recurrence(dhseq, bptt, [dhseq, dhn, dcn, cseq, acts, c0c, *wt], persistent)
        grads: List[Optional[Tensor]] = []
        dx = None
        need_dx = ctx.needs_input_grad[0]
        x2 = x.reshape(T * B, I)
        if cdt != torch.float32:
            return _backward_gemms16(ctx, dgates, dh0, dc0, hseq, h0c, x2, wih)
        # fp32 layers: every product on the fp32-product MFMA GEMM
        # (kernels/gemm_f32.hip): dW_hh over shifted views of the output
        # sequence with the initial-state pairing as a second K segment, dW_ih
        # with db as the row sums of dgates^T in the same pass, dX of both
        # directions in one launch (K segments) -- first, so the layer below
        # can start its recurrence beside this layer's dW (run_recurrence)
        if need_dx:
            Gd = [dgates[d].view(T * B, 4 * H) for d in range(ndir)]
            dx = gemm_f32(Gd[0], False, wih[0], True, pairs2=(Gd[1], wih[1]) if ndir > 1 else None)[0]
            dx = mark_ready(dx.view(T, B, I))
        for d in range(ndir):
            G = dgates[d].view(T * B, 4 * H)                         # gate-blocked = parameter order
            hd = hseq[:, :, d * H:(d + 1) * H]                       # strided view, row stride ndir*H
            # dW_hh = sum_t dgates_t^T h_prev(t): forward h_prev(t) = h_{t-1},
            # reverse h_{t+1}; the step next to the initial state pairs with h0
            g0 = G[:B] if d == 0 else G[(T - 1) * B:]
            seg2 = (g0, h0c[d]) if h0c is not None else None
            if T > 1:
                Gs = G[B:] if d == 0 else G[:(T - 1) * B]
                hs = (hd[:-1] if d == 0 else hd[1:]).reshape((T - 1) * B, H)
                dwhh = gemm_f32(Gs, True, hs, True, pairs2=seg2)[0]
            elif seg2 is not None:
                dwhh = gemm_f32(seg2[0], True, seg2[1], True)[0]
            else:
                dwhh = torch.zeros(4 * H, H, device=x.device, dtype=torch.float32)
            dwih, db = gemm_f32(G, True, x2, True, rowsum=True)
            grads += [dwih, dwhh, db if has_w[4 * d + 2] else None, db if has_w[4 * d + 3] else None]
        # (a detached carried state -- truncated BPTT -- needs no cast kernels)
        dh0_out = dh0.to(h0_dtype) if has_h0 and ctx.needs_input_grad[1] else None
        dc0_out = dc0.to(c0_dtype) if has_c0 and ctx.needs_input_grad[2] else None
        return (dx, dh0_out, dc0_out, None, *grads)


def _backward_gemms16(ctx, dgates, dh0, dc0, hseq, h0c, x2, wih):
    """16-bit layers: weight and input gradients on the in-tree MFMA GEMM
    (ops/gemm.py): dW_hh = sum_t dgates_t^T h_prev(t) with the initial-state
    pairing folded in as a second K segment, dW_ih = dG^T X, dX of both
    directions in one launch (K segments), fp32 accumulation throughout."""
    H, ndir, tile, rev_mask, has_w, has_h0, has_c0, h0_dtype, c0_dtype = ctx.cfg
    T, B, I = ctx.saved_tensors[0].shape
    grads: List[Optional[Tensor]] = []
    Gs = []
    params = getattr(ctx, "params", None)
    for d in range(ndir):
        G = dgates[d].view(T * B, 4 * H)                         # gate-blocked = parameter order
        Gs.append(G)
        hd = hseq[:, :, d * H:(d + 1) * H]                       # strided view, row stride ndir*H
        pairs = []
        if T > 1:
            if d == 0:
                pairs.append((G[B:], hd[:-1].reshape((T - 1) * B, H)))
            else:
                pairs.append((G[:(T - 1) * B], hd[1:].reshape((T - 1) * B, H)))
        if h0c is not None:
            pairs.append((G[:B] if d == 0 else G[(T - 1) * B:], h0c[d]))
        # direct mode (ops/gradsink.py): this direction's weight and bias
        # gradients accumulated into the flat gradient views by the GEMM
        # epilogue / split-K sum and the column-sum pass -- nothing for
        # autograd to add
        pw = params[4 * d:4 * d + 4] if params is not None else (None,) * 4
        sinks = [gradsink.sink(w, ctx.direct) if w is not None else None for w in pw]
        if params is not None and pairs and all(sk is not None for sk, w in zip(sinks, pw) if w is not None) and \
                sinks[0] is not None and sinks[1] is not None:
            mm_kk(pairs, accumulate_into=sinks[1])
            mm_kk([(G, x2)], accumulate_into=sinks[0])
            bs = [sk for sk in sinks[2:] if sk is not None]
            if bs:
                col_sum(G, accumulate_into=bs)
            grads += [None, None, None, None]
            continue
        dwhh = mm_kk(pairs) if pairs else torch.zeros(4 * H, H, device=G.device, dtype=torch.float32)
        dwih = mm_kk([(G, x2)])
        db = col_sum(G)  # in-tree deterministic column sums (fp32 accumulation of the 16-bit G)
        grads += [dwih, dwhh, db if has_w[4 * d + 2] else None, db if has_w[4 * d + 3] else None]
    dx = mm_nk16([(Gs[d], wih[d]) for d in range(ndir)]).view(T, B, I) if ctx.needs_input_grad[0] else None
    dh0_out = dh0.to(h0_dtype) if has_h0 and ctx.needs_input_grad[1] else None
    dc0_out = dc0.to(c0_dtype) if has_c0 and ctx.needs_input_grad[2] else None
    return (dx, dh0_out, dc0_out, None, *grads)


# ---------------------------------------------------------------------------
# Stacked-layer pipeline (fp32, one direction, H = 128 on the row-owning
# kernels).  The sequence is cut into C time chunks and every layer runs on a
# stream of its own (layer 0 on the caller's): layer l + 1 computes chunk c --
# its input projection, then its recurrence -- while layer l computes chunk
# c + 1, so the layers' recurrences (90 of 256 CUs each at the motion batch)
# overlap instead of running one after the other.  The backward is the mirror
# image: layer l's BPTT of chunk c starts as soon as the layer above has
# produced dX for that chunk, and each layer's weight gradients follow its
# recurrence on its stream (beside the recurrences of the layers below).
# Chunk boundaries carry the state through the full-length tensors
# (lstm_rows_fwd_range / lstm_rows_bwd_range), so the forward is
# bit-identical to one whole-sequence launch per layer.
#
# One stream per layer, nothing more: with GPU_MAX_HW_QUEUES = 4 (HIP's
# default) further streams share hardware queues, and an event wait on one of
# them stalls the others (measured: separate projection and weight-gradient
# streams made the step 25-70 % slower, profiles/r4/pipe/).
_PIPE_STREAMS = {}


def _pipe_stream(device, l: int) -> "torch.cuda.Stream":
    if l == 0:
        return torch.cuda.current_stream(device)
    s = _PIPE_STREAMS.get((device, l))
    if s is None:
        s = _PIPE_STREAMS[(device, l)] = torch.cuda.Stream(device=device, priority=-1)
    return s


def pipeline_chunks(T: int) -> List[Tuple[int, int]]:
    """[t0, t1) time chunks of the stacked-layer pipeline (PDRNN_TUNE large_chunks,
    default 3: at T = 128 4.54-4.57 ms/step against 4.69-4.79 with 2, 4 or 5
    chunks and 4.92 with 6, profiles/r4/pipe/p6_*)."""
    c = max(1, min(tune_int("large_chunks", 3), T))
    return [(T * i // c, T * (i + 1) // c) for i in range(c)]


def pipeline_ok(x: Tensor, hidden: int, num_layers: int, bidirectional: bool, dropout: float,
                training: bool) -> bool:
    """The stacked-layer pipeline covers unidirectional fp32 stacks of >= 2
    layers at the row-owning kernels' H (PDRNN_TUNE large_pipe=0 turns it off)."""
    if tune("large_pipe", "1") == "0" or _tile() >= 0:
        return False
    if x.dtype != torch.float32 or not x.is_cuda or bidirectional or num_layers < 2 or (dropout > 0 and training):
        return False
    mod = _ext.native(x.device)
    return mod is not None and hasattr(mod, "lstm_rows_range_supported") and bool(mod.lstm_rows_range_supported(hidden))


def _event(stream) -> "torch.cuda.Event":
    ev = torch.cuda.Event()
    ev.record(stream)
    return ev


def pipeline_streams(device, L: int) -> List["torch.cuda.Stream"]:
    """One stream per layer (layer 0: the caller's); the side streams first
    wait for everything the caller has queued (weights, shadows, buffers)."""
    main = torch.cuda.current_stream(device)
    streams = [_pipe_stream(device, l) for l in range(L)]
    for s in streams[1:]:
        s.wait_stream(main)
    return streams


def pipeline_join(streams) -> None:
    main = streams[0]
    for s in streams[1:]:
        main.wait_stream(s)


def pipeline_forward(streams, chunks, project, recur) -> None:
    """Issue the stacked-layer forward: for every chunk and layer,
    ``project(l, t0, t1)`` (l > 0, once the layer below has finished the
    chunk) then ``recur(l, t0, t1)``, on layer l's stream."""
    L = len(streams)
    done = [[None] * len(chunks) for _ in range(L)]
    for ci, (t0, t1) in enumerate(chunks):
        for l in range(L):
            with torch.cuda.stream(streams[l]):
                if l > 0:
                    streams[l].wait_event(done[l - 1][ci])
                    project(l, t0, t1)
                recur(l, t0, t1)
                done[l][ci] = _event(streams[l])


def pipeline_backward(streams, chunks, project, recur, finish) -> None:
    """Issue the stacked-layer backward, last chunk first: ``project(l, t0,
    t1)`` (dX of layer l + 1 for the chunk, once that layer has finished it),
    ``recur(l, first, t0, t1)`` (first: the chunk that starts the layer's
    BPTT), and after a layer's last chunk ``finish(l)`` (its weight
    gradients), on layer l's stream."""
    L = len(streams)
    done = [[None] * len(chunks) for _ in range(L)]
    last = len(chunks) - 1
    for ci in range(last, -1, -1):
        t0, t1 = chunks[ci]
        for l in range(L - 1, -1, -1):
            with torch.cuda.stream(streams[l]):
                if l < L - 1:
                    streams[l].wait_event(done[l + 1][ci])
                    project(l, t0, t1)
                recur(l, ci == last, t0, t1)
                done[l][ci] = _event(streams[l])
                if ci == 0:
                    finish(l)


class _PipelinedLSTMStack(torch.autograd.Function):
    """All layers of a unidirectional fp32 stack, chunk-pipelined (see above).
    x: [T, B, I] fp32; h0 / c0: [L, B, H] or None; weights: nn.LSTM
    ``_all_weights`` order, ``per`` (2 or 4) tensors per layer."""

    @staticmethod
    def forward(ctx, x, h0, c0, cfg, *weights):
        ctx.set_materialize_grads(False)
        H, L, per, chunks = cfg
        T, B, I = x.shape
        dev = x.device
        f32 = torch.float32
        mod = _ext.native(dev)
        lw = [list(weights[l * per:(l + 1) * per]) + ([None, None] if per == 2 else []) for l in range(L)]
        wih = [shadow(w[0], "i", f32, H) for w in lw]                 # [4H, I_l] gate-interleaved
        whh = [shadow(w[1], "i", f32, H) for w in lw]
        bias = [_bias_cat(w, 1, H, dev) for w in lw]
        h0s = [h0[l].float().contiguous() if h0 is not None else None for l in range(L)]
        c0s = [c0[l].float().contiguous() if c0 is not None else None for l in range(L)]
        hseq = [x.new_empty(T, B, H) for _ in range(L)]
        cseq = [x.new_empty(T, B, H) for _ in range(L)]
        acts = [x.new_empty(T, B, 4 * H) for _ in range(L)]
        xps = [gemm_f32(x.reshape(T * B, I), False, wih[0], False, bias=bias[0])[0].view(T, B, 4 * H)]
        xps += [x.new_empty(T, B, 4 * H) for _ in range(1, L)]
        rec = pipeline_streams(dev, L)

        def project(l, t0, t1):  # this chunk's input projection
            gemm_f32(hseq[l - 1][t0:t1].view(-1, H), False, wih[l], False, bias=bias[l],
                     out=xps[l][t0:t1].view(-1, 4 * H))

        def recur(l, t0, t1):
            mod.lstm_rows_fwd_range(xps[l][t0:t1], whh[l], h0s[l], c0s[l], hseq[l], cseq[l], acts[l], t0, t1, 0)

        pipeline_forward(rec, chunks, project, recur)
        pipeline_join(rec)
        # final h and c of every layer: one pack launch (ops/shadow.py)
        hn = hseq[0].new_empty(L, *hseq[0].shape[1:])
        cn = cseq[0].new_empty(L, *cseq[0].shape[1:])
        _sh.pack([_sh.job(hn[l], hq[T - 1]) for l, hq in enumerate(hseq)] +
                 [_sh.job(cn[l], cq[T - 1]) for l, cq in enumerate(cseq)], x.device)
        ctx.save_for_backward(x, *hseq, *cseq, *acts, *[shadow(w[0], "p", f32, H) for w in lw],
                              *[shadow(w[1], "t", f32, H) for w in lw])
        ctx.states = (h0s, c0s)
        ctx.params = lw  # (gradsink: the backward may accumulate into their .grad itself)
        ctx.direct = gradsink.enabled()
        ctx.cfg = (H, L, per, chunks, [[w is not None for w in ws] for ws in lw],
                   h0.dtype if h0 is not None else None, c0.dtype if c0 is not None else None)
        return hseq[L - 1], hn, cn

    @staticmethod
    def backward(ctx, dhseq, dhn, dcn):
        H, L, per, chunks, has_w, h0_dtype, c0_dtype = ctx.cfg
        h0s, c0s = ctx.states
        sv = ctx.saved_tensors
        x = sv[0]
        hseq, cseq, acts = sv[1:1 + L], sv[1 + L:1 + 2 * L], sv[1 + 2 * L:1 + 3 * L]
        wp, wt = sv[1 + 3 * L:1 + 4 * L], sv[1 + 4 * L:1 + 5 * L]
        T, B, I = x.shape
        dev = x.device
        mod = _ext.native(dev)
        dgates = [x.new_empty(T, B, 4 * H) for _ in range(L)]
        douts = [x.new_empty(T, B, H) for _ in range(L - 1)]
        douts.append(dhseq.float().contiguous() if dhseq is not None else None)
        dhb = [x.new_empty(B, H) for _ in range(L)]  # gradients leaving a chunk's first step
        dcb = [x.new_empty(B, H) for _ in range(L)]
        carry = [x.new_empty(B, H) for _ in range(L)]
        dhn_l = [dhn[l].float().contiguous() if dhn is not None else None for l in range(L)]
        dcn_l = [dcn[l].float().contiguous() if dcn is not None else None for l in range(L)]
        ins = [x] + list(hseq[:-1])  # each layer's input sequence
        # direct mode (ops/gradsink.py): a layer whose w_ih / w_hh (and biases)
        # all have flat .grad views accumulates into them in the GEMM epilogue
        sinks = [[gradsink.sink(w, ctx.direct) for w in ctx.params[l]] for l in range(L)]
        direct = [all(sk is not None for sk, w in zip(sinks[l], ctx.params[l]) if w is not None)
                  for l in range(L)]
        dwih = [sinks[l][0] if direct[l] else x.new_empty(4 * H, t.shape[2]) for l, t in enumerate(ins)]
        dwhh = [sinks[l][1] if direct[l] else x.new_empty(4 * H, H) for l in range(L)]
        db = [x.new_empty(4 * H) for _ in range(L)]
        rec = pipeline_streams(dev, L)

        def project(l, t0, t1):  # this chunk's dout = dX of the layer above
            # (one K slice: split-K partials and their sum beside the
            # recurrences cost more than they recover, profiles/r4/pipe/p6_*)
            gemm_f32(dgates[l + 1][t0:t1].view(-1, 4 * H), False, wp[l + 1], True, out=douts[l][t0:t1].view(-1, H),
                     splitk=1)

        def recur(l, first, t0, t1):
            dout = douts[l][t0:t1] if douts[l] is not None else None
            mod.lstm_rows_bwd_range(dout, dhn_l[l] if first else dhb[l], dcn_l[l] if first else dcb[l], wt[l],
                                    cseq[l], acts[l], c0s[l], dgates[l], dhb[l], dcb[l], carry[l], t0, t1, 0)

        def finish(l):  # the layer's recurrence is done: its weight gradients, on its stream
            # (direct mode: the row sums are added into the bias gradients as
            # they come out of the dW_ih pass, no copy into db first)
            rs = _chunk_weight_grads(dwih[l], dwhh[l], None if direct[l] else db[l], dgates[l], hseq[l], h0s[l],
                                     ins[l], 0, T, not direct[l], db_first=True)
            if direct[l]:
                db[l] = rs
                bi, bh = sinks[l][2], sinks[l][3]
                # (same storage too: two separately allocated gradients can sit
                # side by side in the caching allocator -- ADVICE r5)
                if bi is not None and bh is not None and bh.data_ptr() == bi.data_ptr() + bi.numel() * 4 and \
                        bi.untyped_storage().data_ptr() == bh.untyped_storage().data_ptr():
                    # b_ih, b_hh adjacent in the flat gradient: one launch for both
                    torch.as_strided(bi, (2, bi.numel()), (bi.numel(), 1)).add_(db[l])
                else:
                    for bg in (bi, bh):
                        if bg is not None:
                            bg.add_(db[l])

        pipeline_backward(rec, chunks, project, recur, finish)
        dx = None
        if ctx.needs_input_grad[0]:  # (layer 0's stream is the caller's)
            dx = gemm_f32(dgates[0].view(T * B, 4 * H), False, wp[0], True)[0].view(T, B, I)
        pipeline_join(rec)
        grads: List[Optional[Tensor]] = []
        for l in range(L):
            if direct[l]:  # already accumulated into the parameters' .grad
                grads += [None, None] + ([None, None] if per == 4 else [])
                continue
            grads += [dwih[l], dwhh[l]]
            if per == 4:
                grads += [db[l] if has_w[l][2] else None, db[l] if has_w[l][3] else None]
        dh0 = torch.stack(dhb).to(h0_dtype) if h0_dtype is not None else None
        dc0 = torch.stack(dcb).to(c0_dtype) if c0_dtype is not None else None
        return (dx, dh0, dc0, None, *grads)


def padded_cols(x2: Tensor, mult: int = 32) -> Tensor:
    """x2 [K, n] zero-padded to a multiple of ``mult`` columns (one copy).  A
    weight-gradient GEMM against a narrow, unaligned input (the motion model's
    9 features: rows of 36 bytes) runs gemm_f32's bounds-checked loop, whose
    loads do not overlap its MFMAs; padded, every tile is whole and aligned
    (layer 0's dW_ih 214 -> ~90 us at the motion batch, profiles/r4/gemm_probe/)."""
    n = x2.shape[1]
    shape = (x2.shape[0], -(-n // mult) * mult)
    # the padded buffer is kept per (shape, dtype, device, stream): its pad
    # columns are zeroed once, a step only copies the data columns (one
    # dispatch, not a fill and a copy); reuse is stream-ordered
    if x2.is_cuda and torch.cuda.is_current_stream_capturing():  # (graph-pool memory: never cached)
        out = x2.new_zeros(shape)
        out[:, :n].copy_(x2)
        return out
    key = (shape, x2.dtype, x2.device, torch.cuda.current_stream(x2.device).cuda_stream if x2.is_cuda else 0)
    out = _PADDED.get(key)
    if out is None:
        if len(_PADDED) >= 8:
            _PADDED.clear()
        out = _PADDED[key] = x2.new_zeros(shape)
    out[:, :n].copy_(x2)
    return out


_PADDED: dict = {}


def _chunk_weight_grads(dwih: Tensor, dwhh: Tensor, db: Optional[Tensor], G3: Tensor, hd: Tensor, h0: Optional[Tensor],
                        xin: Tensor, t0: int, t1: int, first: bool, db_first: Optional[bool] = None) -> Tensor:
    """Steps [t0, t1) of one unidirectional fp32 layer's dW_ih, dW_hh and db,
    written (first chunk) or accumulated into the fp32 outputs: dW_hh pairs
    dgates_t with h_{t-1} (h0 at t = 0), dW_ih dgates_t with the layer input,
    db = the row sums of the dW_ih pass."""
    H4 = G3.shape[2]
    H = H4 // 4
    lo = max(t0, 1)
    seg0 = (G3[0], h0) if t0 == 0 and h0 is not None else None
    if t1 > lo:
        gemm_f32(G3[lo:t1].view(-1, H4), True, hd[lo - 1:t1 - 1].reshape(-1, H), True, pairs2=seg0, out=dwhh,
                 accumulate=not first)
    elif seg0 is not None:
        gemm_f32(seg0[0], True, seg0[1], True, out=dwhh, accumulate=not first)
    elif first:
        dwhh.zero_()
    x2 = xin[t0:t1].reshape(-1, xin.shape[2])
    if x2.shape[1] % 32:  # narrow input (motion: 9 features): whole, aligned column tiles
        c, rs = gemm_f32(G3[t0:t1].view(-1, H4), True, padded_cols(x2), True, rowsum=True)
        dwih.copy_(c[:, :x2.shape[1]]) if first else dwih.add_(c[:, :x2.shape[1]])
    else:
        _, rs = gemm_f32(G3[t0:t1].view(-1, H4), True, x2, True, rowsum=True, out=dwih, accumulate=not first)
    if db is None:  # the caller takes the row sums as they are
        return rs
    if first if db_first is None else db_first:
        db.copy_(rs)
    else:
        db.add_(rs)
    return db


def lstm_large_forward(x: Tensor, weights: Sequence[Optional[Tensor]], h0: Optional[Tensor],
                       c0: Optional[Tensor], *, hidden: int, num_layers: int, batch_first: bool,
                       bidirectional: bool = False, dropout: float = 0.0,
                       training: bool = False) -> Tuple[Tensor, Tensor, Tensor]:
    """Stacked (bi)LSTM on the MFMA step kernels; nn.LSTM-compatible outputs.

    ``weights``: nn.LSTM ``_all_weights`` order (per layer and direction
    w_ih, w_hh[, b_ih, b_hh])."""
    ndir = 2 if bidirectional else 1
    per = len(weights) // (num_layers * ndir)
    seq = x.transpose(0, 1) if batch_first else x
    seq = seq.contiguous()  # (a no-op for an index-gathered batch: see lstm_forward)
    B = seq.shape[1]
    if pipeline_ok(seq, hidden, num_layers, bidirectional, dropout, training):
        out, hn, cn = _PipelinedLSTMStack.apply(seq, h0, c0, (hidden, num_layers, per, pipeline_chunks(seq.shape[0])),
                                                *weights)
        return (out.transpose(0, 1) if batch_first else out), hn, cn
    tile = _tile()
    hns, cns = [], []
    for l in range(num_layers):
        ws: List[Optional[Tensor]] = []
        for d in range(ndir):
            chunk = list(weights[(l * ndir + d) * per:(l * ndir + d + 1) * per])
            if per == 2:
                chunk += [None, None]
            ws += chunk
        h0l = h0[l * ndir:(l + 1) * ndir] if h0 is not None else None
        c0l = c0[l * ndir:(l + 1) * ndir] if c0 is not None else None
        seq, hn, cn = _LargeLSTMLayer.apply(seq, h0l, c0l, (hidden, ndir, tile), *ws)
        hns.append(hn)
        cns.append(cn)
        if dropout > 0 and training and l < num_layers - 1:
            seq = torch.nn.functional.dropout(seq, dropout, True)
    out = seq.transpose(0, 1) if batch_first else seq
    if num_layers == 1:
        return out, hns[0], cns[0]
    hn, cn = _StackStates.apply(num_layers, *hns, *cns)
    return out, hn, cn
