"""Time-batched GEMMs of the large-H layers on the in-tree MFMA kernel
(``csrc/kernels/gemm.hip``), with the library (hipBLASLt through torch) as the
fallback for shapes the kernel does not cover, CPU tensors and fp32.

* :func:`linear16`  -- ``Xp = x W^T + b`` (input projection, 16-bit out, fp32 bias);
* :func:`mm_kk`     -- ``sum_s A_s^T B_s`` over K-major pairs, fp32 out (weight
  gradients; a second pair folds the initial-state term of dW_hh into the same
  launch); split-K when the output has too few 256 x 256 tiles to fill the GPU;
* :func:`mm_nk16`   -- ``sum_s G_s W_s`` with W stored [K, N] (input gradient
  of both directions in one launch), 16-bit out.

``PDRNN_GEMM=torch`` forces the library path (A/B comparisons).
SURVEY N1: input projection and dW/dX on the matrix cores; the reference
trains the same cell through torch.nn.LSTM (reference: src/motion/model.py:9).
"""
from __future__ import annotations

import os
from typing import Optional, Sequence, Tuple

import torch
from torch import Tensor

from .. import _ext
from . import shadow as _shadow

_CUS = {}


def _native(t: Tensor):
    if os.environ.get("PDRNN_GEMM", "mfma") == "torch":
        return None
    if t.device.type != "cuda" or t.dtype not in (torch.bfloat16, torch.float16):
        return None
    mod = _ext.native(t.device)
    return mod if mod is not None and hasattr(mod, "gemm16") else None


def _variant() -> int:
    # the build's default schedule (kernels/gemm.hip: 3 = B_n1 refill in Q3 +
    # DMA after the fragment reads; +32 = raster groups of 4 tile-rows, +2-4 %
    # over 8 on the bi-LSTM shapes, profiles/r3_gemm/raster.log)
    return 0


def _cus(dev) -> int:
    n = _CUS.get(dev)
    if n is None:
        n = _CUS[dev] = torch.cuda.get_device_properties(dev).multi_processor_count
    return n


def _splitk(dev, M: int, N: int, K: int) -> int:
    """K splits that bring the launch to >= 1.5 workgroups per CU (fp32 partials
    summed in fixed order), at least 16 K-tiles per split."""
    tiles = ((M + 255) // 256) * ((N + 255) // 256)
    cus = _cus(dev)
    if tiles >= cus:
        return 1
    s = min((3 * cus // 2 + tiles - 1) // tiles, max(1, K // (64 * 16)), 16)
    return max(1, s)


def _rowmajor(t: Tensor) -> bool:
    """Row-major 2-D operand the in-tree GEMM can stream: unit column stride,
    row stride a multiple of 8 elements and a 16-byte aligned base (its LDS
    DMA issues 16-byte loads from base + row * ld + 8 * chunk)."""
    return t.dim() == 2 and t.stride(1) == 1 and t.stride(0) >= t.shape[1] and t.stride(0) % 8 == 0 and \
        t.data_ptr() % 16 == 0


def linear16(x: Tensor, w: Tensor, bias: Optional[Tensor]) -> Tensor:
    """x [M, K] @ w[N, K]^T + bias[N] in x's dtype (fp32 bias and accumulation)."""
    mod = _native(x)
    M, K = x.shape
    N = w.shape[0]
    if mod is not None and _rowmajor(x) and _rowmajor(w) and w.dtype == x.dtype and \
            mod.gemm16_supported(M, N, K, 0, False, False, True):
        b = bias.float().contiguous() if bias is not None else None
        return mod.gemm16(x, False, w, False, bias=b, out16=True, variant=_variant())
    if bias is None:
        return torch.mm(x, w.t())
    return torch.addmm(bias.to(x.dtype), x, w.t())


def mm_kk(pairs: Sequence[Tuple[Tensor, Tensor]], accumulate_into: Optional[Tensor] = None) -> Tensor:
    """sum over (a [K_s, M], b [K_s, N]) of a^T b, fp32 [M, N] (1 or 2 pairs);
    ``accumulate_into``: added into that contiguous fp32 [M, N] tensor by the
    GEMM's epilogue / split-K sum (a parameter's gradient, ops/gradsink.py)."""
    a, b = pairs[0]
    mod = _native(a)
    M, N = a.shape[1], b.shape[1]
    K1 = a.shape[0]
    K2 = pairs[1][0].shape[0] if len(pairs) > 1 else 0
    ok = mod is not None and all(_rowmajor(p) and p.dtype == a.dtype for pr in pairs for p in pr) and \
        len(pairs) <= 2 and mod.gemm16_supported(M, N, K1, K2, True, True, False)
    if ok:
        sk = _splitk(a.device, M, N, K1 + K2)
        kw = dict(out=accumulate_into, accumulate=True) if accumulate_into is not None else {}
        if len(pairs) == 2:
            return mod.gemm16(a, True, b, True, A2=pairs[1][0], B2=pairs[1][1], splitk=sk, variant=_variant(), **kw)
        return mod.gemm16(a, True, b, True, splitk=sk, variant=_variant(), **kw)
    out = accumulate_into
    for a_, b_ in pairs:
        try:
            r = torch.mm(a_.t(), b_, out_dtype=torch.float32)
        except (RuntimeError, TypeError):
            r = torch.mm(a_.t().float(), b_.float())
        out = r if out is None else out.add_(r)
    return out


def mm_nk16(pairs: Sequence[Tuple[Tensor, Tensor]]) -> Tensor:
    """sum over (g [M, K_s], w [K_s, N]) of g w in g's dtype (1 or 2 pairs)."""
    g, w = pairs[0]
    mod = _native(g)
    M, N = g.shape[0], w.shape[1]
    K1 = g.shape[1]
    K2 = pairs[1][0].shape[1] if len(pairs) > 1 else 0
    ok = mod is not None and all(_rowmajor(p) and p.dtype == g.dtype for pr in pairs for p in pr) and \
        len(pairs) <= 2 and mod.gemm16_supported(M, N, K1, K2, False, True, True)
    if ok:
        if len(pairs) == 2:
            return mod.gemm16(g, False, w, True, A2=pairs[1][0], B2=pairs[1][1], out16=True, variant=_variant())
        return mod.gemm16(g, False, w, True, out16=True, variant=_variant())
    out = torch.mm(g, w)
    for g_, w_ in pairs[1:]:
        out.addmm_(g_, w_)
    return out


class _Linear16(torch.autograd.Function):
    """y = x W^T + b with 16-bit x, fp32 master W / b: the forward, dX and dW
    products on the in-tree GEMM (fp32 dW / db straight into the masters'
    gradients, no cast kernels on the backward)."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        from . import gradsink
        shp = x.shape
        x2 = x.reshape(-1, shp[-1])
        w16 = _shadow.cast(weight, x.dtype)  # converted once per optimizer step (ops/shadow.py)
        y = linear16(x2, w16, bias.detach() if bias is not None else None)
        ctx.save_for_backward(x2, w16)
        ctx.has_bias = bias is not None
        ctx.shp = shp
        ctx.params = (weight, bias)  # (gradsink: the backward may accumulate into their .grad)
        ctx.direct = gradsink.enabled()
        return y.view(*shp[:-1], w16.shape[0])

    @staticmethod
    def backward(ctx, dy):
        from . import gradsink
        x2, w16 = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1]).to(x2.dtype).contiguous()
        dx = mm_nk16([(dy2, w16)]).view(ctx.shp) if ctx.needs_input_grad[0] else None
        sw, sb = gradsink.sink(ctx.params[0], ctx.direct), gradsink.sink(ctx.params[1], ctx.direct)
        if sw is not None and (not ctx.has_bias or sb is not None):
            # direct mode: dW and db added into the flat gradient views
            mm_kk([(dy2, x2)], accumulate_into=sw)
            if ctx.has_bias:
                col_sum(dy2, accumulate_into=[sb])
            return dx, None, None
        dw = mm_kk([(dy2, x2)]) if ctx.needs_input_grad[1] else None
        db = col_sum(dy2) if ctx.has_bias and ctx.needs_input_grad[2] else None
        return dx, dw, db


class _LinearNarrow(torch.autograd.Function):
    """y = x W^T + b with fp32 master W / b on the fp32-product GEMM
    (kernels/gemm_f32.hip): fp32 x (any width), or a 16-bit x with a narrow
    output (N < 128, e.g. a classifier head: 32 / 64-wide tiles instead of an
    idle 256-wide ping-pong tile) -- forward, dX, dW and db (the row sums of
    dy^T, fused into the dW pass)."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        shp = x.shape
        x2 = x.reshape(-1, shp[-1])
        w16 = _shadow.cast(weight, x.dtype)  # converted once per optimizer step (ops/shadow.py)
        o16 = x.dtype != torch.float32
        y, _ = gemm_f32(x2, False, w16, False, bias=bias.detach().float() if bias is not None else None, out16=o16)
        ctx.save_for_backward(x2, w16)
        ctx.has_bias = bias is not None
        ctx.shp = shp
        from . import gradsink
        ctx.params = (weight, bias)  # (gradsink: the backward may accumulate into their .grad)
        ctx.direct = gradsink.enabled()
        return y.view(*shp[:-1], w16.shape[0])

    @staticmethod
    def backward(ctx, dy):
        from . import gradsink
        x2, w16 = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1]).to(x2.dtype).contiguous()
        o16 = x2.dtype != torch.float32
        dx = gemm_f32(dy2, False, w16, True, out16=o16)[0].view(ctx.shp) if ctx.needs_input_grad[0] else None
        sw, sb = gradsink.sink(ctx.params[0], ctx.direct), gradsink.sink(ctx.params[1], ctx.direct)
        if sw is not None and (not ctx.has_bias or sb is not None):
            # direct mode: dW accumulated into the flat gradient view by the GEMM
            # epilogue, db (its row sums) added: nothing for autograd to add
            _, rs = gemm_f32(dy2, True, x2, True, rowsum=ctx.has_bias, out=sw, accumulate=True)
            if ctx.has_bias:
                sb.add_(rs)
            return dx, None, None
        dw = db = None
        if ctx.needs_input_grad[1] or (ctx.has_bias and ctx.needs_input_grad[2]):
            dw, db = gemm_f32(dy2, True, x2, True, rowsum=ctx.has_bias)
        return dx, dw if ctx.needs_input_grad[1] else None, db if ctx.has_bias and ctx.needs_input_grad[2] else None


def linear(x: Tensor, weight: Tensor, bias: Optional[Tensor]) -> Tensor:
    """F.linear(x, weight.to(x.dtype), bias.to(x.dtype)) for a 16-bit x and fp32
    parameters; on the in-tree GEMM when the shape fits it (output width a
    multiple of 8 and at least 128 -- a narrower head would leave most of a
    256-wide tile idle, the library keeps those)."""
    mod = _native(x)
    N, K = weight.shape
    if mod is not None and x.dtype != torch.float32 and N >= 128 and N % 8 == 0 and K % 64 == 0 and x.shape[-1] == K:
        return _Linear16.apply(x.contiguous(), weight, bias)
    if _native_f32(x) is not None and x.shape[-1] == K and weight.dtype == torch.float32 and (
            (mod is not None and N < 128) or x.dtype == torch.float32):
        return _LinearNarrow.apply(x.contiguous(), weight, bias)
    import torch.nn.functional as F
    return F.linear(x, weight.to(x.dtype), bias.to(x.dtype) if bias is not None else None)


# ------------------------------------------------------------------ fp32 GEMM
def _native_f32(t: Tensor):
    if os.environ.get("PDRNN_GEMM", "mfma") == "torch" or t.device.type != "cuda":
        return None
    mod = _ext.native(t.device)
    return mod if mod is not None and hasattr(mod, "gemm_f32") else None


def _unit_inner(t: Tensor) -> bool:
    # the native binding requires a unit inner stride (a [K, 1] view with any
    # other stride would be rejected there instead of taking the torch path)
    return t.dim() == 2 and t.stride(1) == 1 and t.stride(0) >= 1


def _splitk_f32(dev, M: int, N: int, K: int) -> int:
    """K splits bringing the fp32 GEMM to ~4 workgroups per CU (partials summed
    in fixed order), at least 8 k-tiles of 16 per split.  A few output tiles
    over a long K (the bi-LSTM head's dW: 64 tiles, K = 262144) carry little
    MFMA work per k-tile and are bound by load latency: the more workgroups in
    flight (LDS holds 4 per CU), the more k-tiles in flight."""
    bn = 32 if N <= 32 else 64 if N <= 64 else 128
    tiles = ((M + 127) // 128) * ((N + bn - 1) // bn)
    want = 4 * _cus(dev)
    if tiles >= want:
        return 1
    return max(1, min((want + tiles - 1) // tiles, max(1, K // (16 * 8)), 128))


def gemm_f32(a: Tensor, a_kmajor: bool, b: Tensor, b_kmajor: bool, pairs2=None, bias: Optional[Tensor] = None,
             rowsum: bool = False, out16: bool = False, out: Optional[Tensor] = None,
             accumulate: bool = False, splitk: Optional[int] = None) -> Tuple[Tensor, Optional[Tensor]]:
    """C = op(a) op(b)^T (+ op(a2) op(b2)^T) (+ bias), fp32 products and
    accumulation on the matrix cores (kernels/gemm_f32.hip); ``rowsum``: also
    the sums over K of op(a) (the bias gradient of a dW = G^T X product);
    ``accumulate``: C = out + ..., fp32 ``out`` (the row sums are not
    accumulated); ``splitk``: K slices instead of the occupancy heuristic.
    ``op``: a k-major operand is stored [K, rows].  Torch fallback without the
    extension (CPU)."""
    mod = _native_f32(a)
    ops = [a, b] + (list(pairs2) if pairs2 else [])
    if mod is not None and all(_unit_inner(t) and t.dtype == a.dtype for t in ops):
        M = a.shape[1] if a_kmajor else a.shape[0]
        N = b.shape[1] if b_kmajor else b.shape[0]
        K = (a.shape[0] if a_kmajor else a.shape[1]) + ((pairs2[0].shape[0] if a_kmajor else pairs2[0].shape[1])
                                                         if pairs2 else 0)
        sk = 1 if (bias is not None or out16) else (splitk or _splitk_f32(a.device, M, N, K))
        kw = dict(bias=bias, rowsum=rowsum, out16=out16, splitk=sk)
        if pairs2:
            kw.update(A2=pairs2[0], B2=pairs2[1])
        if out is not None:
            if sk > 1 and not out.is_contiguous():
                kw["splitk"] = 1
            kw["out"] = out
            kw["accumulate"] = accumulate
        c, rs = mod.gemm_f32(a, a_kmajor, b, b_kmajor, **kw)
        return c, (rs if rowsum else None)
    oa = (lambda t: t.t() if a_kmajor else t)
    ob = (lambda t: t if b_kmajor else t.t())
    c = oa(a).float() @ ob(b).float()
    if pairs2:
        c = c + oa(pairs2[0]).float() @ ob(pairs2[1]).float()
    if bias is not None:
        c = c + bias.float()
    rs = None
    if rowsum:
        rs = oa(a).float().sum(1)
        if pairs2:
            rs = rs + oa(pairs2[0]).float().sum(1)
    c = c.to(a.dtype) if out16 else c
    if out is not None:
        out.add_(c) if accumulate else out.copy_(c)
        c = out
    return c, rs


def col_sum(x: Tensor, accumulate_into: Optional[Sequence[Tensor]] = None) -> Tensor:
    """fp32 column sums of a 2-D tensor (fp32 or 16-bit): in-tree and
    deterministic on the GPU, torch on the CPU.  ``accumulate_into``: added
    into each of those fp32 [cols] tensors instead (bias gradients)."""
    mod = _native_f32(x)
    if mod is not None and x.dim() == 2 and x.stride(1) == 1 and x.dtype in (torch.float32, torch.bfloat16,
                                                                              torch.float16):
        return mod.col_sum(x, list(accumulate_into) if accumulate_into else None)
    s = x.sum(0, dtype=torch.float32)
    if accumulate_into:
        for o in accumulate_into:
            o.add_(s)
        return accumulate_into[0]
    return s
