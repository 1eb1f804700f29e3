"""Embedding lookup on the native gather / deterministic CSR-backward kernels
(csrc/kernels/embedding.hip).  New capability for the char-LM configuration
(BASELINE config 4); the reference has no embedding."""
from __future__ import annotations

from typing import Optional

import torch
from torch import Tensor
from torch.nn import functional as F

from .. import _ext


class _Embedding(torch.autograd.Function):
    @staticmethod
    def forward(ctx, weight, idx, out_dtype, padding_idx):
        from . import gradsink
        mod = _ext.native(weight.device)
        out = mod.embedding_fwd(weight.contiguous(), idx, out_dtype)
        ctx.save_for_backward(idx)
        ctx.meta = (weight.shape[0], -1 if padding_idx is None else padding_idx)
        ctx.param = weight  # (gradsink: the backward may accumulate into its .grad)
        ctx.direct = gradsink.enabled()
        return out

    @staticmethod
    def backward(ctx, dout):
        from . import gradsink
        (idx,) = ctx.saved_tensors
        V, pad = ctx.meta
        mod = _ext.native(dout.device)
        sk = gradsink.sink(ctx.param, ctx.direct)
        if sk is not None:  # direct mode: the row sums added into the flat gradient view
            mod.embedding_bwd(dout.contiguous(), idx, V, pad, out=sk)
            return None, None, None, None
        return mod.embedding_bwd(dout.contiguous(), idx, V, pad), None, None, None


def embedding(idx: Tensor, weight: Tensor, out_dtype: Optional[torch.dtype] = None,
              padding_idx: Optional[int] = None) -> Tensor:
    """``F.embedding`` with the cast to ``out_dtype`` fused into the gather."""
    mod = _ext.native(weight.device)
    if mod is not None and weight.dtype == torch.float32 and weight.is_cuda:
        return _Embedding.apply(weight, idx, out_dtype, padding_idx)
    out = F.embedding(idx, weight, padding_idx=padding_idx)
    return out.to(out_dtype) if out_dtype is not None else out
