"""Fused softmax cross-entropy (+ accuracy counts).

Replaces ``CrossEntropyLoss`` plus the ``argmax == labels`` accuracy of the
reference train step (reference: src/motion/trainer/base.py:15,112,114).  On a
GPU one HIP pass computes the mean loss, the number of correct argmax
predictions and the unscaled gradient; the backward is one scale.
"""
from __future__ import annotations

from typing import Tuple

import torch
import torch.nn.functional as F
from torch import Tensor

from .. import _ext


class _FusedXent(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, ignore_index):
        mod = _ext.native(logits.device)
        stats, dlogits = mod.xent_fwd(logits, labels, ignore_index, logits.requires_grad)
        ctx.save_for_backward(dlogits, stats)
        ctx.in_dtype = logits.dtype
        ctx.mark_non_differentiable(stats)
        return stats[0], stats

    @staticmethod
    def backward(ctx, gloss, _gstats):
        dlogits, stats = ctx.saved_tensors
        mod = _ext.native(dlogits.device)
        od = ctx.in_dtype if ctx.in_dtype in (torch.bfloat16, torch.float16) else torch.float32
        g = mod.xent_bwd(dlogits, gloss.reshape(1), stats, od)  # 16-bit logits: 16-bit gradient, no cast
        if g.dtype != ctx.in_dtype:
            g = g.to(ctx.in_dtype)
        return g, None, None


def cross_entropy_with_stats(logits: Tensor, labels: Tensor,
                             ignore_index: int = -100) -> Tuple[Tensor, Tensor]:
    """Returns (mean loss, stats) with stats = [loss, n_valid, n_correct] (device tensor)."""
    if logits.dim() != 2:
        logits = logits.reshape(-1, logits.shape[-1])
    labels = labels.reshape(-1)
    mod = _ext.native(logits.device)
    if mod is not None and logits.stride(-1) == 1:
        return _FusedXent.apply(logits, labels.long().contiguous(), ignore_index)
    loss = F.cross_entropy(logits, labels.long(), ignore_index=ignore_index)
    with torch.no_grad():
        valid = labels != ignore_index
        correct = ((logits.argmax(dim=1) == labels) & valid).sum()
        stats = torch.stack([loss.detach().float(), valid.sum().float(), correct.float()])
    return loss, stats


def cross_entropy(logits: Tensor, labels: Tensor, ignore_index: int = -100) -> Tensor:
    return cross_entropy_with_stats(logits, labels, ignore_index)[0]


class CrossEntropyLoss(torch.nn.Module):
    """Drop-in for ``nn.CrossEntropyLoss()`` (mean reduction) on the fused kernel.

    ``last_stats`` keeps the [loss, n_valid, n_correct] tensor of the latest
    call so trainers can log accuracy without another argmax pass."""

    def __init__(self, ignore_index: int = -100):
        super().__init__()
        self.ignore_index = ignore_index
        self.last_stats = None

    def forward(self, logits: Tensor, labels: Tensor) -> Tensor:
        loss, stats = cross_entropy_with_stats(logits, labels, self.ignore_index)
        self.last_stats = stats
        return loss
