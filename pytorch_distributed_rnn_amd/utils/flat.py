"""Flat parameter / gradient storage.

Every model trained by this framework can have its parameters re-homed into ONE
contiguous buffer per (device, dtype) and its gradients into a matching flat
gradient buffer (``param.grad`` are views).  That single layout is shared by

* the fused Adam kernel (one launch over the whole model),
* the gradient reducer (all-reduce buckets are contiguous slices of the flat
  gradient buffer -- no pack/unpack copies),
* parameter broadcast at wrap time (one collective).

This is the MI355X-native replacement for torch 1.4's per-parameter optimizer
loop and DDP's separate bucket copies (reference: src/motion/trainer/base.py:43,
src/motion/trainer/ddp.py:19).
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import torch
from torch import Tensor, nn


def _storage_key(t: Tensor) -> int:
    return t.untyped_storage().data_ptr()


def contiguous_span(tensors: Sequence[Tensor]) -> Optional[Tuple[Tensor, int, int]]:
    """If ``tensors`` are contiguous views laid back to back (in order) in one
    storage, return (base_flat_view, start, numel)."""
    if not tensors:
        return None
    t0 = tensors[0]
    key = _storage_key(t0)
    esz = t0.element_size()
    start = t0.storage_offset()
    pos = start
    for t in tensors:
        if not t.is_contiguous() or _storage_key(t) != key or t.dtype != t0.dtype:
            return None
        if t.storage_offset() != pos:
            return None
        pos += t.numel()
    total = pos - start
    base = torch.empty(0, dtype=t0.dtype, device=t0.device)
    base.set_(t0.untyped_storage(), start, (total,), (1,))
    del esz
    return base, start, total


class FlatParameters:
    """Re-home ``params`` into one flat buffer (+ flat grad buffer).

    Parameters must share device and dtype.  After construction
    ``p.data`` is a view of :attr:`data` and ``p.grad`` a view of
    :attr:`grad` for every parameter, in the given order."""

    def __init__(self, params: Iterable[nn.Parameter], with_grad: bool = True):
        self.params: List[nn.Parameter] = [p for p in params]
        if not self.params:
            raise ValueError("no parameters")
        dev, dt = self.params[0].device, self.params[0].dtype
        for p in self.params:
            if p.device != dev or p.dtype != dt:
                raise ValueError("FlatParameters needs a single device/dtype group")
        self.numels = [p.numel() for p in self.params]
        self.offsets = []
        off = 0
        for n in self.numels:
            self.offsets.append(off)
            off += n
        self.total = off
        existing = contiguous_span([p.data for p in self.params])
        if existing is not None:
            self.data = existing[0]
        else:
            self.data = torch.empty(self.total, dtype=dt, device=dev)
            for p, o, n in zip(self.params, self.offsets, self.numels):
                self.data[o:o + n].copy_(p.data.reshape(-1))
                p.data = self.data[o:o + n].view_as(p)
        self.grad: Optional[Tensor] = None
        if with_grad:
            self.grad = torch.zeros(self.total, dtype=dt, device=dev)
            self.attach_grads()

    def param_view(self, i: int) -> Tensor:
        o, n = self.offsets[i], self.numels[i]
        return self.data[o:o + n].view_as(self.params[i])

    def grad_view(self, i: int) -> Tensor:
        o, n = self.offsets[i], self.numels[i]
        return self.grad[o:o + n].view_as(self.params[i])

    def attach_grads(self) -> None:
        """(Re-)point every ``p.grad`` at its flat view, folding in any grad
        the autograd engine allocated on its own."""
        for i, p in enumerate(self.params):
            v = self.grad_view(i)
            g = p.grad
            if g is None:
                p.grad = v
            elif g.data_ptr() != v.data_ptr():
                v.copy_(g)
                p.grad = v

    def zero_grad(self) -> None:
        self.grad.zero_()
        self.attach_grads()

    def grads_attached(self) -> bool:
        return all(p.grad is not None and p.grad.data_ptr() == self.grad_view(i).data_ptr()
                   for i, p in enumerate(self.params))


def flatten_module(module: nn.Module, with_grad: bool = True) -> Dict[Tuple[torch.device, torch.dtype], FlatParameters]:
    """Group a module's trainable parameters by (device, dtype) and flatten each group."""
    groups: Dict[Tuple[torch.device, torch.dtype], List[nn.Parameter]] = {}
    for p in module.parameters():
        if p.requires_grad:
            groups.setdefault((p.device, p.dtype), []).append(p)
    out = {k: FlatParameters(v, with_grad=with_grad) for k, v in groups.items()}
    module._pdrnn_flat = out  # type: ignore[attr-defined]
    return out
