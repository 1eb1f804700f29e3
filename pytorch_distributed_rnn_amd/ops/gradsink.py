"""Weight gradients written straight into the flat gradient buffer.

Autograd delivers a custom Function's weight gradient as a new tensor and
``AccumulateGrad`` then adds it into ``param.grad`` -- with the flat gradient
views of :func:`~pytorch_distributed_rnn_amd.utils.flat.flatten_module`, one
``CUDAFunctor_add`` launch per parameter and step (10 of the fp32 H = 128
motion step's 83 dispatches).  Inside :func:`direct_grads` the in-tree
Functions (``ops/lstm_large.py`` stacked-layer pipeline, ``ops/gemm.py``
narrow linear) instead accumulate into ``param.grad`` themselves -- the GEMM
epilogue's ``accumulate`` into the view -- and return no gradient for those
parameters, so autograd has nothing to add.

The trainer enables it for a single process without forced collectives.
(Post-accumulate-grad hooks still fire -- AccumulateGrad runs with an
undefined gradient and leaves ``.grad`` as the Function wrote it -- so DDP's
bucket hooks would see the finished view; multi-rank runs are nevertheless
kept on the plain path, where that ordering is the tested one.)
"""
from __future__ import annotations

import contextlib
import threading
from typing import Optional

import torch
from torch import Tensor

_STATE = threading.local()


def enabled() -> bool:
    return getattr(_STATE, "on", False)


@contextlib.contextmanager
def direct_grads(on: bool = True):
    old = enabled()
    _STATE.on = bool(on)
    try:
        yield
    finally:
        _STATE.on = old


def sink(p: Optional[Tensor], on: bool) -> Optional[Tensor]:
    """``p.grad`` when a backward may accumulate into it in place (``on``: the
    direct mode captured at FORWARD time -- the autograd engine runs a CUDA
    backward on its own worker thread, which does not see this thread's
    flag; an fp32 contiguous gradient that already exists), else None."""
    if p is None or not on or not p.requires_grad:
        return None
    g = p.grad
    if g is None or g.dtype != torch.float32 or not g.is_contiguous() or g.shape != p.shape:
        return None
    return g
