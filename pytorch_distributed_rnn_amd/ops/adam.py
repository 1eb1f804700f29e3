"""Fused Adam / AdamW over flat parameter storage.

The reference optimizer is ``torch.optim.Adam(model.parameters(), lr)``
(reference: src/motion/trainer/base.py:42-43) whose torch 1.4 implementation
is a Python loop of ATen ops per parameter.  :class:`FusedAdam` keeps the exact
``torch.optim.Adam`` API and ``state_dict`` format (per-parameter ``step``,
``exp_avg``, ``exp_avg_sq``; same param_group keys) so checkpoints are
interchangeable, but on MI355X a step is ONE HIP launch over the flat
parameter / gradient / moment buffers (``csrc/kernels/adam.hip``).  On CPU it
is exactly ``torch.optim.Adam``.
"""
from __future__ import annotations

from typing import List, Optional

import torch
from torch import Tensor

from .. import _ext
from ..utils.flat import contiguous_span


class FusedAdam(torch.optim.Adam):
    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, amsgrad: bool = False, *, maximize: bool = False,
                 decoupled_weight_decay: bool = False, grad_scale: float = 1.0):
        kw = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=amsgrad,
                  maximize=maximize)
        try:
            super().__init__(params, decoupled_weight_decay=decoupled_weight_decay, **kw)
        except TypeError:  # older torch without the flag
            super().__init__(params, **kw)
            for g in self.param_groups:
                g["decoupled_weight_decay"] = decoupled_weight_decay
        self._pdrnn_grad_scale = grad_scale
        self._flat_state = {}

    # -- flat state -------------------------------------------------------
    def materialize_state(self) -> None:
        """Allocate (zero) the flat moment buffers of every group now instead
        of inside the first step; no parameter or step count changes."""
        with torch.no_grad():
            for gi, g in enumerate(self.param_groups):
                self._group_flat(gi, g)

    def _group_flat(self, gi: int, group) -> Optional[dict]:
        params: List[Tensor] = [p for p in group["params"]]
        if not params:
            return None
        cached = self._flat_state.get(gi)
        if cached is not None and cached["n_params"] == len(params) and \
                cached["param_ptr"] == params[0].data_ptr():
            return cached
        span = contiguous_span([p.data for p in params])
        if span is None:
            return None
        flat_p = span[0]
        n = flat_p.numel()
        # optimizer moments as flat buffers; per-param state entries are views
        exp_avg = torch.zeros(n, dtype=flat_p.dtype, device=flat_p.device)
        exp_avg_sq = torch.zeros_like(exp_avg)
        max_sq = torch.zeros_like(exp_avg) if group["amsgrad"] else None
        off = 0
        step0 = None
        for p in params:
            k = p.numel()
            st = self.state[p]
            if "exp_avg" in st:  # migrate pre-existing (e.g. loaded) state
                exp_avg[off:off + k].copy_(st["exp_avg"].reshape(-1))
                exp_avg_sq[off:off + k].copy_(st["exp_avg_sq"].reshape(-1))
                if max_sq is not None and "max_exp_avg_sq" in st:
                    max_sq[off:off + k].copy_(st["max_exp_avg_sq"].reshape(-1))
                step0 = float(st["step"]) if step0 is None else step0
            st["exp_avg"] = exp_avg[off:off + k].view_as(p)
            st["exp_avg_sq"] = exp_avg_sq[off:off + k].view_as(p)
            if max_sq is not None:
                st["max_exp_avg_sq"] = max_sq[off:off + k].view_as(p)
            off += k
        step_t = torch.tensor(step0 or 0.0, dtype=torch.float32)
        for p in params:
            self.state[p]["step"] = step_t
        cached = dict(n_params=len(params), param_ptr=params[0].data_ptr(), flat_p=flat_p,
                      exp_avg=exp_avg, exp_avg_sq=exp_avg_sq, max_sq=max_sq, step=step_t)
        self._flat_state[gi] = cached
        return cached

    @torch.no_grad()
    def step(self, closure=None, skip: Optional[Tensor] = None):
        """``skip``: device int32 word read by the native launch -- nonzero at
        run time leaves parameters and moments untouched (the step count still
        advances on the host: :meth:`rewind` takes such steps back)."""
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for gi, group in enumerate(self.param_groups):
            params = group["params"]
            if not params:
                continue
            dev = params[0].device
            mod = _ext.native(dev)
            if mod is None or params[0].dtype != torch.float32:
                if skip is not None and bool(skip.item()):
                    continue
                self._reference_group_step(group)
                continue
            fs = self._group_flat(gi, group)
            grads = [p.grad if p.grad is not None else torch.zeros_like(p) for p in params]
            gspan = contiguous_span(grads)
            if fs is None:
                if skip is not None and bool(skip.item()):
                    continue
                self._reference_group_step(group)
                continue
            gflat = gspan[0] if gspan is not None else torch.cat([g.reshape(-1) for g in grads])
            beta1, beta2 = group["betas"]
            fs["step"] += 1.0
            step = float(fs["step"])
            mod.adam_flat(fs["flat_p"], gflat, fs["exp_avg"], fs["exp_avg_sq"], fs["max_sq"],
                          float(group["lr"]), beta1, beta2, group["eps"], group["weight_decay"],
                          step, self._pdrnn_grad_scale, bool(group.get("decoupled_weight_decay", False)),
                          bool(group.get("maximize", False)), None, None, None, skip)
            self.native_steps = getattr(self, "native_steps", 0) + 1  # groups stepped by the native kernel
            # the native kernel wrote the parameters through raw pointers: move
            # their version counters like any in-place torch update would, so
            # derived copies keyed on versions (16-bit shadow weights of the
            # large-H LSTM, ops/lstm_large.py) see the change
            for p in params:
                torch.autograd.graph.increment_version(p)
        return loss

    def rewind(self, steps: int) -> None:
        """Take ``steps`` native steps back from the step count (steps whose
        launch was skipped on the device, see :meth:`step`)."""
        for fs in self._flat_state.values():
            fs["step"] -= float(steps)

    def _reference_group_step(self, group):
        # torch's own Adam for this group only (CPU path / unsupported layout).
        # Un-share the flat path's common step counter first: torch increments
        # every parameter's step tensor separately.
        for p in group["params"]:
            st = self.state.get(p)
            if st and "step" in st:
                st["step"] = st["step"].clone()
        self._flat_state = {}
        saved = self.param_groups
        self.param_groups = [group]
        try:
            if self._pdrnn_grad_scale != 1.0:
                for p in group["params"]:
                    if p.grad is not None:
                        p.grad.mul_(self._pdrnn_grad_scale)
            super().step()
        finally:
            self.param_groups = saved

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._flat_state = {}  # rebuilt (and state migrated) on the next step

    def zero_grad(self, set_to_none: bool = True):
        # Flat gradient buffers must survive zero_grad: zero in place.
        flat_groups = []
        for group in self.param_groups:
            grads = [p.grad for p in group["params"] if p.grad is not None]
            span = contiguous_span(grads) if len(grads) == len(group["params"]) else None
            if span is not None:
                span[0].zero_()
                flat_groups.append(group)
        if len(flat_groups) != len(self.param_groups):
            remaining = [g for g in self.param_groups if g not in flat_groups]
            saved = self.param_groups
            self.param_groups = remaining
            try:
                super().zero_grad(set_to_none=set_to_none)
            finally:
                self.param_groups = saved
