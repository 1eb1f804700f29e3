"""The autograd training step replayed from one HIP graph per batch shape.

Models outside the fused motion step (``train/fused_step.py``) train through
autograd: forward, fused cross-entropy, ``loss.backward()`` and the native
:class:`~pytorch_distributed_rnn_amd.ops.adam.FusedAdam`.  At the fp32
``--hidden-units 128`` shape (reference src/motion/main.py:20-21,
src/motion/trainer/base.py:111-118) that step is ~80 launches issued from
Python on two streams, and the host's issue gaps between the small glue
kernels (gathers, shadow-weight refreshes, gradient accumulation) sit on the
critical path.  Captured once, a step is one ``hipGraphLaunch``:

* the zero-fill of the flat gradient, the whole forward / backward (including
  the stacked-layer pipeline's side streams, which fork from and join the
  capture stream) and the Adam launch are graph nodes;
* the batch indices are read from a static device buffer (one copy per step);
* Adam takes its step count from a device counter that the kernel itself
  advances (``adam_flat``'s arrival ticket), shared by every captured batch
  shape so the full and the short last batch of an epoch stay in sequence;
  the host mirror of the count advances per replay (``state_dict`` parity);
* derived weight copies keyed on parameter versions (the large-H LSTM's
  shadow weights, ``ops/lstm_large.py:shadow``) are forced stale before the
  capture, so their refresh is recorded in the graph, and the parameters'
  version counters are moved after every replay for eager users.

Only single-process training with index batches on the GPU and a
single-group FusedAdam (the flat-buffer path) is captured; anything else, or
a capture that fails, keeps the eager step.

Opt-in (``cuda_graph=True`` / ``--cuda-graph`` / ``PDRNN_CUDA_GRAPH=1``):
measured slower at the fp32 H = 128 shape it was built for -- 5.37 against
3.82 ms/step (LSTM), 5.58 against 3.78 (GRU), profiles/r5/graphed/.  The host
gaps do go away, but the replayed graph spreads the stacked-layer pipeline
over three hardware queues without the side stream's priority, and the
90-workgroup recurrences then share the CUs with the weight-gradient GEMMs
(one BPTT chunk 245 -> 478 us in the replay's timeline).
"""
from __future__ import annotations

import logging
import os
from typing import Optional

import torch


def supported(trainer) -> bool:
    from ..ops.adam import FusedAdam
    if not (trainer.cuda_graph is True or os.environ.get("PDRNN_CUDA_GRAPH", "") == "1"):
        return False
    if trainer.device.type != "cuda" or trainer.world_size() != 1:
        return False
    opt = trainer.optimizer
    if type(opt) is not FusedAdam or len(opt.param_groups) != 1:
        return False
    g = opt.param_groups[0]
    if g.get("amsgrad") or not callable(getattr(g["lr"], "__float__", None)):
        return False
    return getattr(trainer.train_loader, "gather_in_kernel", False)


class GraphedAutogradStep:
    """Callable (features, labels_all, idx) -> (stats [loss, n, correct], n)."""

    def __init__(self, trainer):
        self.tr = trainer
        self.entries = {}
        self.step_t: Optional[torch.Tensor] = None
        self.ticket: Optional[torch.Tensor] = None
        self.replays = 0

    def _flat(self):
        opt = self.tr.optimizer
        fs = opt._group_flat(0, opt.param_groups[0])
        params = opt.param_groups[0]["params"]
        from ..utils.flat import contiguous_span
        gspan = contiguous_span([p.grad for p in params]) if all(p.grad is not None for p in params) else None
        return fs, params, (gspan[0] if gspan is not None else None)

    def _eager_pass(self, features, labels_all, idx):
        """forward + loss + backward (no update): allocations, lazy kernel
        loads and cached operand layouts happen outside the capture."""
        tr = self.tr
        tr.optimizer.zero_grad()
        out, labels = tr._forward((features, labels_all, idx))
        loss = tr.loss_fn(out, labels.long().reshape(-1))
        loss.backward()

    def _capture(self, features, labels_all, idx):
        tr = self.tr
        dev = idx.device
        sidx = idx.clone()
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            self._eager_pass(features, labels_all, sidx)
        torch.cuda.current_stream(dev).wait_stream(side)
        fs, params, gflat = self._flat()
        if fs is None or gflat is None:
            raise RuntimeError("graphed step: flat parameter / gradient buffers expected")
        if self.step_t is None:
            self.step_t = torch.full((1,), float(fs["step"]), dtype=torch.float32, device=dev)
            self.ticket = torch.zeros(1, dtype=torch.int32, device=dev)
        from .. import _ext
        mod = _ext.native(dev)
        group = tr.optimizer.param_groups[0]
        b1, b2 = group["betas"]
        # derived copies of the weights (shadow layouts) must be refreshed by
        # the graph itself: make every cached copy stale now
        for p in params:
            torch.autograd.graph.increment_version(p)
        torch.cuda.synchronize(dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            tr.optimizer.zero_grad()
            out, labels = tr._forward((features, labels_all, sidx))
            loss = tr.loss_fn(out, labels.long().reshape(-1))
            stats = tr.loss_fn.last_stats
            loss.backward()
            mod.adam_flat(fs["flat_p"], gflat, fs["exp_avg"], fs["exp_avg_sq"], None, float(group["lr"]), b1, b2,
                          group["eps"], group["weight_decay"], 1.0, tr.optimizer._pdrnn_grad_scale,
                          bool(group.get("decoupled_weight_decay", False)), bool(group.get("maximize", False)),
                          None, self.step_t, self.ticket)
        ent = dict(graph=g, idx=sidx, stats=stats, lr=float(group["lr"]), feats=features, labels=labels_all)
        return ent

    def __call__(self, features, labels_all, idx):
        key = (features.data_ptr(), labels_all.data_ptr(), idx.numel(), idx.device)
        ent = self.entries.get(key)
        lr = float(self.tr.optimizer.param_groups[0]["lr"])
        if ent is not None and ent["lr"] != lr:  # hyper-parameters are baked into the graph
            self.entries.clear()
            ent = None
        if ent is None:
            ent = self.entries[key] = self._capture(features, labels_all, idx)
        ent["idx"].copy_(idx)
        ent["graph"].replay()
        self.replays += 1
        opt = self.tr.optimizer
        fs = opt._flat_state.get(0)
        if fs is not None:
            fs["step"] += 1.0  # host mirror of the device count
        opt.native_steps = getattr(opt, "native_steps", 0) + 1
        for p in opt.param_groups[0]["params"]:
            torch.autograd.graph.increment_version(p)
        return ent["stats"].clone(), idx.numel()


def make(trainer) -> Optional[GraphedAutogradStep]:
    try:
        return GraphedAutogradStep(trainer) if supported(trainer) else None
    except Exception as e:  # pragma: no cover - defensive
        logging.warning("graphed step unavailable: %s", e)
        return None
