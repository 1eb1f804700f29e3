"""Module-wrapping synchronous data parallelism (DDP).

Replaces ``torch.nn.parallel.DistributedDataParallel`` over ProcessGroupMPI
as used by the reference (reference: src/motion/trainer/ddp.py:18-19,
src/example/example_ddp.py:46):

* at wrap time the module's parameters are re-homed into one flat buffer
  (``utils.flat``) and broadcast from rank 0 in ONE collective (+ buffers);
* gradients land in a flat buffer whose contiguous slices are the all-reduce
  buckets of the native :class:`GradReducer` (csrc/runtime/reducer.cpp);
* a post-accumulate-grad hook per parameter marks readiness; full buckets
  are all-reduced (RCCL ``ncclAvg`` over xGMI on the communicator's own
  stream) while the backward continues; a callback queued on the autograd
  engine finalises at the end of backward;
* ``state_dict`` keys carry the ``module.`` prefix exactly like torch DDP
  (checkpoint compatibility, SURVEY.md §5 "Checkpoint").

Bucket size: the first bucket is small so communication starts as soon as the
top layers' gradients exist; later buckets default to 32 MiB -- on an 8-GPU
xGMI mesh that puts >= 4 MiB on each of the 7 peer links per ring step, well
past the latency-bound regime (see docs/DESIGN.md, "Bucket sizing").
"""
from __future__ import annotations

import contextlib
import logging
import os
import re
from typing import Dict, List, Optional

import torch
import torch.distributed as dist
from torch import nn

from .. import _ext
from ..utils.flat import FlatParameters
from ..utils.tracing import trace_range
from .comm import get_comm

DEFAULT_BUCKET_MB = float(os.environ.get("PDRNN_BUCKET_MB", 32))
DEFAULT_FIRST_BUCKET_MB = float(os.environ.get("PDRNN_FIRST_BUCKET_MB", 1))


_RNN_PARAM = re.compile(r"^(?P<base>.*_l\d+)(?P<rev>_reverse)?$")


def param_group_ids(module: nn.Module, params) -> List[int]:
    """One id per (RNN layer, direction) -- ``weight_ih_l1_reverse`` and
    ``bias_hh_l1_reverse`` share one, ``*_l1`` another -- and per owning
    module for everything else (head, embedding).  Ids are consecutive in
    registration order, so a bucket boundary falls on every layer-direction
    boundary (buckets aligned to the weights a BPTT layer
    finishes together)."""
    names = {id(p): n for n, p in module.named_parameters()}
    keys: Dict[str, int] = {}
    out = []
    for p in params:
        n = names.get(id(p), f"<unnamed {len(out)}>")
        mod_path, _, leaf = n.rpartition(".")
        m = _RNN_PARAM.match(leaf)
        key = f"{mod_path}:{m.group('base').split('_')[-1]}{m.group('rev') or ''}" if m else mod_path
        out.append(keys.setdefault(key, len(keys)))
    return out


def format_bucket_layout(layout) -> str:
    def one(b):
        sl = f" elements {b['slice'][0]}:{b['slice'][1]}" if "slice" in b else ""
        return f"#{b['bucket']} {b['mib']:.2f} MiB {b['params']} params [{', '.join(b['names'])}]{sl}"
    return "; ".join(one(b) for b in layout)


class _PyReducer:
    """Python twin of the native reducer (used only without the extension)."""

    def __init__(self, params, comm, flat_grad):
        self.params, self.comm, self.flat_grad = params, comm, flat_grad
        self._views = []
        off = 0
        for p in params:
            self._views.append(flat_grad[off:off + p.numel()].view_as(p))
            off += p.numel()
        self.ready = [False] * len(params)
        self.launched = 0

    def grad_views(self):
        return self._views

    def mark_ready(self, i, grad):
        repoint = False
        if grad is not None and grad.data_ptr() != self._views[i].data_ptr():
            self._views[i].copy_(grad)
            repoint = True
        self.ready[i] = True
        return repoint

    def finalize(self):
        op = "avg" if self.comm.native_avg else "sum"
        self.comm.all_reduce(self.flat_grad, op)
        self.comm.wait()
        if not self.comm.native_avg and self.comm.world > 1:
            self.flat_grad.div_(self.comm.world)
        self.ready = [False] * len(self.params)

    def reset(self):
        self.ready = [False] * len(self.params)

    def all_reduce_now(self):
        self.finalize()

    all_reduce_inline = all_reduce_now


class DistributedDataParallel(nn.Module):
    def __init__(self, module: nn.Module, device_ids=None, output_device=None,
                 process_group=None, bucket_cap_mb: Optional[float] = None,
                 first_bucket_cap_mb: Optional[float] = None, broadcast_buffers: bool = True,
                 find_unused_parameters: bool = False, average: bool = True):
        super().__init__()
        if not dist.is_initialized():
            raise RuntimeError("call parallel.init_distributed() before wrapping with DDP")
        self.module = module
        self.process_group = process_group
        self.broadcast_buffers = broadcast_buffers
        self.find_unused_parameters = find_unused_parameters
        self.require_backward_grad_sync = True
        params = [p for p in module.parameters() if p.requires_grad]
        flat_groups = getattr(module, "_pdrnn_flat", None)
        if flat_groups and len(flat_groups) == 1:
            self.flat = next(iter(flat_groups.values()))
        else:
            self.flat = FlatParameters(params)
            module._pdrnn_flat = {(params[0].device, params[0].dtype): self.flat}
        self._pdrnn_flat = module._pdrnn_flat
        self.comm = get_comm(process_group)
        self.world_size = self.comm.world
        self.rank = self.comm.rank
        self._sync_params_and_buffers()
        cap = int((bucket_cap_mb if bucket_cap_mb is not None else DEFAULT_BUCKET_MB) * 2 ** 20)
        first = int((first_bucket_cap_mb if first_bucket_cap_mb is not None
                     else DEFAULT_FIRST_BUCKET_MB) * 2 ** 20)
        mod = _ext.extension()
        self.param_groups_ids = param_group_ids(module, self.flat.params)
        if mod is not None:
            self.reducer = mod.GradReducer(self.flat.params, self.comm, cap, first, average,
                                           self.flat.grad, self.param_groups_ids)
        else:
            self.reducer = _PyReducer(self.flat.params, self.comm, self.flat.grad)
        if self.rank == 0:
            logging.info("DDP buckets (launch order): " + format_bucket_layout(self.bucket_layout()))
        self._views = list(self.reducer.grad_views())
        for p, v in zip(self.flat.params, self._views):
            p.grad = v
        self._finalize_queued = False
        self._hooks = [p.register_post_accumulate_grad_hook(self._make_hook(i))
                       for i, p in enumerate(self.flat.params)]

    def bucket_layout(self) -> List[Dict]:
        """Buckets in launch order: size, parameter count and names."""
        names = {id(p): n for n, p in self.module.named_parameters()}
        if not hasattr(self.reducer, "bucket_indices"):  # python twin: one flat bucket
            idx = [list(range(len(self.flat.params) - 1, -1, -1))]
        else:
            idx = [list(b) for b in self.reducer.bucket_indices()]
        # (offset, length) of a bucket that is a slice of one oversized parameter
        chunks = list(self.reducer.bucket_chunks()) if hasattr(self.reducer, "bucket_chunks") else \
            [(-1, 0)] * len(idx)
        out = []
        for b, ids in enumerate(idx):
            ps = [self.flat.params[i] for i in ids]
            off, length = chunks[b]
            nbytes = length * ps[0].element_size() if off >= 0 else sum(p.numel() * p.element_size() for p in ps)
            ent = {"bucket": b, "params": len(ps), "mib": nbytes / 2 ** 20,
                   "names": [names.get(id(p), "?") for p in ps]}
            if off >= 0:
                ent["slice"] = [int(off), int(off + length)]
            out.append(ent)
        return out

    # -------------------------------------------------------------- sync
    @torch.no_grad()
    def _sync_params_and_buffers(self):
        if self.world_size == 1:
            return
        self.comm.broadcast(self.flat.data, 0)
        if self.broadcast_buffers:
            for b in self.module.buffers():
                if b.is_floating_point() or b.dtype in (torch.long, torch.int):
                    self.comm.broadcast(b.data if b.is_contiguous() else b.data.contiguous(), 0)
        self.comm.wait()

    def _make_hook(self, i: int):
        def hook(p):
            if not self.require_backward_grad_sync:
                return
            if not self._finalize_queued:
                self._finalize_queued = True
                torch.autograd.Variable._execution_engine.queue_callback(self._finalize)
            if self.reducer.mark_ready(i, p.grad):
                p.grad = self._views[i]
        return hook

    def _finalize(self):
        self._finalize_queued = False
        with trace_range("pdrnn.grad_allreduce"):
            self.reducer.finalize()

    # -------------------------------------------------------------- api
    def forward(self, *args, **kwargs):
        return self.module(*args, **kwargs)

    @contextlib.contextmanager
    def no_sync(self):
        old = self.require_backward_grad_sync
        self.require_backward_grad_sync = False
        try:
            yield
        finally:
            self.require_backward_grad_sync = old

