"""Horovod-compatible optimizer-wrapping data parallelism on the native runtime.

The reference's second strategy (reference: src/motion/trainer/horovod.py:17-42,
src/example/example_horovod.py:42-53,82) uses ``horovod.torch``: ``init``,
``rank``/``size``, ``broadcast_parameters(state_dict, root_rank)``,
``DistributedOptimizer(optimizer, named_parameters=...)``.  Horovod is not
part of this stack; this module provides the same API surface on the native
communicator (RCCL over xGMI on GPUs, gloo on the CPU):

* ``DistributedOptimizer`` returns an instance of a dynamic subclass of the
  wrapped optimizer's class (as Horovod does) that registers per-parameter
  gradient hooks; ready gradients are packed in canonical order into a
  tensor-fusion buffer (:class:`FusionReducer`, csrc/runtime/reducer.cpp) and
  all-reduced with averaging; ``step()`` first ``synchronize()``s.
* ``broadcast_parameters`` accepts a ``state_dict`` or ``named_parameters``
  iterable and broadcasts everything in one packed collective per dtype.

Unlike the module-wrapping DDP, the model is not wrapped, so ``state_dict``
keys have no ``module.`` prefix (checkpoint layout parity).
"""
from __future__ import annotations

import os
from typing import Dict, Iterable, List, Optional, Tuple, Union

import torch
import torch.distributed as dist

from .. import _ext
from . import env
from .comm import get_comm

FUSION_THRESHOLD = int(float(os.environ.get("HOROVOD_FUSION_THRESHOLD", 64 * 2 ** 20)))

Average = "avg"
Sum = "sum"


def init(backend: Optional[str] = None) -> None:
    env.init_distributed(backend)


def is_initialized() -> bool:
    return env.is_distributed()


def rank() -> int:
    return env.get_rank()


def size() -> int:
    return env.get_world_size()


def local_rank() -> int:
    return env.discover().local_rank


def local_size() -> int:
    return env.discover().local_world_size


def _comm():
    return get_comm(None)


def comm():
    """The native communicator Horovod mode runs on (the default group's)."""
    return _comm()


def _skip_world1() -> bool:
    # one rank: an in-place reduction is the identity -- unless
    # PDRNN_FORCE_COLLECTIVE=1 or PDRNN_FORCE_GRAD_SYNC=1 keeps it (the
    # communicator then really issues it: tests of the comm-stream hop and its
    # graph capture on one GPU; the multi-GPU step's launch sequence at world 1)
    return size() == 1 and os.environ.get("PDRNN_FORCE_COLLECTIVE", "0") != "1" and \
        os.environ.get("PDRNN_FORCE_GRAD_SYNC", "0") != "1"


def _tensors_of(params) -> List[Tuple[str, torch.Tensor]]:
    if isinstance(params, dict):
        return list(params.items())
    return list(params)


@torch.no_grad()
def broadcast_parameters(params: Union[Dict[str, torch.Tensor], Iterable[Tuple[str, torch.Tensor]]],
                         root_rank: int = 0) -> None:
    """Broadcast every tensor of ``params`` from ``root_rank`` in place."""
    items = [(k, t) for k, t in _tensors_of(params) if torch.is_tensor(t)]
    if size() == 1 or not items:
        return
    comm = _comm()
    groups: Dict[Tuple[torch.device, torch.dtype], List[torch.Tensor]] = {}
    for _, t in items:
        groups.setdefault((t.device, t.dtype), []).append(t)
    for (_dev, _dt), ts in groups.items():
        flat = torch.cat([t.detach().reshape(-1) for t in ts])
        comm.broadcast(flat, root_rank)
        comm.wait()
        off = 0
        for t in ts:
            n = t.numel()
            t.data.copy_(flat[off:off + n].view_as(t))
            off += n


@torch.no_grad()
def broadcast_optimizer_state(optimizer, root_rank: int = 0) -> None:
    state = []
    for group in optimizer.param_groups:
        for p in group["params"]:
            st = optimizer.state.get(p, {})
            for k in sorted(st):
                v = st[k]
                if torch.is_tensor(v) and v.is_floating_point():
                    state.append((k, v))
    broadcast_parameters(state, root_rank)


def allreduce(tensor: torch.Tensor, average: Optional[bool] = None, name: Optional[str] = None,
              op: Optional[str] = None) -> torch.Tensor:
    out = tensor.detach().clone().contiguous()
    allreduce_(out, average=average, op=op)
    return out


def allreduce_(tensor: torch.Tensor, average: Optional[bool] = None, name: Optional[str] = None,
               op: Optional[str] = None) -> torch.Tensor:
    if op is None:
        op = Average if average in (None, True) else Sum
    if _skip_world1():
        return tensor
    comm = _comm()
    if op == Average and not comm.native_avg:
        comm.all_reduce(tensor, "sum")
        comm.wait()
        tensor.div_(size())
    else:
        comm.all_reduce(tensor, op)
        comm.wait()
    return tensor


def allgather(tensor: torch.Tensor, name: Optional[str] = None) -> torch.Tensor:
    """Concatenate ``tensor`` from every rank along dim 0 (equal shapes)."""
    if size() == 1:
        return tensor.clone()
    t = tensor.contiguous()
    out = t.new_empty((size() * t.shape[0],) + tuple(t.shape[1:]))
    comm = _comm()
    comm.all_gather(out, t)
    comm.wait()
    return out


def broadcast(tensor: torch.Tensor, root_rank: int, name: Optional[str] = None) -> torch.Tensor:
    out = tensor.detach().clone().contiguous()
    if size() > 1:
        comm = _comm()
        comm.broadcast(out, root_rank)
        comm.wait()
    return out


class _DistributedOptimizerMixin:
    """Hook-driven fused all-reduce; mixed into the wrapped optimizer's class."""

    def _hvd_setup(self, named_parameters, fusion_threshold: int, op: str,
                   backward_passes_per_step: int):
        params = [p for g in self.param_groups for p in g["params"]]
        names = {}
        if named_parameters is not None:
            names = {id(p): n for n, p in named_parameters}
        self._hvd_params = [p for p in params if p.requires_grad]
        self._hvd_names = [names.get(id(p), f"param.{i}") for i, p in enumerate(self._hvd_params)]
        self._hvd_bpps = max(1, backward_passes_per_step)
        self._hvd_counts = [0] * len(self._hvd_params)
        self._hvd_world = size()
        self._hvd_sync_needed = False
        if self._hvd_world == 1:
            return
        comm = _comm()
        avg = op == Average
        mod = _ext.extension()
        self._hvd_fusion = mod.FusionReducer(comm, fusion_threshold, avg) if mod is not None else None
        self._hvd_comm = comm
        self._hvd_handles = []
        for i, (p, n) in enumerate(zip(self._hvd_params, self._hvd_names)):
            if self._hvd_fusion is not None:
                self._hvd_handles.append(self._hvd_fusion.register_tensor(n, p))
            p.register_post_accumulate_grad_hook(self._hvd_make_hook(i))

    def _hvd_make_hook(self, i: int):
        def hook(p):
            self._hvd_counts[i] += 1
            if self._hvd_counts[i] % self._hvd_bpps:
                return  # local accumulation (backward_passes_per_step)
            self._hvd_sync_needed = True
            if self._hvd_fusion is not None:
                self._hvd_fusion.enqueue(self._hvd_handles[i], p.grad)
        return hook

    def synchronize(self) -> None:
        if self._hvd_world == 1 or not self._hvd_sync_needed:
            return
        if self._hvd_fusion is not None:
            self._hvd_fusion.synchronize()
        else:
            for p in self._hvd_params:
                if p.grad is not None:
                    allreduce_(p.grad)
        self._hvd_sync_needed = False

    def step(self, closure=None):
        self.synchronize()
        return super().step(closure)


def DistributedOptimizer(optimizer, named_parameters=None, compression=None,
                         backward_passes_per_step: int = 1, op: str = Average,
                         fusion_threshold: Optional[int] = None):
    """Wrap ``optimizer`` (instance) Horovod-style; returns the wrapped instance."""
    cls = type(optimizer.__class__.__name__, (_DistributedOptimizerMixin, optimizer.__class__), {})
    wrapped = cls.__new__(cls)
    wrapped.__dict__.update(optimizer.__dict__)
    wrapped._hvd_setup(named_parameters, fusion_threshold or FUSION_THRESHOLD, op,
                       backward_passes_per_step)
    return wrapped
