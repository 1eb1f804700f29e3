"""Rank-aware trainers: DistributedTrainer (shared policy), DDPTrainer
(module-wrapping all-reduce) and HorovodTrainer (optimizer-wrapping fused
all-reduce).

Policy parity with the reference (reference: src/motion/trainer/distributed.py:7-62,
ddp.py:7-36, horovod.py:6-42):

* only rank 0 evaluates and checkpoints;
* the training set is sharded with DistributedSampler semantics (rank r takes
  ``perm[r::world]``);
* strong scaling: the per-rank batch is ``batch_size // world_size`` so the
  union of the rank batches at step s is exactly the single-process batch --
  which makes the per-step mean loss identical at every world size (the
  reference's implicit correctness oracle);
* log prefix carries the rank.

``weak_scaling=True`` keeps ``batch_size`` per rank instead (extension used by
the weak-scaling benchmark).
"""
from __future__ import annotations

import logging
import os
from typing import Optional

import torch
from torch import nn

from ..data.loader import ShardedSampler
from ..parallel import env
from ..parallel import horovod as hvd
from ..parallel.ddp import DistributedDataParallel
from .formatter import TrainingMessageFormatter
from .trainer import Trainer


class DistributedTrainer(Trainer):
    def __init__(self, model, training_set, batch_size, learning_rate, rank, world_size,
                 validation_set=None, test_set=None, checkpoint_dir=None, *,
                 weak_scaling: bool = False, **kwargs):
        if rank != 0:
            validation_set = None
            test_set = None
        self.rank = rank
        self._world_size = world_size
        self.weak_scaling = weak_scaling
        if not weak_scaling and batch_size is not None and batch_size % world_size:
            logging.warning("global batch %d is not divisible by world size %d: per-rank batch is "
                            "floored (world-size invariance of the loss no longer holds)",
                            batch_size, world_size)
        super().__init__(model=model, training_set=training_set, validation_set=validation_set,
                         test_set=test_set, batch_size=batch_size, learning_rate=learning_rate,
                         checkpoint_dir=checkpoint_dir,
                         sampler=ShardedSampler(len(training_set), num_replicas=world_size, rank=rank),
                         **kwargs)

    def world_size(self) -> int:
        return self._world_size

    def _get_data_loader(self, dataset, batch_size=None, sampler=None):
        if batch_size is not None and not self.weak_scaling:
            batch_size = batch_size // self._world_size
        return super()._get_data_loader(dataset, batch_size=batch_size, sampler=sampler)

    def _get_formatter(self, epochs: int) -> TrainingMessageFormatter:
        return TrainingMessageFormatter(epochs, self.rank)

    def _save_checkpoint(self, epoch, loss, best=False):
        if self.rank == 0:
            return super()._save_checkpoint(epoch, loss, best=best)
        return None


class DDPTrainer(DistributedTrainer):
    """Synchronous DP with the native bucketed reducer (RCCL over xGMI)."""

    def __init__(self, model, training_set, batch_size, learning_rate, validation_set=None,
                 test_set=None, checkpoint_dir=None, *, backend: Optional[str] = None,
                 bucket_cap_mb: Optional[float] = None, **kwargs):
        env.init_distributed(backend)
        device = kwargs.pop("device", None) or self._device()
        model = model.to(device)
        model = DistributedDataParallel(model, bucket_cap_mb=bucket_cap_mb)
        super().__init__(rank=env.get_rank(), world_size=env.get_world_size(), model=model,
                         training_set=training_set, validation_set=validation_set, test_set=test_set,
                         batch_size=batch_size, learning_rate=learning_rate,
                         checkpoint_dir=checkpoint_dir, device=device, **kwargs)

    def _grad_sync(self):
        # the fused step has nothing to overlap the all-reduce with (every
        # gradient comes out of one reduction kernel): reduce inline on the
        # compute stream.  PDRNN_FORCE_GRAD_SYNC=1 keeps the sync at world 1
        # (diagnostic: the multi-GPU step's launch sequence on one GPU).
        reducer = self.model.reducer
        if self._world_size == 1 and os.environ.get("PDRNN_FORCE_GRAD_SYNC", "0") != "1":
            return None
        return reducer.all_reduce_inline

    def _grad_comm(self):
        return self.model.comm

    @staticmethod
    def _device() -> torch.device:
        if torch.cuda.is_available() and torch.distributed.get_backend() == "nccl":
            return torch.device("cuda", torch.cuda.current_device())
        return torch.device("cpu")

    def _reset_hidden_state(self):
        inner = self.model.module
        if hasattr(inner, "reset_hidden_state"):
            inner.reset_hidden_state()


class HorovodTrainer(DistributedTrainer):
    """Optimizer-wrapping DP: per-tensor hooks + tensor fusion + synchronize."""

    def __init__(self, model, training_set, batch_size, learning_rate, validation_set=None,
                 test_set=None, checkpoint_dir=None, *, backend: Optional[str] = None, **kwargs):
        hvd.init(backend)
        device = kwargs.pop("device", None) or DDPTrainer._device()
        super().__init__(rank=hvd.rank(), world_size=hvd.size(), model=model.to(device),
                         training_set=training_set, validation_set=validation_set, test_set=test_set,
                         batch_size=batch_size, learning_rate=learning_rate,
                         checkpoint_dir=checkpoint_dir, device=device, **kwargs)

    def _get_optimizer(self, model: nn.Module, lr: float):
        optimizer = super()._get_optimizer(model, lr)
        return hvd.DistributedOptimizer(optimizer, named_parameters=model.named_parameters())

    def _grad_sync(self):
        if self._world_size == 1 and os.environ.get("PDRNN_FORCE_GRAD_SYNC", "0") != "1":
            return None
        flat = next(iter(getattr(self.model, "_pdrnn_flat").values()))
        # the fused step bypasses the per-tensor hooks: one fused all-reduce of
        # the whole flat gradient (= Horovod's fusion buffer holding every tensor)
        return lambda: hvd.allreduce_(flat.grad, average=True)

    def _grad_comm(self):
        return hvd.comm() if self._world_size > 1 or os.environ.get("PDRNN_FORCE_GRAD_SYNC", "0") == "1" else None

    def train(self, epochs: int):
        hvd.broadcast_parameters(self.model.state_dict(), root_rank=0)
        return super().train(epochs)
