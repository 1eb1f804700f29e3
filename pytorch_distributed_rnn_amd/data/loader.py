"""Samplers and device-resident batch loaders.

The reference feeds each rank through ``DataLoader(dataset, batch_size,
sampler=DistributedSampler(...))`` (reference: src/motion/trainer/base.py:22-31,
45-60; src/motion/trainer/distributed.py:35-49).  The invariance oracle of the
reference (per-step mean loss identical for 1/2/4/8/12 ranks)
depends on the sampler's exact semantics, which are reproduced here:

* permutation = ``torch.randperm(N, generator=manual_seed(seed + epoch))``,
* padded by wrap-around to a multiple of ``num_replicas``,
* rank ``r`` takes ``indices[r::num_replicas]``,
* batches are consecutive slices of the rank's index list (last one short).

:class:`DeviceBatchLoader` keeps the whole dataset in HBM (the motion training
set is 32 MB) and yields batches gathered on the device: no host collation, no
H2D copy per step.
"""
from __future__ import annotations

import math
from typing import Iterator, List, Optional, Tuple

import torch
from torch import Tensor


class ShardedSampler(torch.utils.data.Sampler):
    """``torch.utils.data.DistributedSampler``-compatible shuffled shard."""

    def __init__(self, dataset_len: int, num_replicas: int = 1, rank: int = 0, shuffle: bool = True,
                 seed: int = 0, drop_last: bool = False):
        if rank < 0 or rank >= num_replicas:
            raise ValueError(f"rank {rank} out of range for {num_replicas} replicas")
        self.n = dataset_len
        self.num_replicas = num_replicas
        self.rank = rank
        self.shuffle = shuffle
        self.seed = seed
        self.drop_last = drop_last
        self.epoch = 0
        if drop_last and self.n % num_replicas:
            self.num_samples = math.ceil((self.n - num_replicas) / num_replicas)
        else:
            self.num_samples = math.ceil(self.n / num_replicas)
        self.total_size = self.num_samples * num_replicas

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch

    def index_tensor(self, epoch: Optional[int] = None) -> Tensor:
        """This rank's indices of the current epoch (or of ``epoch``) as an
        int64 CPU tensor (the same values as :meth:`indices`, built with
        tensor ops: no Python list of N ints on the per-epoch path)."""
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + (self.epoch if epoch is None else epoch))
            idx = torch.randperm(self.n, generator=g)
        else:
            idx = torch.arange(self.n)
        if not self.drop_last:
            pad = self.total_size - idx.numel()
            if pad > 0:
                reps = math.ceil(pad / idx.numel())
                idx = torch.cat([idx, idx.repeat(reps)[:pad]])
        else:
            idx = idx[:self.total_size]
        return idx[self.rank:self.total_size:self.num_replicas]

    def indices(self) -> List[int]:
        return self.index_tensor().tolist()

    def __iter__(self) -> Iterator[int]:
        return iter(self.indices())

    def __len__(self) -> int:
        return self.num_samples


class DeviceBatchLoader:
    """DataLoader-equivalent over device-resident ``features``/``labels``.

    ``len(loader)`` is the number of batches and ``loader.dataset`` the
    underlying dataset, like ``torch.utils.data.DataLoader``.  Iteration yields
    ``(x, y)`` already on ``device``.  With ``gather_in_kernel=True`` it yields
    ``(features, labels, idx)`` -- the full device tables plus the batch's row
    indices -- so models that accept an index (the fused LSTM gathers rows
    inside the kernel) skip the gather copy."""

    def __init__(self, dataset, batch_size: Optional[int], sampler: Optional[ShardedSampler] = None,
                 device: Optional[torch.device] = None, gather_in_kernel: bool = False,
                 feature_dtype: Optional[torch.dtype] = None):
        self.dataset = dataset
        self.device = torch.device(device) if device is not None else dataset.features.device
        self.features = dataset.features.to(self.device, dtype=feature_dtype)
        self.labels = dataset.labels.to(self.device)
        self.sampler = sampler
        n = len(sampler) if sampler is not None else len(dataset)
        self.batch_size = batch_size if batch_size is not None else n
        if self.batch_size <= 0:
            raise ValueError("batch size must be positive (global batch smaller than world size?)")
        self.num_items = n
        self.gather_in_kernel = gather_in_kernel

    def __len__(self) -> int:
        return math.ceil(self.num_items / self.batch_size)

    def prefetch(self, epoch: Optional[int] = None) -> None:
        """Build the batch indices of sampler epoch ``epoch`` (default: the
        sampler's current one) now -- the trainer calls it while the GPU still
        runs the previous epoch's steps, so the next epoch's first launch does
        not wait for the host permutation and its copy (a DataLoader
        prefetch).  Consumed by the next :meth:`batch_indices` of that epoch."""
        if self.sampler is None:
            return
        e = self.sampler.epoch if epoch is None else epoch
        self._prefetched = (e, self._build_indices(self.sampler.index_tensor(e)))

    def batch_indices(self) -> List[Tensor]:
        """This epoch's per-batch row indices, on the device.  The host
        permutation goes through a persistent pinned staging buffer with an
        asynchronous copy (a pageable-memory copy would be synchronous)."""
        pre = getattr(self, "_prefetched", None)
        if pre is not None and self.sampler is not None and pre[0] == self.sampler.epoch:
            self._prefetched = None
            return pre[1]
        if self.sampler is not None:
            idx = self.sampler.index_tensor()
        else:
            idx = torch.arange(self.num_items)
        return self._build_indices(idx)

    def _build_indices(self, idx: Tensor) -> List[Tensor]:
        if self.device.type == "cuda":
            stage = getattr(self, "_pinned", None)
            if stage is None or stage.numel() < idx.numel():
                stage = self._pinned = torch.empty(idx.numel(), dtype=torch.long, pin_memory=True)
                self._pinned_ev = None
            if self._pinned_ev is not None:
                self._pinned_ev.synchronize()  # the previous epoch's copy out of the buffer is done
            stage = stage[:idx.numel()]
            stage.copy_(idx)
            idx = stage.to(self.device, non_blocking=True)
            self._pinned_ev = torch.cuda.Event()
            self._pinned_ev.record()
        else:
            idx = idx.to(self.device)
        return list(torch.split(idx, self.batch_size))

    def make_batch(self, bidx: Tensor):
        """(x, y) gathered batch, or -- in in-kernel gather mode -- the
        (features, labels, idx) triple: full device tables + this batch's rows."""
        if self.gather_in_kernel:
            return self.features, self.labels, bidx
        return self.features.index_select(0, bidx), self.labels.index_select(0, bidx)

    def __iter__(self):
        for bidx in self.batch_indices():
            yield self.make_batch(bidx)
