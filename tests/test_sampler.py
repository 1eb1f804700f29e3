"""ShardedSampler == torch DistributedSampler (reference: base.py:22-26,
distributed.py:35-39): the permutation semantics the invariance oracle needs."""
import pytest
import torch
from torch.utils.data import DistributedSampler

from pytorch_distributed_rnn_amd.data.loader import ShardedSampler


class _Len:
    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n


@pytest.mark.parametrize("n,world", [(96, 1), (96, 2), (96, 4), (100, 3), (6912, 8)])
@pytest.mark.parametrize("shuffle", [True, False])
def test_matches_distributed_sampler(n, world, shuffle):
    for epoch in (0, 3):
        for rank in range(world):
            ref = DistributedSampler(_Len(n), num_replicas=world, rank=rank, shuffle=shuffle, seed=0)
            ref.set_epoch(epoch)
            ours = ShardedSampler(n, num_replicas=world, rank=rank, shuffle=shuffle)
            ours.set_epoch(epoch)
            assert list(ours) == list(ref)
            assert len(ours) == len(ref)


def test_union_of_shards_is_single_process_batch_order():
    n, world = 96, 4
    single = list(ShardedSampler(n))
    shards = [list(ShardedSampler(n, world, r)) for r in range(world)]
    # rank r holds perm[r::world]: interleaving restores the single-process order
    inter = [shards[i % world][i // world] for i in range(n)]
    assert inter == single


def test_bad_rank():
    with pytest.raises(ValueError):
        ShardedSampler(10, num_replicas=2, rank=2)
