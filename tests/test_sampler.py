"""ShardSampler == torch.utils.data.DistributedSampler (imagenet.py:346-347,375)."""

import pytest
import torch
from torch.utils.data.distributed import DistributedSampler

from imagent_amd.parallel.sampler import ShardSampler


class _DS:
    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n


@pytest.mark.parametrize("n,world", [(1001, 4), (50000, 16), (7, 3), (5, 8), (1281167 // 97, 16)])
@pytest.mark.parametrize("shuffle", [True, False])
@pytest.mark.parametrize("drop_last", [False, True])
def test_matches_torch(n, world, shuffle, drop_last):
    for epoch in (0, 3):
        for rank in range(world):
            ref = DistributedSampler(_DS(n), num_replicas=world, rank=rank, shuffle=shuffle, seed=0,
                                     drop_last=drop_last)
            ref.set_epoch(epoch)
            ours = ShardSampler(n, world, rank, shuffle=shuffle, seed=0, drop_last=drop_last)
            ours.set_epoch(epoch)
            assert list(ours) == list(ref)
            assert len(ours) == len(ref)


def test_imagenet_padding_numbers():
    s = ShardSampler(1281167, 16, 0)
    assert s.total_size == 1281168 and s.num_samples == 80073
    v = ShardSampler(50000, 16, 0)
    assert v.num_samples == 3125
    assert s.num_batches(128) == 626                              # 626 steps/epoch


def test_batches_partition_the_shard():
    s = ShardSampler(1000, 3, 1, shuffle=True, seed=5)
    bs = list(s.batches(64))
    assert torch.cat(bs).tolist() == list(s)
    assert all(len(b) == 64 for b in bs[:-1])
