"""Rank-sharding sampler with ``torch.utils.data.DistributedSampler`` semantics.

The reference builds ``DistributedSampler(trainset)`` / ``(valset)`` with the
defaults ``shuffle=True, seed=0, drop_last=False`` (``imagenet.py:346-347``)
and calls ``set_epoch(epoch)`` on the train sampler only (``imagenet.py:375``;
quirk Q2: the val sampler therefore shuffles with the epoch-0 permutation
every epoch).

Semantics reproduced exactly ([torch] ``utils/data/distributed.py``):
permutation = ``torch.randperm(n, generator seeded seed+epoch)``; pad by
wrapping to a multiple of the world size (1,281,167 -> 1,281,168); rank r takes
``indices[r::world]``. Indices are produced as an int64 tensor (no Python list
of 1.28 M ints) and can be chunked into batches without leaving torch.
"""

from __future__ import annotations

import math
from typing import Iterator, Optional

import torch


class ShardSampler:
    def __init__(self, num_items: int, num_replicas: int = 1, rank: int = 0,
                 shuffle: bool = True, seed: int = 0, drop_last: bool = False):
        if num_replicas < 1 or not (0 <= rank < num_replicas):
            raise ValueError(f"invalid rank {rank} for world size {num_replicas}")
        self.n = int(num_items)
        self.num_replicas = num_replicas
        self.rank = rank
        self.shuffle = shuffle
        self.seed = seed
        self.drop_last = drop_last
        self.epoch = 0
        if drop_last and self.n % num_replicas != 0:
            self.num_samples = math.ceil((self.n - num_replicas) / num_replicas)
        else:
            self.num_samples = math.ceil(self.n / num_replicas)
        self.total_size = self.num_samples * num_replicas

    def set_epoch(self, epoch: int) -> None:
        self.epoch = int(epoch)

    def indices(self) -> torch.Tensor:
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            idx = torch.randperm(self.n, generator=g)
        else:
            idx = torch.arange(self.n)
        if not self.drop_last:
            pad = self.total_size - idx.numel()
            if pad > 0:
                reps = math.ceil(pad / idx.numel())
                idx = torch.cat([idx, idx.repeat(reps)[:pad]])
        else:
            idx = idx[: self.total_size]
        assert idx.numel() == self.total_size
        idx = idx[self.rank: self.total_size: self.num_replicas]
        assert idx.numel() == self.num_samples
        return idx

    def __iter__(self) -> Iterator[int]:
        return iter(self.indices().tolist())

    def __len__(self) -> int:
        return self.num_samples

    def batches(self, batch_size: int, drop_last: bool = False) -> Iterator[torch.Tensor]:
        """Yield index tensors of ``batch_size`` (DataLoader batching order)."""
        idx = self.indices()
        n = idx.numel()
        stop = (n // batch_size) * batch_size if drop_last else n
        for s in range(0, stop, batch_size):
            yield idx[s: s + batch_size]

    def num_batches(self, batch_size: int, drop_last: bool = False) -> int:
        return self.num_samples // batch_size if drop_last else math.ceil(self.num_samples / batch_size)
