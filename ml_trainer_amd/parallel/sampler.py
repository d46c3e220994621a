"""Data sharding with ``torch.utils.data.DistributedSampler`` semantics.

The reference shards the training set with ``DistributedSampler(train_set,
num_replicas=W, rank=r)`` (``src/trainer.py:60-61``): seeded permutation
(``seed + epoch``), padded by wrapping to a multiple of W, then
``indices[rank::W]``. :func:`shard_indices` reproduces that partition exactly
(same generator, same padding) as a flat index array, so it can be uploaded
to the device once per epoch for the HBM-resident input path.

Fix vs. the reference: the Trainer calls ``set_epoch`` every
epoch, so the order changes between epochs.
"""
from __future__ import annotations

import math
from typing import Iterator, List, Optional

import torch


def shard_indices(n: int, world: int, rank: int, shuffle: bool = True, seed: int = 0, epoch: int = 0,
                  drop_last: bool = False) -> List[int]:
    if n <= 0:
        return []
    if shuffle:
        g = torch.Generator()
        g.manual_seed(seed + epoch)
        indices = torch.randperm(n, generator=g).tolist()
    else:
        indices = list(range(n))
    if drop_last and n % world != 0:
        num_samples = math.ceil((n - world) / world)
    else:
        num_samples = math.ceil(n / world)
    total = num_samples * world
    if not drop_last:
        pad = total - len(indices)
        if pad <= len(indices):
            indices += indices[:pad]
        else:
            indices += (indices * math.ceil(pad / len(indices)))[:pad]
    else:
        indices = indices[:total]
    return indices[rank:total:world]


class ShardSampler(torch.utils.data.Sampler):
    """Drop-in for DistributedSampler (same partition), usable without an
    initialised process group (explicit ``num_replicas``/``rank``)."""

    def __init__(self, dataset, num_replicas: Optional[int] = None, rank: Optional[int] = None,
                 shuffle: bool = True, seed: int = 0, drop_last: bool = False):
        if num_replicas is None or rank is None:
            import torch.distributed as dist
            num_replicas = dist.get_world_size() if num_replicas is None else num_replicas
            rank = dist.get_rank() if rank is None else rank
        if rank < 0 or rank >= num_replicas:
            raise ValueError(f"invalid rank {rank} for {num_replicas} replicas")
        self.dataset = dataset
        self.num_replicas = num_replicas
        self.rank = rank
        self.shuffle = shuffle
        self.seed = seed
        self.drop_last = drop_last
        self.epoch = 0
        n = len(dataset)
        if drop_last and n % num_replicas != 0:
            self.num_samples = math.ceil((n - num_replicas) / num_replicas)
        else:
            self.num_samples = math.ceil(n / num_replicas)
        self.total_size = self.num_samples * num_replicas

    def indices(self) -> List[int]:
        return shard_indices(len(self.dataset), self.num_replicas, self.rank, self.shuffle, self.seed, self.epoch,
                             self.drop_last)

    def __iter__(self) -> Iterator[int]:
        return iter(self.indices())

    def __len__(self) -> int:
        return self.num_samples

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch
