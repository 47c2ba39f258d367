"""Rank-sharded sampler (``torch.utils.data.distributed.DistributedSampler`` semantics,
used at mnist_distributed.py:73-75).

Defaults match torch: ``shuffle=True, seed=0, drop_last=False``; the
permutation is ``randperm(n, generator=seed+epoch)``, padded by wrapping to a
multiple of ``num_replicas``, and rank ``r`` takes ``indices[r::W]``.  Unlike
the reference we expose (and our trainers call) ``set_epoch`` — the reference
never does, so every epoch reuses one permutation.
"""
from __future__ import annotations

import math
from typing import Iterator, Optional

import torch


class DistributedSampler:
    def __init__(self, dataset_len: int, num_replicas: Optional[int] = None, rank: Optional[int] = None,
                 shuffle: bool = True, seed: int = 0, drop_last: bool = False):
        from . import distributed as tdist

        if num_replicas is None:
            num_replicas = tdist.get_world_size()
        if rank is None:
            rank = tdist.get_rank()
        if not 0 <= rank < num_replicas:
            raise ValueError(f"Invalid rank {rank}, rank should be in the interval [0, {num_replicas - 1}]")
        if hasattr(dataset_len, "__len__"):
            dataset_len = len(dataset_len)
        self.n = int(dataset_len)
        self.num_replicas, self.rank = num_replicas, rank
        self.shuffle, self.seed, self.drop_last = shuffle, seed, drop_last
        self.epoch = 0
        if drop_last and self.n % num_replicas != 0:
            self.num_samples = math.ceil((self.n - num_replicas) / num_replicas)
        else:
            self.num_samples = math.ceil(self.n / num_replicas)
        self.total_size = self.num_samples * num_replicas

    def __iter__(self) -> Iterator[int]:
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            indices = torch.randperm(self.n, generator=g).tolist()
        else:
            indices = list(range(self.n))
        if not self.drop_last:
            pad = self.total_size - len(indices)
            if pad <= len(indices):
                indices += indices[:pad]
            else:
                indices += (indices * math.ceil(pad / len(indices)))[:pad]
        else:
            indices = indices[: self.total_size]
        assert len(indices) == self.total_size
        return iter(indices[self.rank: self.total_size: self.num_replicas])

    def __len__(self) -> int:
        return self.num_samples

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch
