"""Deterministic per-rank data sharding (reference: HF Trainer + accelerate shard the dataset
per DP rank with seed 42).  Epoch-seeded permutation, padded so every rank gets the
same number of samples, rank r takes indices r, r+W, r+2W, ...  ``skip`` resumes mid-epoch."""
from __future__ import annotations

from typing import Iterator

import torch


class ShardedSampler:
    def __init__(self, n: int, rank: int, world: int, seed: int = 42, shuffle: bool = True):
        self.n, self.rank, self.world, self.seed, self.shuffle = n, rank, world, seed, shuffle
        self.per_rank = (n + world - 1) // world

    def __len__(self):
        return self.per_rank

    def indices(self, epoch: int):
        if self.shuffle:
            g = torch.Generator().manual_seed(self.seed + epoch)
            perm = torch.randperm(self.n, generator=g).tolist()
        else:
            perm = list(range(self.n))
        total = self.per_rank * self.world
        perm = perm + perm[: total - self.n]
        return perm[self.rank:total:self.world]

    def iter(self, epoch: int, skip: int = 0) -> Iterator[int]:
        return iter(self.indices(epoch)[skip:])
