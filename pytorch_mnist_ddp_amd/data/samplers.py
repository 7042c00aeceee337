"""Index streams bit-identical to torch's samplers, produced as whole-epoch tensors.

The reference drives data order with ``DistributedSampler(shuffle=True)`` when
distributed, ``RandomSampler`` otherwise, and ``SequentialSampler`` for the test
set (``mnist_ddp.py:161-165``); ``mnist.py`` uses ``shuffle=True`` (a
RandomSampler) only on CUDA (``mnist.py:103-110``).  The device-resident
pipeline needs the epoch's full index vector up front (uploaded once per epoch
and gathered on-device), so these classes return an int64 tensor per epoch
instead of a Python iterator, with exactly the same values and the same global
RNG consumption as torch:

* DistributedSampler (``torch/utils/data/distributed.py``): generator seeded
  with ``seed + epoch``; ``randperm(N)``; pad by wrapping to
  ``ceil(N/W)*W``; shard ``[rank::W]``.
* RandomSampler (``torch/utils/data/sampler.py``): draws one int64 seed from the
  *global* CPU RNG per epoch, then ``randperm`` on a fresh generator.
* DataLoader: every ``iter(loader)`` first draws one int64 "base seed" from the
  global CPU RNG (``_BaseDataLoaderIter.__init__``), *before* the sampler's
  draw.  :func:`consume_loader_base_seed` reproduces that so the shuffle order
  of the non-distributed path matches the reference epoch for epoch.
"""
from __future__ import annotations

import math

import torch


def consume_loader_base_seed() -> int:
    """Emulate the DataLoader iterator's base-seed draw from the global RNG."""
    return int(torch.empty((), dtype=torch.int64).random_().item())


class SequentialIndexStream:
    def __init__(self, n: int):
        self.n = n

    def __len__(self) -> int:
        return self.n

    def epoch_indices(self) -> torch.Tensor:
        return torch.arange(self.n, dtype=torch.int64)


class RandomIndexStream:
    """RandomSampler(data_source) without replacement, default num_samples."""

    def __init__(self, n: int):
        self.n = n

    def __len__(self) -> int:
        return self.n

    def epoch_indices(self) -> torch.Tensor:
        seed = int(torch.empty((), dtype=torch.int64).random_().item())
        g = torch.Generator()
        g.manual_seed(seed)
        return torch.randperm(self.n, generator=g)


class DistributedIndexStream:
    """DistributedSampler(dataset, num_replicas, rank, shuffle, seed=0, drop_last=False)."""

    def __init__(self, n: int, num_replicas: int, rank: int, shuffle: bool = True,
                 seed: int = 0, drop_last: bool = False):
        if not 0 <= rank < num_replicas:
            raise ValueError(f"Invalid rank {rank}, rank should be in [0, {num_replicas - 1}]")
        self.n, self.num_replicas, self.rank = n, num_replicas, rank
        self.shuffle, self.seed, self.drop_last = shuffle, seed, drop_last
        self.epoch = 0
        if drop_last and n % num_replicas != 0:
            self.num_samples = math.ceil((n - num_replicas) / num_replicas)
        else:
            self.num_samples = math.ceil(n / num_replicas)
        self.total_size = self.num_samples * num_replicas

    def __len__(self) -> int:
        return self.num_samples

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch

    def epoch_indices(self) -> torch.Tensor:
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            idx = torch.randperm(self.n, generator=g)
        else:
            idx = torch.arange(self.n, dtype=torch.int64)
        if not self.drop_last:
            pad = self.total_size - self.n
            if pad > 0:
                reps = math.ceil(pad / self.n)
                idx = torch.cat([idx, idx.repeat(reps)[:pad]]) if pad > self.n else torch.cat([idx, idx[:pad]])
        else:
            idx = idx[: self.total_size]
        out = idx[self.rank: self.total_size: self.num_replicas]
        assert out.numel() == self.num_samples
        return out


def num_batches(num_samples: int, batch_size: int, drop_last: bool = False) -> int:
    return num_samples // batch_size if drop_last else math.ceil(num_samples / batch_size)
