"""Index samplers with the exact semantics the reference inherits.

* ``ShardedSampler`` == ``torch.utils.data.DistributedSampler(num_replicas, rank,
  shuffle=True, seed=0, drop_last=False)`` (reference train_ddp.py:121-127; SURVEY.md I5b;
  torch/utils/data/distributed.py:98-134): permutation from a generator seeded
  ``seed + epoch``, padded by repeating indices up to ``ceil(N/ws)*ws``, strided shard
  ``indices[rank::ws]``.
* ``RandomSampler`` == the single-process ``DataLoader(shuffle=True)`` sampler: a fresh
  generator seeded from the global torch RNG each epoch.
* ``SequentialSampler`` == the validation loader order (shuffle=False).

They return index *tensors* (host int64) that the device loaders move to HBM once per
epoch: the batch gather then happens on the GPU, with no worker processes.
"""
from __future__ import annotations

import math

import torch


class ShardedSampler:
    def __init__(self, num_samples: int, num_replicas: int, rank: int, shuffle: bool = True,
                 seed: int = 0, drop_last: bool = False) -> None:
        if not 0 <= rank < num_replicas:
            raise ValueError(f"invalid rank {rank} for {num_replicas} replicas")
        self.dataset_len, self.num_replicas, self.rank = num_samples, num_replicas, rank
        self.shuffle, self.seed, self.drop_last, self.epoch = shuffle, seed, drop_last, 0
        if drop_last and num_samples % num_replicas != 0:
            self.num_samples = math.ceil((num_samples - num_replicas) / num_replicas)
        else:
            self.num_samples = math.ceil(num_samples / num_replicas)
        self.total_size = self.num_samples * num_replicas

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch

    def indices(self) -> torch.Tensor:
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            idx = torch.randperm(self.dataset_len, generator=g)
        else:
            idx = torch.arange(self.dataset_len)
        if not self.drop_last:
            pad = self.total_size - idx.numel()
            if pad > 0:
                if pad <= idx.numel():
                    idx = torch.cat([idx, idx[:pad]])
                else:
                    reps = math.ceil(pad / idx.numel())
                    idx = torch.cat([idx, idx.repeat(reps)[:pad]])
        else:
            idx = idx[:self.total_size]
        return idx[self.rank:self.total_size:self.num_replicas]

    def __iter__(self):
        return iter(self.indices().tolist())

    def __len__(self) -> int:
        return self.num_samples


class RandomSampler:
    def __init__(self, num_samples: int) -> None:
        self.num_samples = num_samples

    def set_epoch(self, epoch: int) -> None:  # torch's RandomSampler ignores epochs
        pass

    def indices(self) -> torch.Tensor:
        seed = int(torch.empty((), dtype=torch.int64).random_().item())
        g = torch.Generator()
        g.manual_seed(seed)
        return torch.randperm(self.num_samples, generator=g)

    def __len__(self) -> int:
        return self.num_samples


class SequentialSampler:
    def __init__(self, num_samples: int) -> None:
        self.num_samples = num_samples

    def set_epoch(self, epoch: int) -> None:
        pass

    def indices(self) -> torch.Tensor:
        return torch.arange(self.num_samples)

    def __len__(self) -> int:
        return self.num_samples
