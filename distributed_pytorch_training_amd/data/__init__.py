"""Data pipeline: samplers with DistributedSampler semantics, CIFAR-10 readers, device loaders.

``get_dataloaders`` mirrors the reference's ``get_dataloaders(args, rank, world_size)``
(reference train_ddp.py:81-150): a sharded, shuffled train loader when distributed, a
shuffled one otherwise, and an UNSHARDED validation loader (every rank evaluates the whole
test split, as in the reference).
"""
from __future__ import annotations

import math

import torch

from ..utils.dist import barrier, is_distributed
from .cifar import MEAN, STD, find_cifar10, load_cifar10
from .loader import DeviceImageLoader, SyntheticLoader
from .sampler import RandomSampler, SequentialSampler, ShardedSampler


def get_dataloaders(args, rank: int, world_size: int, device: torch.device):
    """Returns ``(train_loader, val_loader, train_sampler)`` like the reference."""
    distributed = world_size > 1
    max_steps = getattr(args, "max_steps", 0)
    cl = getattr(args, "channels_last", False)
    if args.dataset == "synthetic":
        n_train = args.synthetic_train_size
        per_rank = math.ceil(n_train / world_size) if distributed else n_train
        task = getattr(args, "synthetic_task", "random")
        noise = getattr(args, "synthetic_noise", 2.0)
        train = SyntheticLoader(per_rank, args.batch_size, args.image_size, args.num_classes, device,
                                channels_last=cl, seed=args.seed + rank, max_steps=max_steps,
                                task=task, noise=noise)
        val = SyntheticLoader(args.synthetic_val_size, args.batch_size, args.image_size,
                              args.num_classes, device, channels_last=cl, seed=args.seed + 10_000,
                              pool=2, task=task, noise=noise)
        return train, val, None

    # CIFAR-10 from local files (rank 0 "downloads" = checks presence, then barrier).
    if rank == 0:
        find_cifar10(args.data_dir) or load_cifar10(args.data_dir, True)  # raises with a clear message
    if distributed or is_distributed():
        barrier()
    xtr, ytr = load_cifar10(args.data_dir, train=True)
    xte, yte = load_cifar10(args.data_dir, train=False)
    if distributed:
        train_sampler = ShardedSampler(len(xtr), world_size, rank, shuffle=True)
    else:
        train_sampler = None
    sampler = train_sampler if train_sampler is not None else RandomSampler(len(xtr))
    train = DeviceImageLoader(torch.from_numpy(xtr), torch.from_numpy(ytr), sampler, args.batch_size,
                              device, augment=True, mean=MEAN, std=STD, channels_last=cl,
                              max_steps=max_steps)
    val = DeviceImageLoader(torch.from_numpy(xte), torch.from_numpy(yte), SequentialSampler(len(xte)),
                            args.batch_size, device, augment=False, mean=MEAN, std=STD, channels_last=cl)
    return train, val, train_sampler


__all__ = ["get_dataloaders", "DeviceImageLoader", "SyntheticLoader", "ShardedSampler",
           "RandomSampler", "SequentialSampler", "load_cifar10", "find_cifar10", "MEAN", "STD"]
