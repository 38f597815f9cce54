"""Device-resident data loaders.

The reference's input pipeline is 4 DataLoader worker processes per rank doing PIL/CPU
augmentation, a pin-memory thread and a per-step H2D copy (reference train_ddp.py:131-148,
198-199).  On MI355X the whole CIFAR-10 train split is 150 MiB of
uint8 - nothing next to 288 GB of HBM - so it is uploaded once and every batch is
produced on the GPU: gather by sampler index + random crop + flip + normalise in one HIP
kernel (``ops.augment``), output already in the model's memory format.  No worker
processes, no pinned staging, no per-step H2D copy.

``SyntheticLoader`` is the benchmark input: a small pool of random ImageNet-shape batches
generated on the device once and cycled (the GPU box has no network / no dataset).
Both loaders honour the reference's step-count semantics: ``len = ceil(samples / batch)``
with a short last batch (``drop_last=False``).
"""
from __future__ import annotations

import math
from typing import Optional, Sequence

import torch

from .. import ops


class DeviceImageLoader:
    def __init__(self, images: torch.Tensor, labels: torch.Tensor, sampler, batch_size: int,
                 device: torch.device, augment: bool, mean: Sequence[float], std: Sequence[float],
                 pad: int = 4, channels_last: bool = False, out_dtype: torch.dtype = torch.float32,
                 max_steps: int = 0) -> None:
        if images.dtype != torch.uint8 or images.dim() != 4:
            raise ValueError("images must be uint8 [N, C, H, W]")
        self.device = torch.device(device)
        self.images = images.to(self.device).contiguous()
        self.labels = labels.to(self.device, torch.int64)
        self.sampler, self.batch_size = sampler, batch_size
        self.augment, self.pad = augment, pad
        self.mean, self.std = tuple(mean), tuple(std)
        self.channels_last, self.out_dtype = channels_last, out_dtype
        self.max_steps = max_steps

    def set_epoch(self, epoch: int) -> None:
        self.sampler.set_epoch(epoch)

    def __len__(self) -> int:
        n = math.ceil(len(self.sampler) / self.batch_size)
        return min(n, self.max_steps) if self.max_steps else n

    def __iter__(self):
        idx = self.sampler.indices().to(self.device)
        _, c, h, w = self.images.shape
        for step in range(len(self)):
            bidx = idx[step * self.batch_size:(step + 1) * self.batch_size]
            b = bidx.numel()
            if self.augment:
                offs = torch.randint(0, 2 * self.pad + 1, (b, 2), dtype=torch.int32, device=self.device)
                flips = torch.randint(0, 2, (b,), dtype=torch.uint8, device=self.device)
            else:
                offs = flips = None
            mf = torch.channels_last if self.channels_last else torch.contiguous_format
            out = torch.empty((b, c, h, w), dtype=self.out_dtype, device=self.device, memory_format=mf)
            ops.augment(self.images, bidx, offs, flips, out, nhwc=self.channels_last, pad=self.pad,
                        mean=self.mean, std=self.std)
            yield out, self.labels.index_select(0, bidx)


def class_prototypes(num_classes: int, image_size: int, device, seed: int = 1234) -> torch.Tensor:
    """Fixed per-class mean images of the learnable synthetic task: smooth random fields
    (upsampled 4x4 noise, unit variance), the same for every rank, split and engine."""
    g = torch.Generator(device="cpu")
    g.manual_seed(seed)
    low = torch.randn((num_classes, 3, 4, 4), generator=g)
    up = torch.nn.functional.interpolate(low, size=(image_size, image_size), mode="bilinear", align_corners=False)
    up = up / up.flatten(1).std(dim=1).clamp_min(1e-6).view(-1, 1, 1, 1)
    return up.to(device)


class SyntheticLoader:
    """On-device synthetic batches.

    ``task="random"`` (benchmarks): a pool of ``pool`` random batches with random labels, cycled -
    the model can only memorise it.  ``task="prototypes"`` (training-outcome checks): every sample
    is its class prototype (``class_prototypes``) plus ``noise`` x N(0, 1) pixel noise, drawn
    fresh for every batch from a generator seeded by (seed, epoch, step) - the same data for any
    engine, and a held-out split (another seed) that is learnable and measures generalisation."""

    def __init__(self, num_samples: int, batch_size: int, image_size: int, num_classes: int,
                 device: torch.device, channels_last: bool = False, pool: int = 4,
                 dtype: torch.dtype = torch.float32, seed: int = 0, max_steps: int = 0,
                 task: str = "random", noise: float = 2.0) -> None:
        self.num_samples, self.batch_size = num_samples, batch_size
        self.device = torch.device(device)
        self.max_steps = max_steps
        self.task, self.noise, self.seed, self.epoch = task, float(noise), seed, 0
        self.dtype, self.num_classes, self.image_size = dtype, num_classes, image_size
        self.mf = torch.channels_last if channels_last else torch.contiguous_format
        self.pool_x, self.pool_y = [], []
        if task == "prototypes":
            self.protos = class_prototypes(num_classes, image_size, self.device)
            return
        if task != "random":
            raise ValueError(f"unknown synthetic task {task!r}")
        g = torch.Generator(device=self.device)
        g.manual_seed(seed)
        mf = self.mf
        for _ in range(max(1, pool)):
            x = torch.randn((batch_size, 3, image_size, image_size), generator=g, device=self.device,
                            dtype=torch.float32).to(dtype)
            self.pool_x.append(x.contiguous(memory_format=mf))
            self.pool_y.append(torch.randint(0, num_classes, (batch_size,), generator=g,
                                             device=self.device, dtype=torch.int64))

    def set_epoch(self, epoch: int) -> None:
        self.epoch = int(epoch)

    def __len__(self) -> int:
        n = math.ceil(self.num_samples / self.batch_size)
        return min(n, self.max_steps) if self.max_steps else n

    def _prototype_batch(self, step: int, b: int):
        g = torch.Generator(device=self.device)
        g.manual_seed((self.seed * 1_000_003 + self.epoch * 10_007 + step) & 0x7FFFFFFF)
        y = torch.randint(0, self.num_classes, (b,), generator=g, device=self.device, dtype=torch.int64)
        x = torch.randn((b, 3, self.image_size, self.image_size), generator=g, device=self.device)
        x = (self.protos.index_select(0, y) + self.noise * x).to(self.dtype)
        return x.contiguous(memory_format=self.mf), y

    def __iter__(self):
        n = len(self)
        for step in range(n):
            if self.task == "prototypes":
                yield self._prototype_batch(step, min(self.batch_size, self.num_samples - step * self.batch_size))
                continue
            k = step % len(self.pool_x)
            b = min(self.batch_size, self.num_samples - step * self.batch_size)
            if b == self.batch_size:
                yield self.pool_x[k], self.pool_y[k]
            else:
                yield self.pool_x[k][:b], self.pool_y[k][:b]
