"""Distributed runtime: torchrun ``env://`` bootstrap, backend selection, seeding, scalar reductions.

Reference behaviour:
* ``is_distributed()`` is ``WORLD_SIZE > 1``, re-read on every call (reference ``train_ddp.py:49-50``).
* ``setup_distributed()`` returns ``(0, 1, 0)`` when not distributed, else reads
  ``WORLD_SIZE/RANK/LOCAL_RANK`` and initialises the process group (``train_ddp.py:53-68``).
* ``set_seed(seed, rank)`` seeds ``seed + rank`` (``train_ddp.py:76-78``).
* ``reduce_tensor`` is an in-place SUM all-reduce, identity when single-process (``:159-167``).

Differences by design: the reference hard-codes ``backend="nccl"``
(``train_ddp.py:65``) so it cannot run multi-process without GPUs.  Here the backend is
``auto``: RCCL (torch's ``"nccl"`` backend *is* RCCL on ROCm) when a GPU is visible, gloo
otherwise.  The device is bound *before* the process group is created so RCCL's
communicator is created on the right GPU and eagerly (``device_id=``), and an explicit
timeout is configurable.
"""
from __future__ import annotations

import datetime
import os
import random
from dataclasses import dataclass
from typing import Optional, Tuple

import torch
import torch.distributed as dist


def is_distributed() -> bool:
    return int(os.environ.get("WORLD_SIZE", "1")) > 1


def gpu_available() -> bool:
    return torch.cuda.is_available()


def resolve_backend(backend: str = "auto") -> str:
    """Map the CLI backend name to a torch.distributed backend string."""
    if backend in ("rccl", "nccl"):
        return "nccl"
    if backend == "gloo":
        return "gloo"
    return "nccl" if gpu_available() else "gloo"


@dataclass
class DistInfo:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    backend: str = "none"
    device: torch.device = torch.device("cpu")

    @property
    def distributed(self) -> bool:
        return self.world_size > 1

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def setup_distributed(backend: str = "auto", timeout_s: int = 1800) -> Tuple[int, int, int]:
    """Reference-compatible signature: returns ``(rank, world_size, local_rank)``."""
    info = init_distributed(backend, timeout_s)
    return info.rank, info.world_size, info.local_rank


def init_distributed(backend: str = "auto", timeout_s: int = 1800, shared_gpu: bool = False) -> DistInfo:
    """``shared_gpu`` (testing, ``--rehearse-shared-gpu``): every rank on cuda:0 over a gloo group."""
    if shared_gpu and is_distributed():
        if not gpu_available():
            raise RuntimeError("--rehearse-shared-gpu needs a visible GPU")
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        if not dist.is_initialized():
            dist.init_process_group(backend="gloo", init_method="env://",
                                    timeout=datetime.timedelta(seconds=timeout_s))
        return DistInfo(int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"]),
                        int(os.environ.get("LOCAL_RANK", "0")), "gloo", dev)
    if not is_distributed():
        dev = torch.device("cuda:0") if gpu_available() else torch.device("cpu")
        if dev.type == "cuda":
            torch.cuda.set_device(dev)
        return DistInfo(0, 1, 0, "none", dev)

    world_size = int(os.environ["WORLD_SIZE"])
    rank = int(os.environ["RANK"])
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    be = resolve_backend(backend)
    kw = {}
    if be == "nccl":
        if not gpu_available():
            raise RuntimeError("backend rccl requested but no GPU is visible")
        dev = torch.device(f"cuda:{local_rank}")
        torch.cuda.set_device(dev)
        kw["device_id"] = dev
    else:
        dev = torch.device(f"cuda:{local_rank}") if (gpu_available() and backend == "auto") else torch.device("cpu")
        if dev.type == "cuda":
            torch.cuda.set_device(dev)
    if not dist.is_initialized():
        dist.init_process_group(backend=be, init_method="env://",
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
    return DistInfo(rank, world_size, local_rank, be, dev)


def cleanup_distributed() -> None:
    if is_distributed() and dist.is_initialized():
        dist.destroy_process_group()


def set_seed(seed: int, rank: int) -> None:
    torch.manual_seed(seed + rank)
    random.seed(seed + rank)
    if gpu_available():
        torch.cuda.manual_seed_all(seed + rank)


def reduce_tensor(tensor: torch.Tensor, op=dist.ReduceOp.SUM) -> torch.Tensor:
    if not is_distributed():
        return tensor
    dist.all_reduce(tensor, op=op)
    return tensor


def all_reduce_(tensor: torch.Tensor, op=dist.ReduceOp.SUM) -> torch.Tensor:
    """In-place all-reduce that never hands a GPU tensor to gloo: with a gloo process group
    (CPU runs, or ranks sharing one GPU) a device tensor is reduced through a host copy -
    gloo's own CUDA path is not relied on (it returned wrong sums in this environment)."""
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return tensor
    if tensor.is_cuda and dist.get_backend() == "gloo":
        host = tensor.detach().cpu()
        dist.all_reduce(host, op=op)
        tensor.copy_(host)
    else:
        dist.all_reduce(tensor, op=op)
    return tensor


def barrier() -> None:
    if is_distributed() and dist.is_initialized():
        dist.barrier()


def broadcast_object(obj, src: int = 0):
    if not (is_distributed() and dist.is_initialized()):
        return obj
    box = [obj]
    dist.broadcast_object_list(box, src=src)
    return box[0]


def world_max(value: float, device: Optional[torch.device] = None) -> float:
    """MAX over ranks of a host float (used for step-time reporting)."""
    if not (is_distributed() and dist.is_initialized()):
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device or torch.device("cpu"))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
