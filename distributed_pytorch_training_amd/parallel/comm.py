"""Communicator bootstrap: the framework-owned RCCL communicator for the gradient hot path.

Control plane: torch's process group (``env://`` TCPStore rendezvous, reference
train_ddp.py:65) carries the 128-byte RCCL unique id from rank 0 to every rank.  Data
plane: the C++ ``RcclComm`` (csrc/rccl_comm.cpp) owns the communicator and a
high-priority HIP stream that the C++ reducer enqueues bucket all-reduces on.

On CPU (gloo) there is no RCCL; ``make_comm`` returns ``None`` and the reducer drives
``torch.distributed`` through a Python callback instead.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from .. import ops


def make_comm(device: torch.device, rank: int, world_size: int):
    """Create an RcclComm on ``device`` (GPU) or return None (CPU/gloo path)."""
    if device.type != "cuda":
        return None
    C = ops.native()
    if world_size > 1:
        if not dist.is_initialized():
            raise RuntimeError("make_comm needs an initialised torch.distributed process group")
        box = [C.RcclComm.new_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        uid = box[0]
    else:
        uid = C.RcclComm.new_unique_id()
    return C.RcclComm(uid, rank, world_size, device.index if device.index is not None else 0)


def broadcast_(tensor: torch.Tensor, comm, src: int = 0) -> None:
    """Broadcast on the current stream through the RCCL comm (GPU) or torch.distributed."""
    if comm is not None:
        comm.broadcast(tensor, src)
    elif dist.is_initialized() and dist.get_world_size() > 1:
        dist.broadcast(tensor, src)


def all_reduce_(tensor: torch.Tensor, comm=None) -> None:
    if comm is not None:
        comm.all_reduce(tensor, True)
    elif dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(tensor)
