"""Mixed precision: autocast policy + device-resident GradScaler."""
from __future__ import annotations

import contextlib

import torch

from .grad_scaler import DeviceGradScaler

_DTYPES = {"fp16": torch.float16, "bf16": torch.bfloat16}


def autocast(device: torch.device, enabled: bool, dtype: str = "fp16"):
    """``torch.autocast`` for the device type (the reference uses the deprecated
    ``torch.cuda.amp.autocast()`` = fp16, reference train_ddp.py:204)."""
    if not enabled:
        return contextlib.nullcontext()
    return torch.autocast(device_type=torch.device(device).type, dtype=_DTYPES[dtype])


__all__ = ["DeviceGradScaler", "autocast"]
