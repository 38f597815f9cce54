"""Checkpoint / resume (extension; the reference writes no checkpoint).

Format: one ``torch.save`` file written by rank 0 holding plain PyTorch objects only:
  * ``model``     - the unwrapped ``state_dict`` with torchvision key names
                    (``conv1.weight``, ``layer1.0.bn1.running_mean``, ...);
  * ``optimizer`` - torch.optim-layout ``state_dict`` (SGD ``momentum_buffer`` / Adam
                    ``exp_avg``/``exp_avg_sq``/``step`` per parameter index);
  * ``scaler``    - torch GradScaler keys (``scale``, ``growth_factor``, ``backoff_factor``,
                    ``growth_interval``, ``_growth_tracker``);
  * ``epoch``, ``args``, ``format``.
Flat-arena internals are mapped back to per-parameter tensors, so the file loads into stock
torch models/optimizers, and it loads with ``weights_only=True`` (nothing executable).
"""
from __future__ import annotations

import os
import tempfile
from typing import Any, Dict, Optional

import torch

FORMAT = "dpt-amd-ckpt-v1"


def _plain_args(args) -> Dict[str, Any]:
    out = {}
    for k, v in vars(args).items():
        if isinstance(v, (int, float, str, bool)) or v is None:
            out[k] = v
        elif isinstance(v, (tuple, list)) and all(isinstance(x, (int, float, str, bool)) for x in v):
            out[k] = list(v)
    return out


def save_checkpoint(path: str, trainer, epoch: int, args) -> None:
    state = {
        "format": FORMAT,
        "epoch": epoch,
        "model": {k: v.detach().cpu() for k, v in trainer.model_state().items()},
        "optimizer": _to_cpu(trainer.optimizer_state()),
        "scaler": trainer.scaler_state(),
        "args": _plain_args(args),
    }
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    fd, tmp = tempfile.mkstemp(dir=d, suffix=".tmp")
    os.close(fd)
    torch.save(state, tmp)
    os.replace(tmp, path)  # atomic: a crash never leaves a half-written checkpoint


def _to_cpu(obj):
    if isinstance(obj, torch.Tensor):
        return obj.detach().cpu()
    if isinstance(obj, dict):
        return {k: _to_cpu(v) for k, v in obj.items()}
    if isinstance(obj, list):
        return [_to_cpu(v) for v in obj]
    if isinstance(obj, tuple):
        return tuple(_to_cpu(v) for v in obj)
    return obj


def load_checkpoint(path: str, trainer, map_location: Optional[str] = "cpu") -> int:
    """Restore model/optimizer/scaler; returns the epoch to resume from."""
    state = torch.load(path, map_location=map_location, weights_only=True)
    trainer.module.load_state_dict(state["model"])
    trainer.optimizer.load_state_dict(state["optimizer"])
    if state.get("scaler"):
        trainer.scaler.load_state_dict(state["scaler"])
    if hasattr(trainer, "sync_weights"):
        trainer.sync_weights()
    return int(state["epoch"])
