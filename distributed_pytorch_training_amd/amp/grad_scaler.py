"""Device-resident dynamic loss scaler.

Same state machine and defaults as the ``torch.cuda.amp.GradScaler(enabled=args.amp)`` the
reference constructs (reference train_ddp.py:346; torch/amp/grad_scaler.py:126-129,
529-536): init_scale 2**16, growth_factor 2, backoff_factor 0.5, growth_interval 2000,
skip the optimizer step on non-finite gradients, back off, grow after ``growth_interval``
clean steps.

What changes is *where* it runs.  torch's ``scaler.step`` does ``found_inf.item()``
(torch/amp/grad_scaler.py:356): one host sync per step.  Here ``scale``,
``growth_tracker`` and ``found_inf`` live on the device; the non-finite check is fused
into the reducer's per-bucket post-all-reduce pass (or one ``grad_check`` launch when
there is no reducer), the fused optimizer kernel reads the flag and skips itself, and a
one-thread tail kernel updates the scale - no host synchronisation at all.

``state_dict`` uses torch's keys (``scale``, ``growth_factor``, ``backoff_factor``,
``growth_interval``, ``_growth_tracker``; torch/amp/grad_scaler.py:607-630) so checkpoints
are interchangeable with torch's GradScaler.
"""
from __future__ import annotations

from typing import Any, Dict, Optional

import torch


class DeviceGradScaler:
    def __init__(self, device: torch.device, init_scale: float = 2.0 ** 16,
                 growth_factor: float = 2.0, backoff_factor: float = 0.5,
                 growth_interval: int = 2000, enabled: bool = True) -> None:
        if growth_factor <= 1.0 or not 0.0 < backoff_factor < 1.0:
            raise ValueError("growth_factor must be > 1 and backoff_factor in (0, 1)")
        self.device = torch.device(device)
        self._enabled = enabled
        self._init_scale = init_scale
        self.growth_factor = growth_factor
        self.backoff_factor = backoff_factor
        self.growth_interval = growth_interval
        self._scale = torch.full((1,), init_scale, dtype=torch.float32, device=self.device)
        self._growth_tracker = torch.zeros(1, dtype=torch.int32, device=self.device)
        # Written by the reducer / grad_check, read by the optimizer, cleared by the tail.
        self.found_inf = torch.zeros(1, dtype=torch.float32, device=self.device)

    # -- torch.amp.GradScaler-compatible surface ------------------------------------------
    def is_enabled(self) -> bool:
        return self._enabled

    def scale(self, loss: torch.Tensor) -> torch.Tensor:
        if not self._enabled:
            return loss
        return loss * self._scale.to(dtype=loss.dtype).reshape(())

    @property
    def scale_tensor(self) -> Optional[torch.Tensor]:
        """Device scale (None when disabled) - what the kernels read."""
        return self._scale if self._enabled else None

    @property
    def growth_tracker(self) -> Optional[torch.Tensor]:
        return self._growth_tracker if self._enabled else None

    def get_scale(self) -> float:
        """Host copy of the scale (synchronises; logging/checkpoint only)."""
        return float(self._scale.item()) if self._enabled else 1.0

    def get_growth_tracker(self) -> int:
        return int(self._growth_tracker.item()) if self._enabled else 0

    def state_dict(self) -> Dict[str, Any]:
        if not self._enabled:
            return {}
        return {"scale": self.get_scale(), "growth_factor": self.growth_factor,
                "backoff_factor": self.backoff_factor, "growth_interval": self.growth_interval,
                "_growth_tracker": self.get_growth_tracker()}

    def load_state_dict(self, state: Dict[str, Any]) -> None:
        if not self._enabled:
            return
        if len(state) == 0:
            raise RuntimeError("The source state dict is empty, possibly because it was saved "
                               "from a disabled instance of GradScaler.")
        self._scale.fill_(float(state["scale"]))
        self.growth_factor = float(state["growth_factor"])
        self.backoff_factor = float(state["backoff_factor"])
        self.growth_interval = int(state["growth_interval"])
        self._growth_tracker.fill_(int(state["_growth_tracker"]))
