"""Model zoo.  ``build_model`` is the factory the reference calls ``build_model(device)``
(reference ``train_ddp.py:153-156``), widened with the BASELINE.json model families."""
from __future__ import annotations

from typing import Callable, Dict

import torch
import torch.nn as nn

from .resnet import ResNet, resnet18, resnet34, resnet50, resnet101
from .vit import VisionTransformer, vit_b_16

MODELS: Dict[str, Callable[..., nn.Module]] = {
    "resnet18": resnet18,
    "resnet34": resnet34,
    "resnet50": resnet50,
    "resnet101": resnet101,
    "vit_b_16": vit_b_16,
}

# Expected parameter counts (torchvision parity).
PARAM_COUNTS = {
    ("resnet18", 10): 11_181_642,
    ("resnet18", 1000): 11_689_512,
    ("resnet50", 1000): 25_557_032,
    ("vit_b_16", 1000): 86_567_656,
}


def build_model(name: str = "resnet18", num_classes: int = 10, device=None,
                image_size: int = 224, channels_last: bool = False) -> nn.Module:
    if name not in MODELS:
        raise ValueError(f"unknown model {name!r}; choose from {sorted(MODELS)}")
    kw = {"image_size": image_size} if name.startswith("vit") else {}
    model = MODELS[name](num_classes=num_classes, **kw)
    if device is not None:
        model = model.to(device)
    if channels_last:
        model = model.to(memory_format=torch.channels_last)
    return model


def count_params(model: nn.Module) -> int:
    return sum(p.numel() for p in model.parameters())


__all__ = ["build_model", "count_params", "MODELS", "PARAM_COUNTS", "ResNet", "VisionTransformer",
           "resnet18", "resnet34", "resnet50", "resnet101", "vit_b_16"]
