from .fused import FusedAdam, FusedSGD, build_optimizer

__all__ = ["FusedAdam", "FusedSGD", "build_optimizer"]
