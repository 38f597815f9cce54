from .dist import (DistInfo, barrier, broadcast_object, cleanup_distributed, init_distributed,
                   is_distributed, reduce_tensor, resolve_backend, set_seed, setup_distributed,
                   world_max)

__all__ = ["DistInfo", "barrier", "broadcast_object", "cleanup_distributed", "init_distributed",
           "is_distributed", "reduce_tensor", "resolve_backend", "set_seed", "setup_distributed",
           "world_max"]
