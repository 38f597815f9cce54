# train_ddp.py
"""Single-script entry point (same name, flags and outputs as the reference's train_ddp.py).

    torchrun --nproc_per_node=N train_ddp.py [--epochs 10 --batch-size 128 --amp ...]

Launch contract: torchrun's env:// variables (WORLD_SIZE, RANK, LOCAL_RANK, MASTER_ADDR,
MASTER_PORT), one process per GPU.  Everything underneath is the MI355X-native stack in
``distributed_pytorch_training_amd`` (see README.md); ``--impl torch`` runs the stock
PyTorch DDP mechanics of the reference for comparison.
"""
import sys

from distributed_pytorch_training_amd.engine.run import main

if __name__ == "__main__":
    sys.exit(main())
