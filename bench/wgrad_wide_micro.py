"""Microbenchmark: 1x1 backward-weight with a 64-channel side, default 128-wide tiles vs one
256-wide tile (conv_set_wgrad_wide), ResNet-50 layer-1 shapes at batch 256."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_training_amd import ops  # noqa: E402

C_ = ops.native()
CL = torch.channels_last
for (N, C, H, W, Co) in [(256, 64, 56, 56, 256), (256, 256, 56, 56, 64)]:
    x = torch.randn(N, C, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    gy = torch.randn(N, Co, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    res = []
    for mode in (0, 1, 0, 1):
        C_.conv_set_wgrad_wide(mode)
        for _ in range(3):
            C_.conv_wgrad(gy, x, [Co, C, 1, 1], 1, 0, False)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            C_.conv_wgrad(gy, x, [Co, C, 1, 1], 1, 0, False)
        e1.record()
        torch.cuda.synchronize()
        res.append(e0.elapsed_time(e1) / 20)
    print(f"{C}x{H}x{W}->{Co}: " + " ".join(f"w{m}={t:.4f}ms" for m, t in zip((0, 1, 0, 1), res)), flush=True)
C_.conv_set_wgrad_wide(0)
