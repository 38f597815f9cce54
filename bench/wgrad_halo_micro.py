import os, sys; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
"""Microbenchmark: 3x3 / stride-1 backward-weight per halo mode (conv_set_wgrad_halo) at the
ResNet-50 batch-256 shapes; WH_MODES=0,3 picks the modes.  Results: profiles/wgrad_halo_r2.md."""
import torch, sys
from distributed_pytorch_training_amd import ops
C_ = ops.native()
MODES = [int(m) for m in os.environ.get("WH_MODES", "0,1,2,3,4").split(",")]
CL = torch.channels_last
shapes = [(256, 64, 56, 56, 64), (256, 128, 28, 28, 128), (256, 256, 14, 14, 256), (256, 512, 7, 7, 512)]
for (N, C, H, W, Co) in shapes:
    x = torch.randn(N, C, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    gy = torch.randn(N, Co, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    res = []
    for mode in MODES:
        C_.conv_set_wgrad_halo(mode)
        for _ in range(3):
            C_.conv_wgrad(gy, x, [Co, C, 3, 3], 1, 1, False)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            C_.conv_wgrad(gy, x, [Co, C, 3, 3], 1, 1, False)
        e1.record(); torch.cuda.synchronize()
        res.append(e0.elapsed_time(e1) / 20)
    print(f"{C}x{H}x{W}->{Co}: " + " ".join(f"m{m}={t:.4f}ms" for m, t in zip(MODES, res)), flush=True)
C_.conv_set_wgrad_halo(0)
