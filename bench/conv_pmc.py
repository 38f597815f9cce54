"""Tiny driver for rocprofv3 --pmc runs: a few launches of the MFMA conv kernels on fixed shapes."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_training_amd import ops  # noqa: E402

C_ = ops.native()
dev = torch.device("cuda")
cl = torch.channels_last
for (cin, hw, cout, k, s, p) in [(256, 14, 256, 3, 1, 1), (64, 56, 256, 1, 1, 0)]:
    x = torch.randn(256, cin, hw, hw, device=dev, dtype=torch.bfloat16).contiguous(memory_format=cl)
    w = (torch.randn(cout, cin, k, k, device=dev, dtype=torch.bfloat16) * 0.05).contiguous(memory_format=cl)
    for _ in range(3):
        y = C_.conv_fwd(x, w, s, p, False)[0]
    gy = torch.randn_like(y)
    for _ in range(3):
        C_.conv_wgrad(gy, x, list(w.shape), s, p, True)
torch.cuda.synchronize()
print("ok")
