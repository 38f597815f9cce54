"""Tiny deterministic driver for rocprofv3 --pmc passes over the fused attention kernels at the
ViT-B/16 shape (batch 128, 12 heads, 197 tokens, head dim 64): a few forward + backward calls.

    rocprofv3 --pmc SQ_WAVES ... -d gpurun_out/apmc/p1 -- python3 bench/attn_pmc.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from distributed_pytorch_training_amd import ops

    C = ops.native()
    torch.manual_seed(0)
    B, S, H = 128, 197, 12
    qkv = torch.randn(B, S, 3 * H * 64, device="cuda").to(torch.bfloat16)
    dout = torch.randn(B, S, H * 64, device="cuda").to(torch.bfloat16)
    for _ in range(3):
        out, lse = C.attn_fwd(qkv, H, 0.125)
        C.attn_bwd(qkv, out, dout, lse, H, 0.125)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
