"""Attention backward at the ViT-B/16 shape: one two-phase kernel vs the two phase kernels
(attn_set_bwd_split), time per call and bitwise agreement.

    python bench/attn_bwd_ab.py
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
    out, lse = C.attn_fwd(qkv, H, 0.125)
    res = {}
    for split in (0, 1, 0, 1):
        C.attn_set_bwd_split(split)
        g = C.attn_bwd(qkv, out, dout, lse, H, 0.125)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(3):
            C.attn_bwd(qkv, out, dout, lse, H, 0.125)
        torch.cuda.synchronize()
        s.record()
        for _ in range(20):
            C.attn_bwd(qkv, out, dout, lse, H, 0.125)
        e.record()
        torch.cuda.synchronize()
        res.setdefault(split, []).append(s.elapsed_time(e) / 20 * 1e3)
        res[f"g{split}"] = g
    C.attn_set_bwd_split(0)
    same = torch.equal(res["g0"], res["g1"])
    print(f"one kernel {res[0]} us, split {res[1]} us, bitwise equal: {same}")


if __name__ == "__main__":
    main()
