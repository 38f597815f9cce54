"""1x1 stride-1 convolution: MIOpen conv vs GEMM (hipBLASLt) on channels_last bf16, fwd+bwd.

In channels_last memory a 1x1 stride-1 conv IS a GEMM: y[M, Cout] = x[M, Cin] @ W[Cout, Cin]^T
with M = N*H*W and no data movement; dgrad and wgrad are GEMMs too.  This times both routes
for every 1x1 stride-1 conv shape of ResNet-50 at the bench batch, as autograd runs them.
"""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def t_ms(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    from distributed_pytorch_training_amd.utils.env import setup_miopen_env
    setup_miopen_env()
    torch.backends.cudnn.benchmark = False
    dev = torch.device("cuda")
    B = a.batch
    shapes = [(64, 56, 256, 4), (256, 56, 64, 2), (256, 28, 128, 0), (128, 28, 512, 4), (512, 28, 128, 3),
              (512, 14, 256, 0), (256, 14, 1024, 6), (1024, 14, 256, 5), (1024, 7, 512, 0), (512, 7, 2048, 3),
              (2048, 7, 512, 2), (64, 56, 64, 1), (256, 56, 128, 1), (512, 28, 256, 1), (1024, 14, 512, 1)]
    print("| Cin x HW -> Cout | count | MIOpen fwd+bwd ms | GEMM fwd+bwd ms | speedup |\n|---|---|---|---|---|")
    tot_c = tot_g = 0.0
    for cin, hw, cout, count in shapes:
        count = max(count, 1)
        x = torch.randn(B, cin, hw, hw, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(cout, cin, 1, 1, device=dev, dtype=torch.bfloat16) * 0.05).contiguous(memory_format=torch.channels_last)
        x.requires_grad_()
        w.requires_grad_()
        gy = torch.randn(B, cout, hw, hw, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)

        def conv():
            y = F.conv2d(x, w)
            torch.autograd.backward(y, gy)

        def gemm():
            xm = x.permute(0, 2, 3, 1).reshape(-1, cin)
            y = (xm @ w.view(cout, cin).t()).view(B, hw, hw, cout).permute(0, 3, 1, 2)
            torch.autograd.backward(y, gy)

        tc, tg = t_ms(conv), t_ms(gemm)
        tot_c += tc * count
        tot_g += tg * count
        print(f"| {cin}x{hw}x{hw} -> {cout} | {count} | {tc:.3f} | {tg:.3f} | {tc/tg:.2f} |", flush=True)
    print(f"\nweighted totals: MIOpen {tot_c:.2f} ms, GEMM {tot_g:.2f} ms")


if __name__ == "__main__":
    main()
