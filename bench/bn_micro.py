"""Microbenchmark of the fused BN kernels at ResNet-50's block-tail shapes (batch 256).

Reports achieved HBM-equivalent bandwidth per pass (bytes the kernel chain must move / time).
The geometry constants it was used to pick (kBnMaxChunks etc., bn_kernels.hip) are compile-time
constants now: edit and rebuild to re-sweep.  Per-layer roofline table: bench/bn_roofline.py.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_training_amd import ops  # noqa: E402

SHAPES = [(256, 256, 56, 56), (256, 512, 28, 28), (256, 1024, 14, 14), (256, 2048, 7, 7), (256, 64, 56, 56)]


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
    C_ = ops.native()
    dev = torch.device("cuda")
    tot_f = tot_b = 0.0
    for shape in SHAPES:
        n, c, h, w = shape
        mk = lambda: torch.randn(shape, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        x, r, dy, dy2 = mk(), mk(), mk(), mk()
        wgt = torch.ones(c, device=dev)
        b = torch.zeros(c, device=dev)
        rm, rv = torch.zeros(c, device=dev), torch.ones(c, device=dev)
        nb = torch.zeros(1, dtype=torch.long, device=dev)
        y, mean, invstd, _coef = C_.bn_fwd_train(x, r, wgt, b, rm, rv, nb, 0.1, 1e-5, True)
        bytes_pass = x.numel() * 2
        tf = t_ms(lambda: C_.bn_fwd_train(x, r, wgt, b, rm, rv, nb, 0.1, 1e-5, True))
        tb = t_ms(lambda: C_.bn_bwd(dy, dy2, y, x, wgt, mean, invstd, True, True, True))
        # fwd: stats read x (1) + apply read x, r + write y (3) = 4 passes
        # bwd: stats read dy, dy2, y, x + write dz (5) + apply read dz, x + write dx (3) = 8 passes
        tot_f += tf
        tot_b += tb
        print(f"{shape}: fwd {tf:.3f} ms = {4 * bytes_pass / tf / 1e9:.2f} TB/s | "
              f"bwd {tb:.3f} ms = {8 * bytes_pass / tb / 1e9:.2f} TB/s", flush=True)
    print(f"total fwd {tot_f:.3f} ms, bwd {tot_b:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
