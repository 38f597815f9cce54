"""Backward-weight split-K block target per ResNet-50 conv shape (conv_set_wgrad_target): time of
the full backward-weight (GEMM + split reduce) for each target, bf16, batch 256.

    python bench/wgrad_target_sweep.py [--targets 384 512 640 768 1024] > gpurun_out/wt.md
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench.conv_roofline import resnet50_convs, time_ms  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--targets", type=int, nargs="+", default=[384, 512, 640, 768, 1024])
    a = ap.parse_args(argv)
    from distributed_pytorch_training_amd import ops

    C_ = ops.native()
    dev = torch.device("cuda")
    cl = torch.channels_last
    print(f"# backward-weight split-K block target, ResNet-50, batch {a.batch}, bf16 NHWC\n")
    print("| conv | x | tiles | steps | " + " | ".join(f"t{t} ms" for t in a.targets) + " | best |")
    print("|---|---|---|---|" + "---|" * len(a.targets) + "---|")
    tot = {t: 0.0 for t in a.targets}
    best = 0.0
    for (cin_hw, cout, k, s, p), count in resnet50_convs(a.batch, a.image).items():
        cin, h, w = cin_hw
        if cin % 64 or cout % 64:
            continue
        x = torch.randn(a.batch, cin, h, w, device=dev, dtype=torch.bfloat16).contiguous(memory_format=cl)
        ho = (h + 2 * p[0] - k[0]) // s[0] + 1
        gy = torch.randn(a.batch, cout, ho, ho, device=dev, dtype=torch.bfloat16).contiguous(memory_format=cl)
        bmw = 128 if cout % 128 == 0 else 64
        bnw = 128 if (cin % 128 == 0 or (cin == 64 and k[0] * k[1] > 1)) else 64
        tiles = (cout // bmw) * ((k[0] * k[1] * cin + bnw - 1) // bnw)
        steps = (a.batch * ho * ho + 63) // 64
        times = {}
        for t in a.targets:
            C_.conv_set_wgrad_target(t)
            times[t] = time_ms(lambda: C_.conv_wgrad(gy, x, [cout, cin, k[0], k[1]], s[0], p[0], False))
            tot[t] += times[t] * count
        C_.conv_set_wgrad_target(0)
        bt = min(times, key=times.get)
        best += times[bt] * count
        name = f"{cin}x{h}x{w}->{cout} k{k[0]} s{s[0]}"
        print(f"| {name} | {count} | {tiles} | {steps} | " + " | ".join(f"{times[t]:.3f}" for t in a.targets)
              + f" | t{bt} |", flush=True)
    print("\nper step (x count): " + ", ".join(f"t{t} {v:.3f} ms" for t, v in tot.items()) + f", best-of {best:.3f} ms")


if __name__ == "__main__":
    main()
