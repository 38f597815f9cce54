"""Backward-weight conv kernel variants per ResNet-50 conv shape: default tiles vs the 8-wave
256 x 256 tile (conv_set_variant(20)), time, TFLOP/s and max relative difference.

    python bench/wgrad_variants.py [--batch 256] > gpurun_out/wv.md
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
    ap.add_argument("--variants", type=int, nargs="+", default=[0, 20])
    a = ap.parse_args(argv)
    from distributed_pytorch_training_amd import ops

    C_ = ops.native()
    dev = torch.device("cuda")
    cl = torch.channels_last
    print(f"# backward-weight variants, ResNet-50, batch {a.batch}, bf16 NHWC\n")
    print("| conv | x | " + " | ".join(f"v{v} ms (TF/s)" for v in a.variants) + " | best | max rel diff |")
    print("|---|---|" + "---|" * len(a.variants) + "---|---|")
    tot = {v: 0.0 for v in a.variants}
    best_tot = 0.0
    for (cin_hw, cout, k, s, p), count in resnet50_convs(a.batch, a.image).items():
        cin, h, w = cin_hw
        if cin % 64 or cout % 64:
            continue
        x = torch.randn(a.batch, cin, h, w, device=dev, dtype=torch.bfloat16).contiguous(memory_format=cl)
        ho, wo = (h + 2 * p[0] - k[0]) // s[0] + 1, (w + 2 * p[1] - k[1]) // s[1] + 1
        gy = torch.randn(a.batch, cout, ho, wo, device=dev, dtype=torch.bfloat16).contiguous(memory_format=cl)
        shape = [cout, cin, k[0], k[1]]
        flops = 2.0 * gy.numel() * cin * k[0] * k[1]
        cells, times, ref, diff = [], {}, None, 0.0
        for v in a.variants:
            C_.conv_set_variant(v)
            dw = C_.conv_wgrad(gy, x, shape, s[0], p[0], True)
            if ref is None:
                ref = dw
            else:
                diff = max(diff, float((dw - ref).abs().max() / ref.abs().max()))
            t = time_ms(lambda: C_.conv_wgrad(gy, x, shape, s[0], p[0], True))
            times[v] = t
            tot[v] += t * count
            cells.append(f"{t:.3f} ({flops / t / 1e9:.0f})")
        C_.conv_set_variant(0)
        bv = min(times, key=times.get)
        best_tot += times[bv] * count
        name = f"{cin}x{h}x{w}->{cout} k{k[0]} s{s[0]}"
        print(f"| {name} | {count} | " + " | ".join(cells) + f" | v{bv} | {diff:.2g} |", flush=True)
    print("\nper step (x count): " + ", ".join(f"v{v} {t:.3f} ms" for v, t in tot.items())
          + f", best-of {best_tot:.3f} ms")


if __name__ == "__main__":
    main()
