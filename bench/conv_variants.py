"""Forward conv kernel variants (conv_kernels.hip ``conv_set_variant``) per ResNet-50 conv shape:
time, TFLOP/s and max |difference| against the default variant's output.

    python bench/conv_variants.py [--variants 0 9 10 11] [--batch 256] [--stats] > gpurun_out/cv.md
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
    ap.add_argument("--variants", type=int, nargs="+", default=[0, 9, 10, 11])
    ap.add_argument("--stats", action="store_true", help="with the BN-statistics epilogue")
    ap.add_argument("--dgrad", action="store_true",
                    help="time the stride-1 backward-data instead (the forward kernel on dy with the "
                         "flipped weight, as the training step runs it)")
    a = ap.parse_args(argv)
    from distributed_pytorch_training_amd import ops

    C_ = ops.native()
    dev = torch.device("cuda")
    cl = torch.channels_last
    print(f"# {'backward-data' if a.dgrad else 'forward'} conv variants, ResNet-50, batch {a.batch}, bf16 NHWC, "
          f"stats={a.stats}\n")
    print("| conv | x | " + " | ".join(f"v{v} ms (TF/s)" for v in a.variants) + " | best | max diff |")
    print("|---|---|" + "---|" * len(a.variants) + "---|---|")
    tot = {v: 0.0 for v in a.variants}
    best_tot = 0.0
    for (cin_hw, cout, k, s, p), count in resnet50_convs(a.batch, a.image).items():
        cin, h, w = cin_hw
        if cin % 64 or cout % 64:
            continue
        if a.dgrad:
            if s[0] != 1:
                continue
            # dx = conv(dy, flip(w)^T, pad' = R-1-pad): a forward conv cout -> cin on the output grid
            ho = (h + 2 * p[0] - k[0]) // s[0] + 1
            cin, cout, h, w, p = cout, cin, ho, ho, (k[0] - 1 - p[0], k[1] - 1 - p[1])
        x = torch.randn(a.batch, cin, h, w, device=dev, dtype=torch.bfloat16).contiguous(memory_format=cl)
        wt = (torch.randn(cout, cin, *k, device=dev, dtype=torch.bfloat16) * 0.05).contiguous(memory_format=cl)
        cells, times, ref, diff = [], {}, None, 0.0
        for v in a.variants:
            C_.conv_set_variant(v)
            y = C_.conv_fwd(x, wt, s[0], p[0], a.stats)[0]
            if ref is None:
                ref = y.float()
                flops = 2.0 * y.numel() * cin * k[0] * k[1]
            else:
                diff = max(diff, float((y.float() - ref).abs().max()))
            t = time_ms(lambda: C_.conv_fwd(x, wt, s[0], p[0], a.stats))
            times[v] = t
            tot[v] += t * count
            cells.append(f"{t:.3f} ({flops / t / 1e9:.0f})")
        C_.conv_set_variant(0)
        bv = min(times, key=times.get)
        best_tot += times[bv] * count
        name = f"{cin}x{h}x{w}->{cout} k{k[0]} s{s[0]}"
        print(f"| {name} | {count} | " + " | ".join(cells) + f" | v{bv} | {diff:.3g} |", flush=True)
    print("\nper step (x count): " + ", ".join(f"v{v} {t:.3f} ms" for v, t in tot.items())
          + f", best-of {best_tot:.3f} ms")


if __name__ == "__main__":
    main()
