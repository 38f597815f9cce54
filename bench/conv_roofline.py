"""Per-layer roofline of ResNet-50's convolutions on MI355X (bf16, channels_last).

For every distinct conv of ResNet-50 at the bench batch it times forward, backward-data and
backward-weight (MIOpen, whatever the find-db / heuristics pick) and reports achieved
TFLOP/s and TB/s against the chip's dense bf16 peak (2.5 PF) and HBM (~6.3 TB/s
achievable), so the layers worth a hand-written kernel stand out.

    python bench/conv_roofline.py --batch 256 > gpurun_out/conv_roofline.md
"""
from __future__ import annotations

import argparse
import os
import sys
from collections import OrderedDict

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PEAK_TF = 2500.0
HBM_TBS = 6.3


def resnet50_convs(batch: int, image: int):
    from distributed_pytorch_training_amd.models import build_model

    m = build_model("resnet50", 1000, image_size=image)
    shapes = OrderedDict()
    hooks = []

    def hook(mod, inp, out):
        key = (tuple(inp[0].shape[1:]), mod.out_channels, mod.kernel_size, mod.stride, mod.padding)
        shapes[key] = shapes.get(key, 0) + 1

    for mod in m.modules():
        if isinstance(mod, torch.nn.Conv2d):
            hooks.append(mod.register_forward_hook(hook))
    with torch.no_grad():
        m(torch.zeros(1, 3, image, image))
    return shapes


def time_ms(fn, iters=20):
    for _ in range(3):
        fn()
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    start.record()
    for _ in range(iters):
        fn()
    end.record()
    torch.cuda.synchronize()
    return start.elapsed_time(end) / iters


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--image", type=int, default=224)
    a = ap.parse_args(argv)
    from distributed_pytorch_training_amd.utils.env import setup_miopen_env

    setup_miopen_env()
    torch.backends.cudnn.benchmark = False
    dev = torch.device("cuda")
    cl = torch.channels_last
    rows = []
    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}
    for (cin_hw, cout, k, s, p), count in resnet50_convs(a.batch, a.image).items():
        cin, h, w = cin_hw
        x = torch.randn(a.batch, cin, h, w, device=dev, dtype=torch.bfloat16).contiguous(memory_format=cl)
        wt = torch.randn(cout, cin, *k, device=dev, dtype=torch.bfloat16).contiguous(memory_format=cl) * 0.05
        y = F.conv2d(x, wt, stride=s, padding=p)
        gy = torch.randn_like(y)
        ho, wo = y.shape[2], y.shape[3]
        flops = 2.0 * a.batch * ho * wo * cout * cin * k[0] * k[1]
        bx, by, bw = x.numel() * 2, y.numel() * 2, wt.numel() * 2
        t_f = time_ms(lambda: F.conv2d(x, wt, stride=s, padding=p))
        t_d = time_ms(lambda: torch.nn.grad.conv2d_input(x.shape, wt, gy, stride=s, padding=p))
        t_w = time_ms(lambda: torch.nn.grad.conv2d_weight(x, wt.shape, gy, stride=s, padding=p))
        for name, t, byts in (("fwd", t_f, bx + bw + by), ("dgrad", t_d, by + bw + bx), ("wgrad", t_w, bx + by + bw)):
            tf = flops / t / 1e9
            tb = byts / t / 1e9
            bound = max(flops / (PEAK_TF * 1e12), byts / (HBM_TBS * 1e12)) * 1e3
            rows.append((f"{cin}x{h}x{w}->{cout} k{k[0]} s{s[0]}", count, name, t, tf, tb, bound))
            tot[name] += t * count
    print(f"# ResNet-50 conv roofline, batch {a.batch}, bf16 channels_last, MIOpen (immediate mode)\n")
    print("| conv | x | pass | ms | TFLOP/s | TB/s | roofline ms | ms over roofline (x count) |")
    print("|---|---|---|---|---|---|---|---|")
    for r in sorted(rows, key=lambda r: -(r[3] - r[6]) * r[1]):
        print(f"| {r[0]} | {r[1]} | {r[2]} | {r[3]:.3f} | {r[4]:.0f} | {r[5]:.2f} | {r[6]:.3f} | {(r[3]-r[6])*r[1]:.3f} |")
    print(f"\nper-step totals (ms): " + ", ".join(f"{k} {v:.2f}" for k, v in tot.items())
          + f", all {sum(tot.values()):.2f}")


if __name__ == "__main__":
    main()
