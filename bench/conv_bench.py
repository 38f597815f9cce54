"""Hand-written MFMA convs (conv_kernels.hip) vs MIOpen, per ResNet-50 conv shape, batch 256.

    python bench/conv_bench.py [--batch 256] > gpurun_out/conv_bench.md
"""
from __future__ import annotations

import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench.conv_roofline import PEAK_TF, resnet50_convs, time_ms  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--image", type=int, default=224)
    a = ap.parse_args(argv)
    from distributed_pytorch_training_amd import ops
    from distributed_pytorch_training_amd.utils.env import setup_miopen_env

    setup_miopen_env()
    torch.backends.cudnn.benchmark = False
    C_ = ops.native()
    dev = torch.device("cuda")
    cl = torch.channels_last
    print(f"# conv_kernels.hip vs MIOpen, ResNet-50 convs, batch {a.batch}, bf16 channels_last\n")
    print("| conv | x | pass | MIOpen ms | ours ms | ours+stats ms | speedup | ours TF/s | ours TB/s | v4 / v7(pipe3) / v8(pipe4) ms |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    tot = {"fwd": [0.0, 0.0], "dgrad": [0.0, 0.0], "wgrad": [0.0, 0.0]}
    for (cin_hw, cout, k, s, p), count in resnet50_convs(a.batch, a.image).items():
        cin, h, w = cin_hw
        if cin % 64 or cout % 64:
            continue
        x = torch.randn(a.batch, cin, h, w, device=dev, dtype=torch.bfloat16).contiguous(memory_format=cl)
        wt = (torch.randn(cout, cin, *k, device=dev, dtype=torch.bfloat16) * 0.05).contiguous(memory_format=cl)
        y = F.conv2d(x, wt, stride=s, padding=p)
        gy = torch.randn_like(y)
        flops = 2.0 * y.numel() * cin * k[0] * k[1]
        byts = (x.numel() + y.numel() + wt.numel()) * 2
        t_m = time_ms(lambda: F.conv2d(x, wt, stride=s, padding=p))
        t_o = time_ms(lambda: C_.conv_fwd(x, wt, s[0], p[0], False))
        t_os = time_ms(lambda: C_.conv_fwd(x, wt, s[0], p[0], True))
        tv = []
        for v in (4, 7, 8):
            C_.conv_set_variant(v)
            tv.append(time_ms(lambda: C_.conv_fwd(x, wt, s[0], p[0], False)))
        C_.conv_set_variant(0)
        t_reg = " / ".join(f"{t:.3f}" for t in tv)
        name = f"{cin}x{h}x{w}->{cout} k{k[0]} s{s[0]}"
        print(f"| {name} | {count} | fwd | {t_m:.3f} | {t_o:.3f} | {t_os:.3f} | {t_m / t_o:.2f} | "
              f"{flops / t_o / 1e9:.0f} | {byts / t_o / 1e9:.2f} | {t_reg} |", flush=True)
        t_w = time_ms(lambda: torch.ops.aten.convolution_backward(
            gy, x, wt, None, s, p, (1, 1), False, (0, 0), 1, (False, True, False)))
        t_wo = time_ms(lambda: C_.conv_wgrad(gy, x, list(wt.shape), s[0], p[0], True))
        C_.conv_set_variant(1)
        t_wo2 = time_ms(lambda: C_.conv_wgrad(gy, x, list(wt.shape), s[0], p[0], True))
        C_.conv_set_variant(0)
        print(f"| {name} | {count} | wgrad | {t_w:.3f} | {t_wo:.3f} | - | {t_w / t_wo:.2f} | "
              f"{flops / t_wo / 1e9:.0f} | {byts / t_wo / 1e9:.2f} | 2-stage {t_wo2:.3f} |", flush=True)
        tot["wgrad"][0] += t_w * count
        tot["wgrad"][1] += min(t_w, t_wo) * count
        tot["fwd"][0] += t_m * count
        tot["fwd"][1] += min(t_m, t_o) * count
        if s[0] == 1:
            # autograd's own call (torch.nn.grad.conv2d_input takes a slower transposed-conv route)
            t_m = time_ms(lambda: torch.ops.aten.convolution_backward(
                gy, x, wt, None, s, p, (1, 1), False, (0, 0), 1, (True, False, False)))
            t_o = time_ms(lambda: C_.conv_dgrad(gy, wt, p[0]))
            t_of = time_ms(lambda: C_.conv_dgrad_flip(gy, wt, p[0]))
            print(f"| {name} | {count} | dgrad | {t_m:.3f} | {t_o:.3f} | - | {t_m / t_o:.2f} | "
                  f"{flops / t_o / 1e9:.0f} | {byts / t_o / 1e9:.2f} | flip-copy {t_of:.3f} |", flush=True)
            tot["dgrad"][0] += t_m * count
            tot["dgrad"][1] += min(t_m, t_o) * count
    for k_, (m, o) in tot.items():
        print(f"\n{k_}: MIOpen {m:.2f} ms/step, best-of {o:.2f} ms/step")


if __name__ == "__main__":
    main()
