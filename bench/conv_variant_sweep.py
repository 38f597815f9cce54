"""Forward-conv tile variants on the ResNet-50 shapes where the default tile trails MIOpen.

For each shape: MIOpen's forward (cudnn.benchmark off: immediate mode, as conv_bench.py), then
every conv_fwd_kernel tiling the dispatcher can launch - 4 (128x128, default), 5/6 (256-row
blocks), 9..13 (8-wave 256x256 / 256x128 / 128x256, 2- and 3-stage), 7 / 8 / 14 (BK = 32
pipelined K loop, 3 / 4 / 2 stages) - with and without the BN-statistics epilogue the training
step uses.  Mean of 20 timed repeats per cell (conv_roofline.time_ms).

    python bench/conv_variant_sweep.py [--batch 256] [--all | --small-1x1] [--variants 4,14,7]
"""
from __future__ import annotations

import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench.conv_roofline import resnet50_convs, time_ms  # noqa: E402

BEHIND = {(64, 56, 256, 1, 1), (256, 56, 64, 1, 1), (128, 28, 512, 1, 1), (256, 28, 256, 3, 2)}
VARIANTS = (4, 5, 6, 9, 10, 11, 12, 13)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--all", action="store_true", help="every ResNet-50 shape, not just the four behind MIOpen")
    ap.add_argument("--small-1x1", action="store_true",
                    help="the stride-1 1x1 shapes whose 128 x 128 grid is under 1,024 tiles")
    ap.add_argument("--variants", default=",".join(map(str, VARIANTS)))
    a = ap.parse_args(argv)
    variants = [int(v) for v in a.variants.split(",")]
    from distributed_pytorch_training_amd import ops
    from distributed_pytorch_training_amd.utils.env import setup_miopen_env

    setup_miopen_env()
    torch.backends.cudnn.benchmark = False
    C_ = ops.native()
    dev = torch.device("cuda")
    cl = torch.channels_last
    print(f"# forward tile variants vs MIOpen, ResNet-50 batch {a.batch}, bf16 channels_last (ms; +s = with BN statistics)\n")
    print("| conv | MIOpen | " + " | ".join(f"v{v} / +s" for v in variants) + " | best+s vs MIOpen |")
    print("|---|---|" + "---|" * len(variants) + "---|")
    for (cin_hw, cout, k, s, p), count in resnet50_convs(a.batch, 224).items():
        cin, h, w = cin_hw
        if cin % 64 or cout % 64:
            continue
        if a.small_1x1:
            tiles = -(-a.batch * h * w // 128) * (cout // (128 if cout % 128 == 0 else 64))
            if k[0] != 1 or s[0] != 1 or tiles >= 1024:
                continue
        elif not a.all and (cin, h, cout, k[0], s[0]) not in BEHIND:
            continue
        x = torch.randn(a.batch, cin, h, w, device=dev, dtype=torch.bfloat16).contiguous(memory_format=cl)
        wt = (torch.randn(cout, cin, *k, device=dev, dtype=torch.bfloat16) * 0.05).contiguous(memory_format=cl)
        ref = F.conv2d(x.float(), wt.float(), stride=s, padding=p)
        t_m = time_ms(lambda: F.conv2d(x, wt, stride=s, padding=p))
        cells, best = [], None
        for v in variants:
            C_.conv_set_variant(v)
            out = C_.conv_fwd(x, wt, s[0], p[0], False)
            y = out[0] if isinstance(out, (tuple, list)) else out
            err = ((y.float() - ref).norm() / ref.norm()).item()
            if not err < 2e-2:
                cells.append(f"wrong ({err:.1e})")
                continue
            t0 = time_ms(lambda: C_.conv_fwd(x, wt, s[0], p[0], False))
            t1 = time_ms(lambda: C_.conv_fwd(x, wt, s[0], p[0], True))
            cells.append(f"{t0:.3f} / {t1:.3f}")
            if best is None or t1 < best[0]:
                best = (t1, v)
        C_.conv_set_variant(0)
        name = f"{cin}x{h}x{w}->{cout} k{k[0]} s{s[0]} (x{count})"
        tail = f"v{best[1]}: {t_m / best[0]:.2f}x" if best else "-"
        print(f"| {name} | {t_m:.3f} | " + " | ".join(cells) + f" | {tail} |", flush=True)


if __name__ == "__main__":
    main()
