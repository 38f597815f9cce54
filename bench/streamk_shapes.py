"""Per-conv A/B of the stream-K grid (conv_set_streamk) against the data-parallel grid, at the
ResNet-50 batch-256 conv shapes whose tile grids spread unevenly over the 256 CUs: median
microseconds per launch over interleaved rounds (CUDA events around --reps launches).

    python bench/streamk_shapes.py [--reps 50] [--rounds 5] [--json-out f.json]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CL = torch.channels_last
# (name, N, C, H, W, Cout, k, stride, pad, op): op fwd = conv_fwd with BN statistics,
# dgrad = 1x1 backward-data with the BN statistics epilogue
SHAPES = [
    ("l2 1x1 512->128 @28", 256, 512, 28, 28, 128, 1, 1, 0, "fwd"),
    ("l3 1x1 1024->256 @14", 256, 1024, 14, 14, 256, 1, 1, 0, "fwd"),
    ("l4.0 1x1 1024->512 @14", 256, 1024, 14, 14, 512, 1, 1, 0, "fwd"),
    ("l4 1x1 2048->512 @7", 256, 2048, 7, 7, 512, 1, 1, 0, "fwd"),
    ("l3.0 3x3s2 256->256 @28", 256, 256, 28, 28, 256, 3, 2, 1, "fwd"),
    ("l4.0 3x3s2 512->512 @14", 256, 512, 14, 14, 512, 3, 2, 1, "fwd"),
    ("l3 dgrad 1x1 256<-1024 @14", 256, 256, 14, 14, 1024, 1, 1, 0, "dgrad"),
    ("l2 dgrad 1x1 128<-512 @28", 256, 128, 28, 28, 512, 1, 1, 0, "dgrad"),
    ("l4 dgrad 1x1 512<-2048 @7", 256, 512, 7, 7, 2048, 1, 1, 0, "dgrad"),
]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--json-out", default="")
    a = ap.parse_args(argv)
    from distributed_pytorch_training_amd import ops
    C_ = ops.native()
    dev = torch.device("cuda:0")
    C_.conv_sk_prepare()
    rows = []
    for name, N, C, H, W, Co, k, st, pad, op in SHAPES:
        g = torch.Generator(device=dev).manual_seed(0)
        if op == "fwd":
            x = torch.randn(N, C, H, W, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=CL)
            w = (torch.randn(Co, C, k, k, device=dev, generator=g) / (C * k * k) ** 0.5).to(torch.bfloat16)
            w = w.contiguous(memory_format=CL)
            fn = lambda: C_.conv_fwd(x, w, st, pad, True)  # noqa: E731
            Ho, Wo = (H + 2 * pad - k) // st + 1, (W + 2 * pad - k) // st + 1
            M, cout, K = N * Ho * Wo, Co, k * k * C
        else:
            w = (torch.randn(Co, C, 1, 1, device=dev, generator=g) / C ** 0.5).to(torch.bfloat16)
            w = w.contiguous(memory_format=CL)
            gy = torch.randn(N, Co, H, W, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=CL)
            bx = torch.randn(N, C, H, W, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=CL)
            mean = torch.randn(C, device=dev, generator=g)
            coef = torch.randn(2 * C, device=dev, generator=g)
            fn = lambda: C_.conv_dgrad_bnstats(gy, w, 0, bx, mean, coef)  # noqa: E731
            M, cout, K = N * H * W, C, Co
        bn = 128 if cout % 128 == 0 else 64
        tiles = -(-M // 128) * (cout // bn)
        res = {0: [], 1: [], 2: []}
        for _ in range(a.rounds):
            for mode in (0, 1, 2):
                C_.conv_set_streamk(mode)
                fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                res[mode].append(e0.elapsed_time(e1) * 1000 / a.reps)
        C_.conv_set_streamk(0)
        row = {"shape": name, "tiles": tiles, "nk": K // 64, "sk_blocks_auto": C_.conv_sk_blocks(tiles, K // 64, bn, 1),
               "sk_blocks_all": C_.conv_sk_blocks(tiles, K // 64, bn, 2),
               "us_dp": statistics.median(res[0]), "us_auto": statistics.median(res[1]),
               "us_all": statistics.median(res[2])}
        rows.append(row)
        print(json.dumps(row), flush=True)
    assert C_.conv_sk_errors() == 0
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(rows, f, indent=1)
    print("\n| conv (batch 256) | tiles | K-steps | DP grid us | stream-K us (blocks) | ratio |")
    print("|---|---|---|---|---|---|")
    for r in rows:
        print(f"| {r['shape']} | {r['tiles']} | {r['nk']} | {r['us_dp']:.1f} | {r['us_all']:.1f} ({r['sk_blocks_all']}) | "
              f"{r['us_all'] / r['us_dp']:.3f} |")


if __name__ == "__main__":
    main()
