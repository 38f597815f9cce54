"""ViT-B/16 weight gradients dW = dY^T X (K = T = 25,216 tokens at batch 128) on two paths:
the current split-K batched hipBLASLt GEMM with fp32 partials + a sum kernel (ops/vit.py
``wgrad_splitk``), and the native MFMA backward-weight kernel of the 1x1 convolutions
(``conv_wgrad``: the same product over a [1, 1, T, C] channels-last "image", split-K with fp32
partials and a fixed-order reduce).  Median us per call and TFLOP/s, plus the relative L2
difference against an fp64 reference on a slice.

    python bench/vit_wgrad_ab.py [--reps 20]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [(2304, 768), (768, 768), (3072, 768), (768, 3072)]   # (n_out, n_in): qkv, proj, fc1, fc2


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--tokens", type=int, default=128 * 197)
    ap.add_argument("--targets", default="", help="comma list of conv_set_wgrad_target block counts to time "
                                                  "the native kernel at (0 = the shipped policy)")
    a = ap.parse_args(argv)
    from distributed_pytorch_training_amd.ops import native
    from distributed_pytorch_training_amd.ops.vit import wgrad_splitk
    from distributed_pytorch_training_amd.utils.env import setup_tunableop
    dev = torch.device("cuda:0")
    setup_tunableop()
    C = native()
    T = a.tokens
    rows = []
    for n_out, n_in in SHAPES:
        g = torch.Generator(device=dev).manual_seed(n_out + n_in)
        dy = torch.randn(T, n_out, device=dev, generator=g).to(torch.bfloat16)
        x = torch.randn(T, n_in, device=dev, generator=g).to(torch.bfloat16)
        dy4 = dy.view(1, 1, T, n_out).permute(0, 3, 1, 2)   # [1, n_out, 1, T] channels_last view
        x4 = x.view(1, 1, T, n_in).permute(0, 3, 1, 2)
        assert dy4.is_contiguous(memory_format=torch.channels_last)
        fns = {"splitk_hipblaslt": (0, lambda: wgrad_splitk(dy, x, torch.float32)),
               "native_conv_wgrad": (0, lambda: C.conv_wgrad(dy4, x4, [n_out, n_in, 1, 1], 1, 0, True))}
        for t in [int(v) for v in a.targets.split(",") if v.strip()]:
            fns[f"native_target{t}"] = (t, lambda: C.conv_wgrad(dy4, x4, [n_out, n_in, 1, 1], 1, 0, True))
        res = {}
        outs = {}
        for name, (target, fn) in fns.items():
            C.conv_set_wgrad_target(target)
            outs[name] = fn().reshape(n_out, n_in).float()
            torch.cuda.synchronize()
            ts = []
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1000 / a.reps)
            res[name] = statistics.median(ts)
            C.conv_set_wgrad_target(0)
        ref = (dy[:, :256].double().t() @ x[:, :256].double())
        err = {k: ((v[:256, :256].double() - ref).norm() / ref.norm()).item() for k, v in outs.items()}
        flop = 2.0 * T * n_out * n_in
        row = {"n_out": n_out, "n_in": n_in, "T": T,
               **{f"us_{k}": round(v, 1) for k, v in res.items()},
               **{f"tflops_{k}": round(flop / v / 1e6, 1) for k, v in res.items()},
               **{f"relerr_{k}": float(f"{v:.3g}") for k, v in err.items()}}
        rows.append(row)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
