"""ViT-B/16 linear layers (T = 25,216 tokens at batch 128): hipBLASLt (F.linear with the shipped
TunableOp db) against the native MFMA 1x1-conv forward kernel (``conv_fwd`` on a [1, K, 1, T]
channels-last view, no epilogue statistics) for the forward y = x W^T, and against the native
backward-data kernel for dX = dY W.  Median us per call and TFLOP/s; max abs difference vs
F.linear (both round to bf16 once).

    python bench/vit_linear_ab.py [--reps 20]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [(2304, 768), (768, 768), (3072, 768), (768, 3072)]   # (n_out, n_in): qkv, proj, fc1, fc2


def _time(fn, reps):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1000 / reps)
    return statistics.median(ts)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--tokens", type=int, default=128 * 197)
    a = ap.parse_args(argv)
    from distributed_pytorch_training_amd.ops import native
    from distributed_pytorch_training_amd.utils.env import setup_tunableop
    dev = torch.device("cuda:0")
    setup_tunableop()
    C = native()
    T = a.tokens
    cl = torch.channels_last
    for n_out, n_in in SHAPES:
        g = torch.Generator(device=dev).manual_seed(n_out * 7 + n_in)
        x = torch.randn(T, n_in, device=dev, generator=g).to(torch.bfloat16)
        w = (torch.randn(n_out, n_in, device=dev, generator=g) / n_in ** 0.5).to(torch.bfloat16)
        dy = torch.randn(T, n_out, device=dev, generator=g).to(torch.bfloat16)
        x4 = x.view(1, 1, T, n_in).permute(0, 3, 1, 2)
        w4 = w.view(n_out, n_in, 1, 1).contiguous(memory_format=cl)
        dy4 = dy.view(1, 1, T, n_out).permute(0, 3, 1, 2)
        flop = 2.0 * T * n_out * n_in
        row = {"n_out": n_out, "n_in": n_in}
        ref = F.linear(x, w)
        y4 = C.conv_fwd(x4, w4, 1, 0, False)[0]
        row["fwd_maxdiff"] = (y4.permute(0, 2, 3, 1).reshape(T, n_out).float() - ref.float()).abs().max().item()
        row["us_fwd_hipblaslt"] = _time(lambda: F.linear(x, w), a.reps)
        row["us_fwd_native"] = _time(lambda: C.conv_fwd(x4, w4, 1, 0, False), a.reps)
        dref = dy @ w
        dx4 = C.conv_dgrad(dy4, w4, 0)
        dx4 = dx4[0] if isinstance(dx4, (tuple, list)) else dx4
        row["dgrad_maxdiff"] = (dx4.permute(0, 2, 3, 1).reshape(T, n_in).float() - dref.float()).abs().max().item()
        row["us_dgrad_hipblaslt"] = _time(lambda: dy @ w, a.reps)
        row["us_dgrad_native"] = _time(lambda: C.conv_dgrad(dy4, w4, 0), a.reps)
        for k in ("fwd_hipblaslt", "fwd_native", "dgrad_hipblaslt", "dgrad_native"):
            row["tflops_" + k] = round(flop / row["us_" + k] / 1e6, 1)
            row["us_" + k] = round(row["us_" + k], 1)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
