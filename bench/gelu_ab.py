"""ViT-B/16's GELU passes (fc1 output [128 x 197, 3072], bf16) at several occupancies of the
column-stationary kernels (``vit_set_gelu_blocks_per_cu``): median us per call and TB/s of the
bytes each pass must move (forward: u in, h out; backward: gh and u in, gu out).

    python bench/gelu_ab.py [--blocks 4,6,8,12,16]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _time(fn, reps=30):
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
    ap.add_argument("--blocks", default="4,6,8,12,16")
    a = ap.parse_args(argv)
    from distributed_pytorch_training_amd.ops import native
    C = native()
    dev = torch.device("cuda:0")
    T, F = 128 * 197, 3072
    u = torch.randn(T, F, device=dev).to(torch.bfloat16)
    gh = torch.randn(T, F, device=dev).to(torch.bfloat16)
    b = torch.randn(F, device=dev).to(torch.bfloat16)
    nbytes = T * F * 2
    for n in [int(v) for v in a.blocks.split(",")]:
        C.vit_set_gelu_blocks_per_cu(n)
        f = _time(lambda: C.gelu_fwd(u, b))
        g = _time(lambda: C.gelu_bwd(gh, u, b, True))
        print(json.dumps({"blocks_per_cu": n, "us_fwd": round(f, 1), "tbs_fwd": round(2 * nbytes / f / 1e6, 2),
                          "us_bwd": round(g, 1), "tbs_bwd": round(3 * nbytes / g / 1e6, 2)}), flush=True)
    C.vit_set_gelu_blocks_per_cu(6)


if __name__ == "__main__":
    main()
