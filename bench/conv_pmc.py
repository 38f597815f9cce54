"""Tiny driver for rocprofv3 --pmc runs: a few launches of the MFMA conv kernels on fixed shapes.

    rocprofv3 --pmc SQ_WAVE_CYCLES ... -- python3 bench/conv_pmc.py [--shape CIN HW COUT K S P]... [--ops fwd wgrad]

Default shapes: 3x3 256->256 at 14x14 (layer3) and 3x3 64->64 at 56x56 (layer1), batch 256.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_training_amd import ops  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", type=int, nargs=6, action="append", metavar=("CIN", "HW", "COUT", "K", "S", "P"))
    ap.add_argument("--ops", nargs="+", default=["fwd", "wgrad"], choices=["fwd", "wgrad", "dgrad"])
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--wvariant", type=int, default=0)
    ap.add_argument("--fvariants", type=int, nargs="+", default=[0],
                    help="forward / backward-data kernel variants to run, in order (conv_set_variant)")
    a = ap.parse_args(argv)
    shapes = a.shape or [(256, 14, 256, 3, 1, 1), (64, 56, 64, 3, 1, 1)]
    C_ = ops.native()
    dev = torch.device("cuda")
    cl = torch.channels_last
    for (cin, hw, cout, k, s, p) in shapes:
        x = torch.randn(a.batch, cin, hw, hw, device=dev, dtype=torch.bfloat16).contiguous(memory_format=cl)
        w = (torch.randn(cout, cin, k, k, device=dev, dtype=torch.bfloat16) * 0.05).contiguous(memory_format=cl)
        y = C_.conv_fwd(x, w, s, p, True)[0]
        gy = torch.randn_like(y)
        wt = C_.conv_dgrad_flip(gy, w, p)[1] if ("dgrad" in a.ops and s == 1) else None
        for fv in a.fvariants:
            for _ in range(a.reps):
                C_.conv_set_variant(fv)
                if "fwd" in a.ops:
                    C_.conv_fwd(x, w, s, p, True)
                if "dgrad" in a.ops and s == 1:
                    C_.conv_dgrad_preflipped(gy, wt, p)
                C_.conv_set_variant(0)
        for _ in range(a.reps):
            if "wgrad" in a.ops:
                C_.conv_set_variant(a.wvariant)
                C_.conv_wgrad(gy, x, list(w.shape), s, p, True)
                C_.conv_set_variant(0)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
