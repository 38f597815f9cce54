"""Per-kernel roofline of every BatchNorm kernel left in the ResNet-50 bf16 training step.

After the conv epilogues took over every BN statistics pass (docs/DESIGN.md §7), each fused
BatchNorm is a finalize (tiny, per channel) + ONE apply pass per direction.  This tool times
those chains with the exact entry points the step uses, at every ResNet-50 BN shape (batch B,
224 px), and prices them against memory bandwidth:

* relu  (bn1 / bn2 of a bottleneck):   fwd bn_fwd_train(partials) reads x, writes y        4 MC B
                                        bwd bn_bwd_partials        reads dy, x, writes dx   6 MC B
* tail  (bn3 + identity residual):      fwd bn_fwd_train(residual) reads x, r, writes y     6 MC B
                                        bwd bn_bwd_partials(dz)    reads dz, x, writes dx   6 MC B
* tail+ds (bn3 + downsample BN):        fwd bn_apply_aff           reads x, x2, writes y    6 MC B
                                        bwd bn2_bwd_partials       reads dz, x, x2,
                                                                   writes dx, dx2          10 MC B
(M = B*H*W rows, C channels, 2-byte elements.)  The stem BN is applied inside the max-pool
kernels and is not listed.  Roofline = bytes / 6.29 TB/s (the measured HBM copy rate,
MI355X_MICROARCH.md); tensors that were just written by the producing conv and fit the 256 MiB
Infinity Cache can beat it.  Each chain is timed alone (cold L2, warm MALL after the first
iteration), so absolute numbers are the kernels' own, not the step's cache state.

    python bench/bn_roofline.py [--batch 256] > gpurun_out/bn_roofline.md
"""
from __future__ import annotations

import argparse
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench.conv_roofline import time_ms  # noqa: E402

HBM_TBS = 6.29


def resnet50_bn_layers(batch: int):
    """(kind, H, C) -> count for the BN layers of torchvision's ResNet-50 (v1.5 stride on conv2)."""
    out = collections.Counter()
    hw = 56
    inplanes = 64
    for planes, blocks, stride in ((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)):
        for b in range(blocks):
            s = stride if b == 0 else 1
            out_hw = hw // s
            out[("relu", hw, planes)] += 1            # bn1 at the block input resolution
            out[("relu", out_hw, planes)] += 1        # bn2
            out[("tail+ds" if b == 0 else "tail", out_hw, planes * 4)] += 1
            hw = out_hw
            inplanes = planes * 4
    del inplanes
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args(argv)
    from distributed_pytorch_training_amd import ops

    C_ = ops.native()
    dev = torch.device("cuda")
    cl = torch.channels_last
    print(f"# BatchNorm kernels of the ResNet-50 bf16 step, batch {a.batch}: bytes, time, roofline\n")
    print("| layer kind | HxW | C | count | pass | MB moved | ms | TB/s | % of 6.29 TB/s |")
    print("|---|---|---|---|---|---|---|---|---|")
    tot_ms = tot_roof = 0.0
    below = []
    for (kind, hw, c), count in sorted(resnet50_bn_layers(a.batch).items(), key=lambda kv: (-kv[0][1], kv[0][2])):
        M = a.batch * hw * hw
        mk = lambda: torch.randn(a.batch, c, hw, hw, device=dev, dtype=torch.bfloat16).contiguous(memory_format=cl)
        x, r, dy = mk(), mk(), mk()
        w, bias = torch.ones(c, device=dev), torch.zeros(c, device=dev)
        rm, rv = torch.zeros(c, device=dev), torch.ones(c, device=dev)
        nb = torch.zeros(1, dtype=torch.long, device=dev)
        chunks = (M + 127) // 128
        ps = torch.zeros(c, chunks, device=dev)
        pq = torch.full((c, chunks), float(M) / chunks, device=dev)
        mc = M * c / 1e6   # MB per "MC B" unit: one bf16 activation tensor is 2 MC B
        if kind == "relu":
            f_fwd = lambda: C_.bn_fwd_train(x, None, w, bias, rm, rv, nb, 0.1, 1e-5, True, ps, pq)
            _, mean, invstd, coef = f_fwd()
            f_bwd = lambda: C_.bn_bwd_partials(dy, x, w, mean, invstd, coef, ps, pq, True)
            passes = (4, 6)
        elif kind == "tail":
            f_fwd = lambda: C_.bn_fwd_train(x, r, w, bias, rm, rv, nb, 0.1, 1e-5, True, ps, pq)
            _, mean, invstd, coef = f_fwd()
            f_bwd = lambda: C_.bn_bwd_partials(dy, x, w, mean, invstd, None, ps, pq, True, True)
            passes = (6, 6)
        else:
            def f_fwd():
                _, m1, i1, c1 = C_.bn_fwd_train(x, None, w, bias, rm, rv, nb, 0.1, 1e-5, True, ps, pq, False)
                _, m2, i2, c2 = C_.bn_fwd_train(r, None, w, bias, rm, rv, nb, 0.1, 1e-5, False, ps, pq, False)
                return C_.bn_apply_aff(x, r, c1, c2), m1, i1, m2, i2
            _, mean, invstd, mean2, invstd2 = f_fwd()
            f_bwd = lambda: C_.bn2_bwd_partials(dy, x, r, w, w, mean, invstd, mean2, invstd2, ps, pq, ps, True)
            passes = (6, 10)
        for pname, fn, npass in (("fwd", f_fwd, passes[0]), ("bwd", f_bwd, passes[1])):
            t = time_ms(fn)
            mb = npass * mc
            tbs = mb / t / 1e3
            pct = 100.0 * tbs / HBM_TBS
            tot_ms += t * count
            tot_roof += mb / (HBM_TBS * 1e3) * count
            if pct < 85.0:
                below.append(f"{kind} {hw}x{hw}x{c} {pname} ({pct:.0f} %)")
            print(f"| {kind} | {hw}x{hw} | {c} | {count} | {pname} | {mb:.0f} | {t:.3f} | {tbs:.2f} | {pct:.0f} |",
                  flush=True)
    print(f"\nper step (x count): {tot_ms:.3f} ms of BN chains; HBM roofline of their bytes {tot_roof:.3f} ms "
          f"({100.0 * tot_roof / tot_ms:.0f} % of roofline overall)")
    print("below 85 % of the HBM roofline: " + (", ".join(below) if below else "none"))


if __name__ == "__main__":
    main()
