"""Diagnostics for the folded downsample-BN block tail (ops/bn.py _BN2AddReLUPair): per-tensor
max errors of fused vs unfused, with and without the dgrad-epilogue statistics (BNR)."""
import copy

import torch

from distributed_pytorch_training_amd.models.layers import FusedBatchNorm2d
from distributed_pytorch_training_amd.ops import bn as fbn
from distributed_pytorch_training_amd.ops import conv as nc

CL = torch.channels_last
cuda = torch.device("cuda")
g = torch.Generator(device=cuda).manual_seed(9)
N, Cin, C4, C, HW = 4, 128, 256, 64, 14


def t(*s, scale=1.0):
    return torch.randn(*s, device=cuda, generator=g) * scale


x0 = t(N, Cin, HW, HW).to(torch.bfloat16).contiguous(memory_format=CL)
w3 = t(C4, Cin, 1, 1, scale=0.08).to(torch.bfloat16).contiguous(memory_format=CL)
wd = t(C4, Cin, 1, 1, scale=0.08).to(torch.bfloat16).contiguous(memory_format=CL)
w1 = t(C, C4, 1, 1, scale=0.06).to(torch.bfloat16).contiguous(memory_format=CL)
gy = t(N, C, HW, HW).to(torch.bfloat16).contiguous(memory_format=CL)
wv = t(C4, C4, 1, 1, scale=0.06).to(torch.bfloat16).contiguous(memory_format=CL)
gv = t(N, C4, HW, HW).to(torch.bfloat16).contiguous(memory_format=CL)
bns0 = []
for c in (C4, C4, C):
    m = FusedBatchNorm2d(c).to(cuda)
    with torch.no_grad():
        m.weight.uniform_(0.5, 1.5, generator=g)
        m.bias.uniform_(-0.3, 0.3, generator=g)
    bns0.append(m)
names = ["yc", "x.grad", "w3.grad", "wd.grad", "w1.grad", "wv.grad"] + [f"bn{i}.{n}" for i in range(3) for n in ("w", "b")]


def run(fused, bnr):
    nc.BN_BWD_FUSE = bnr
    bns = [copy.deepcopy(m) for m in bns0]
    xi = x0.detach().clone().requires_grad_(True)
    ps = [v.detach().clone().requires_grad_(True) for v in (w3, wd, w1, wv)]
    h3 = nc.conv2d(xi, ps[0], 1, 0, bn_stats=True)
    hd = nc.conv2d(xi, ps[1], 1, 0, bn_stats=True)
    if fused:
        yc, yi = fbn.bn2_add_relu_train(h3, bns[0], hd, bns[1])
    else:
        ident = bns[1].act(hd, False, None)
        yc, yi = bns[0].act(h3, True, ident, pair=True)
    u = bns[2].act(nc.conv2d(yc, ps[2], 1, 0, bn_stats=True), True, None)
    v = nc.conv2d(yi, ps[3], 1, 0)
    torch.autograd.backward([u, v], [gy, gv])
    nc.BN_BWD_FUSE = True
    return [yc.detach().float(), xi.grad.float()] + [p.grad.float() for p in ps] + \
        [v.grad.float() for m in bns for v in (m.weight, m.bias)]


ref = run(False, False)
for fused, bnr in ((False, True), (True, False), (True, True)):
    out = run(fused, bnr)
    print(f"fused={fused} bnr={bnr}")
    for n, a, b in zip(names, out, ref):
        d = (a - b).abs()
        print(f"  {n:10s} maxabs {d.max().item():.4g}  ref max {b.abs().max().item():.4g}  frac>2% {(d > 0.02 * b.abs().max()).float().mean().item():.4f}")
yf, yu = run(True, True)[0], ref[0]
print("mask flips:", ((yf > 0) != (yu > 0)).sum().item(), "of", yf.numel())
