"""Cost of the BN-statistics epilogue of the forward conv, per ResNet-50 conv shape (batch 256):
conv_fwd without / with statistics.  Run once plain and once with DPT_CONV_NO_PSTORE=1 (the
statistics are computed but their partials not stored) to split the epilogue's cost into the
partial stores and the rest."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench.conv_roofline import resnet50_convs, time_ms  # noqa: E402
from distributed_pytorch_training_amd import ops  # noqa: E402

C_ = ops.native()
dev = torch.device("cuda")
cl = torch.channels_last
tag = "nostore" if os.environ.get("DPT_CONV_NO_PSTORE") else "store"
tot0 = tot1 = 0.0
for (cin_hw, cout, k, s, p), count in resnet50_convs(256, 224).items():
    cin, h, w = cin_hw
    if cin % 64 or cout % 64:
        continue
    x = torch.randn(256, cin, h, w, device=dev, dtype=torch.bfloat16).contiguous(memory_format=cl)
    wt = (torch.randn(cout, cin, *k, device=dev, dtype=torch.bfloat16) * 0.05).contiguous(memory_format=cl)
    t0 = time_ms(lambda: C_.conv_fwd(x, wt, s[0], p[0], False))
    t1 = time_ms(lambda: C_.conv_fwd(x, wt, s[0], p[0], True))
    tot0 += t0 * count
    tot1 += t1 * count
    print(f"{tag} {cin}x{h}x{w}->{cout} k{k[0]} s{s[0]} x{count}: plain {t0:.4f} stats {t1:.4f} (+{100 * (t1 / t0 - 1):.0f}%)",
          flush=True)
print(f"{tag} total per step: plain {tot0:.3f} ms, stats {tot1:.3f} ms")
