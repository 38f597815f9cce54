"""Debug: which fused layer breaks whole-network parity?  fp32, fp64 reference."""
import copy
import sys

import torch

sys.path.insert(0, ".")
from distributed_pytorch_training_amd.models import build_model
from distributed_pytorch_training_amd.models.layers import fuse_batchnorm, fuse_native_layers, FusedMaxPool2d
import torch.nn as nn


def rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm()).item()


dev = torch.device("cuda")
for batch in (8, 32):
    torch.manual_seed(0)
    ref = build_model("resnet50", 100, dev, image_size=64, channels_last=True)
    f64 = copy.deepcopy(ref).double()
    x = torch.randn(batch, 3, 64, 64, device=dev).contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        y64 = f64(x.double())
        for name in ("stock", "bn", "pool", "both"):
            m = copy.deepcopy(ref)
            if name == "bn":
                fuse_batchnorm(m)
            elif name == "pool":
                m.maxpool.__class__ = FusedMaxPool2d
            elif name == "both":
                fuse_native_layers(m)
            y = m(x)
            y = y[0] if isinstance(y, tuple) else y
            # stem-only probe
            s_ref = f64.maxpool(f64.relu(f64.bn1(f64.conv1(x.double()))))
            print(f"batch {batch} {name:6s} out rel {rel(y, y64):.3e}", flush=True)
    # stem stage probe in train mode
    m = copy.deepcopy(ref)
    fuse_native_layers(m)
    with torch.no_grad():
        a = m.conv1(x)
        from distributed_pytorch_training_amd.models.layers import bn_act
        s1 = bn_act(m.bn1, a)
        p1 = m.maxpool(s1)
        r = copy.deepcopy(ref)
        s1r = torch.relu(r.bn1(r.conv1(x)))
        p1r = r.maxpool(s1r)
        print("stem bn+relu rel", rel(s1, s1r), "pool rel", rel(p1, p1r), "pool-on-same-input rel",
              rel(m.maxpool(s1r), r.maxpool(s1r)), flush=True)
        l1 = m.layer1(p1r)
        l1 = l1[0] if isinstance(l1, tuple) else l1
        l1r = r.layer1(p1r)
        print("layer1 rel", rel(l1, l1r), flush=True)
