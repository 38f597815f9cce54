"""Layer-by-layer forward comparison (ResNet-50 bf16): MFMA convs vs MIOpen convs."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_training_amd.config import parse_args  # noqa: E402
from distributed_pytorch_training_amd.engine.trainer import Trainer  # noqa: E402
from distributed_pytorch_training_amd.models import build_model  # noqa: E402
from distributed_pytorch_training_amd.ops import conv as native_conv  # noqa: E402

cuda = torch.device("cuda")
torch.manual_seed(0)
base = build_model("resnet50", 100, cuda, image_size=64, channels_last=True)
common = ["--model", "resnet50", "--dataset", "synthetic", "--amp", "--amp-dtype", "bf16",
          "--channels-last", "--num-classes", "100", "--lr", "0.05"]
tr = {}
tr["nat"] = Trainer(copy.deepcopy(base), parse_args(common), 0, 1, cuda, log=lambda s: None)
tr["mio"] = Trainer(copy.deepcopy(base), parse_args(common + ["--no-native-conv"]), 0, 1, cuda, log=lambda s: None)
rec = {"nat": [], "mio": []}
for k, t in tr.items():
    for n, m in t.module.named_modules():
        if isinstance(m, torch.nn.Conv2d) or isinstance(m, torch.nn.BatchNorm2d):
            def hook(mod, inp, out, n=n, k=k):
                o = out[0] if isinstance(out, tuple) else out
                i = inp[0][0] if isinstance(inp[0], tuple) else inp[0]
                rec[k].append((n, i.detach().float().clone(), o.detach().float().clone()))
            m.register_forward_hook(hook)
g = torch.Generator(device=cuda).manual_seed(7)
x = torch.randn(16, 3, 64, 64, device=cuda, generator=g).contiguous(memory_format=torch.channels_last)
for k, t in tr.items():
    native_conv.ENABLED = k == "nat"
    t.module.train()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        t.module(x)
torch.cuda.synchronize()
for (n, i1, o1), (n2, i2, o2) in zip(rec["nat"], rec["mio"]):
    ri = ((i1 - i2).norm() / i2.norm().clamp_min(1e-30)).item()
    ro = ((o1 - o2).norm() / o2.norm().clamp_min(1e-30)).item()
    print(f"{n:32s} in {ri:.2e} out {ro:.2e} shape {tuple(o1.shape)}")
