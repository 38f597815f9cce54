"""Per-parameter comparison of one ResNet-50 bf16 step: MFMA convs vs MIOpen convs."""
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
nat = Trainer(copy.deepcopy(base), parse_args(common), 0, 1, cuda, log=lambda s: None)
mio = Trainer(copy.deepcopy(base), parse_args(common + ["--no-native-conv"]), 0, 1, cuda, log=lambda s: None)
mio2 = Trainer(copy.deepcopy(base), parse_args(common + ["--no-native-conv"]), 0, 1, cuda, log=lambda s: None)
torch.backends.cudnn.deterministic = True
g = torch.Generator(device=cuda).manual_seed(7)
x = torch.randn(16, 3, 64, 64, device=cuda, generator=g).contiguous(memory_format=torch.channels_last)
y = torch.randint(0, 100, (16,), device=cuda, generator=g)
native_conv.ENABLED = True
_, l1 = nat.train_step(x, y)
native_conv.ENABLED = False
_, l2 = mio.train_step(x, y)
_, l3 = mio2.train_step(x, y)
torch.cuda.synchronize()
print("loss mio2", l3.item())
print("loss", l1.item(), l2.item(), "scale", nat.scaler.get_scale(), mio.scaler.get_scale(),
      "found_inf", nat.scaler.found_inf.item(), mio.scaler.found_inf.item())
for (n, a), b, b2, c in zip(nat.module.named_parameters(), mio.module.parameters(), mio2.module.parameters(),
                           base.parameters()):
    ua, ub, ub2 = (a - c).double(), (b - c).double(), (b2 - c).double()
    print(f"{n:40s} |upd_nat| {ua.norm().item():.4e} |upd_mio| {ub.norm().item():.4e} "
          f"rel(nat,mio) {((ua - ub).norm() / ub.norm().clamp_min(1e-30)).item():.3e} "
          f"rel(mio2,mio) {((ub2 - ub).norm() / ub.norm().clamp_min(1e-30)).item():.3e}")
