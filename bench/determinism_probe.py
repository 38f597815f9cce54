"""Which fp32 ops of the reference's default workload are not run-to-run deterministic?

fp32 ResNet-18 / 32 px / batch 128 / channels_last, MIOpen convolutions in find mode (the
``train_ddp.py`` default path, which replays as a hipGraph).  ``bench/replay_noise.py`` showed
eager-vs-eager gradient differences of 3e-3 on some steps and ~1e-6 on others: a rounding-level
difference in the FORWARD flips ReLU masks of near-zero activations, which moves a BatchNorm
parameter's gradient by O(1/batch).  This probe runs, from fixed inputs, each of the eleven
convolution shapes' forward / backward-data / backward-weights ``--repeat`` times and reports
the max |difference| to the first run (0 = bitwise deterministic), then the whole fused model's
forward logits and parameter gradients the same way.  Solver choices: run under
``MIOPEN_LOG_LEVEL=5`` and read the "Chosen Algorithm" lines.

    python bench/determinism_probe.py --repeat 6
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

# (name, cin, cout, k, stride, pad, input hw) of the CIFAR-size ResNet-18 with the ImageNet stem
SHAPES = [("conv1", 3, 64, 7, 2, 3, 32), ("l1.3x3", 64, 64, 3, 1, 1, 8),
          ("l2.3x3s2", 64, 128, 3, 2, 1, 8), ("l2.3x3", 128, 128, 3, 1, 1, 4), ("l2.ds", 64, 128, 1, 2, 0, 8),
          ("l3.3x3s2", 128, 256, 3, 2, 1, 4), ("l3.3x3", 256, 256, 3, 1, 1, 2), ("l3.ds", 128, 256, 1, 2, 0, 4),
          ("l4.3x3s2", 256, 512, 3, 2, 1, 2), ("l4.3x3", 512, 512, 3, 1, 1, 1), ("l4.ds", 256, 512, 1, 2, 0, 2)]


def maxdiff(a, b):
    return (a.double() - b.double()).abs().max().item()


def conv_probe(dev, repeat, batch):
    rows = []
    g = torch.Generator(device=dev).manual_seed(1)
    for name, cin, cout, k, st, pad, hw in SHAPES:
        x = torch.randn(batch, cin, hw, hw, device=dev, generator=g).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(cout, cin, k, k, device=dev, generator=g) * (2.0 / (cin * k * k)) ** 0.5
             ).contiguous(memory_format=torch.channels_last)
        ho = (hw + 2 * pad - k) // st + 1
        dy = torch.randn(batch, cout, ho, ho, device=dev, generator=g).contiguous(memory_format=torch.channels_last)
        outs = []
        for _ in range(repeat):
            xx = x.clone().requires_grad_(True)
            ww = w.clone().requires_grad_(True)
            y = F.conv2d(xx, ww, stride=st, padding=pad)
            dx, dw = torch.autograd.grad(y, (xx, ww), dy)
            torch.cuda.synchronize()
            outs.append((y.detach().clone(), dx.clone(), dw.clone()))
        r = {"conv": name}
        for i, part in enumerate(("y", "dx", "dw")):
            r[part] = max(maxdiff(o[i], outs[0][i]) for o in outs[1:])
        rows.append(r)
        print(json.dumps(r), flush=True)
    return rows


def model_probe(dev, repeat, batch):
    from distributed_pytorch_training_amd.config import parse_args
    from distributed_pytorch_training_amd.engine.trainer import Trainer
    from distributed_pytorch_training_amd.models import build_model
    torch.manual_seed(0)
    model = build_model("resnet18", 10, dev, image_size=32, channels_last=True)
    args = parse_args(["--dataset", "synthetic", "--image-size", "32", "--num-classes", "10", "--no-cuda-graph"])
    tr = Trainer(model, args, 0, 1, dev, log=lambda s: None)
    g = torch.Generator(device=dev).manual_seed(5)
    worst = {"logits": 0.0, "grad": 0.0}
    flips = []
    for step in range(repeat):
        x = (torch.randn(batch, 3, 32, 32, device=dev, generator=g) * 4).contiguous(memory_format=torch.channels_last)
        y = torch.randint(0, 10, (batch,), device=dev, generator=g)
        res = []
        for _ in range(3):
            out = tr.module(x)
            loss = F.cross_entropy(out, y)
            grads = torch.autograd.grad(loss, [p for p in tr.module.parameters()])
            torch.cuda.synchronize()
            res.append((out.detach().clone(), torch.cat([t.reshape(-1) for t in grads]).clone()))
        dl = max(maxdiff(r[0], res[0][0]) for r in res[1:])
        dg = max(((r[1] - res[0][1]).double().norm() / res[0][1].double().norm()).item() for r in res[1:])
        worst["logits"] = max(worst["logits"], dl)
        worst["grad"] = max(worst["grad"], dg)
        flips.append({"batch": step, "logits_maxdiff": dl, "grad_rel": dg})
        print(json.dumps(flips[-1]), flush=True)
    return worst


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--repeat", type=int, default=6)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--benchmark", type=int, default=1)
    ap.add_argument("--model-batches", type=int, default=8)
    a = ap.parse_args()
    from distributed_pytorch_training_amd.utils.env import graph_safe_miopen
    graph_safe_miopen()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    torch.backends.cudnn.benchmark = bool(a.benchmark)
    env = {k: v for k, v in os.environ.items() if k.startswith("MIOPEN_DEBUG")}
    print(json.dumps({"env": env}), flush=True)
    conv_probe(dev, a.repeat, a.batch)
    print(json.dumps({"model_worst": model_probe(dev, a.model_batches, a.batch)}), flush=True)


if __name__ == "__main__":
    main()
