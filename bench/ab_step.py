"""Same-process A/B of kernel-library setters on the headline training step (ResNet-50, bf16,
batch 256, synthetic data): one Trainer, arms interleaved over rounds (cdna_hip_programming.md
§5.4 rule 24 - cross-process runs add variance that looks like a kernel property).

    python bench/ab_step.py --arm base= --arm hb3=conv_set_halo:3 --reset conv_set_halo:1 --rounds 4

An arm is NAME=setter:value[,setter:value...] (setters of the native module, e.g.
conv_set_halo, conv_set_splitk, conv_set_variant, or a dotted Python module attribute such as
distributed_pytorch_training_amd.ops.conv.CONCURRENT_WGRAD_MAX_PIXELS); an empty list is the
default configuration.  --reset setter:value pairs are applied before every arm (give one for
each setter an arm changes, so the next arm starts from the default).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def parse_arm(spec: str):
    name, _, rest = spec.partition("=")
    sets = []
    for item in filter(None, rest.split(",")):
        fn, _, val = item.partition(":")
        sets.append((fn, tuple(int(v) for v in val.split("/"))))  # "fn:a/b/c" -> fn(a, b, c)
    return name, sets


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--arm", action="append", required=True)
    ap.add_argument("--reset", action="append", default=[], help="setter:value applied before every arm")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch-size", type=int, default=256)
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--image-size", type=int, default=224)
    a = ap.parse_args(argv)

    from distributed_pytorch_training_amd import ops
    from distributed_pytorch_training_amd.config import parse_args
    from distributed_pytorch_training_amd.data import SyntheticLoader
    from distributed_pytorch_training_amd.engine.trainer import Trainer
    from distributed_pytorch_training_amd.models import build_model
    from distributed_pytorch_training_amd.utils.env import setup_miopen_env, setup_tunableop

    setup_miopen_env()
    C = ops.native()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    setup_tunableop()
    args = parse_args(["--model", a.model, "--dataset", "synthetic", "--batch-size", str(a.batch_size),
                       "--image-size", str(a.image_size), "--amp", "--amp-dtype", "bf16", "--channels-last",
                       "--no-cuda-graph", "--lr", "0.1", "--momentum", "0.9", "--weight-decay", "5e-4"])
    torch.manual_seed(0)
    model = build_model(a.model, 1000, dev, image_size=a.image_size, channels_last=True)
    tr = Trainer(model, args, 0, 1, dev, log=lambda s: None)
    loader = SyntheticLoader(a.batch_size * 4, a.batch_size, a.image_size, 1000, dev, channels_last=True, pool=4,
                             seed=0)
    batches = list(iter(loader))
    arms = [parse_arm(s) for s in a.arm]
    resets = [parse_arm("r=" + r)[1][0] for r in a.reset]

    import importlib

    def set_one(fn, v):
        # "module.path.ATTR" sets a Python module attribute, anything else a native setter
        if "." in fn:
            mod, _, attr = fn.rpartition(".")
            setattr(importlib.import_module(mod), attr, v[0])
        else:
            getattr(C, fn)(*v)

    def apply(sets):
        for fn, v in resets:
            set_one(fn, v)
        for fn, v in sets:
            set_one(fn, v)

    def run(n):
        for i in range(n):
            x, y = batches[i % len(batches)]
            tr.train_step(x, y)

    times = {name: [] for name, _ in arms}
    for name, sets in arms:  # warm every arm once (kernel loads, first-use allocations)
        apply(sets)
        run(a.warmup)
    torch.cuda.synchronize()
    for rnd in range(a.rounds):
        order = arms if rnd % 2 == 0 else arms[::-1]
        for name, sets in order:
            apply(sets)
            run(2)
            torch.cuda.synchronize()
            t0 = time.time()
            run(a.steps)
            torch.cuda.synchronize()
            times[name].append(1e3 * (time.time() - t0) / a.steps)
    apply([])
    out = {name: {"ms_median": statistics.median(v), "ms_min": min(v),
                  "img_s_median": a.batch_size * 1e3 / statistics.median(v), "ms_all": [round(t, 3) for t in v]}
           for name, v in times.items()}
    print(json.dumps({"tool": "ab_step", "model": a.model, "batch": a.batch_size, "arms": out}))


if __name__ == "__main__":
    main()
