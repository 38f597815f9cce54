"""hipGraph replay vs eager on the reference's own default workload.

Configuration = what ``train_ddp.py --dataset synthetic --image-size 32 --num-classes 10`` runs:
ResNet-18, batch 128, fp32 (no --amp), native engine, channels_last, MIOpen convolutions in
``cudnn.benchmark`` mode, SGD 0.1 / 0.9 / 5e-4, seed 42.

Modes:
* ``teacher``: after warmup + capture, every step k starts from ONE state S_k; the replayed
  step and an eager step are both run from S_k (state restored in place between them) and
  their parameters / arena gradients / BN buffers compared per tensor; the run continues
  from the eager result.  Prints per-step relative differences and the worst tensors.
* ``free``: two trainers from the same init, one replaying, one eager, N free-running steps
  on the 4-batch synthetic pool; prints both loss curves (window means).
* ``startup``: wall-clock marks around the warmup steps, the capture and the first replays.

    python bench/graph_parity.py --mode teacher --steps 20
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from distributed_pytorch_training_amd.config import parse_args  # noqa: E402
from distributed_pytorch_training_amd.data import get_dataloaders  # noqa: E402
from distributed_pytorch_training_amd.engine.graph import restore, snapshot  # noqa: E402
from distributed_pytorch_training_amd.engine.trainer import Trainer  # noqa: E402
from distributed_pytorch_training_amd.models import build_model  # noqa: E402
from distributed_pytorch_training_amd.utils.dist import set_seed  # noqa: E402
from distributed_pytorch_training_amd.utils.env import setup_miopen_env, setup_tunableop  # noqa: E402


def _snap(tr):
    return snapshot(tr)


def _restore(tr, snap):
    restore(tr, snap)


def make(argv, dev):
    args = parse_args(argv)
    set_seed(args.seed, 0)
    model = build_model(args.model, args.num_classes, dev, image_size=args.image_size,
                        channels_last=args.channels_last)
    return args, Trainer(model, args, 0, 1, dev, log=print)


def _eager(G, tr, x, y):
    with G._on_stream():
        tr._native_step(x, y)


def teacher(steps: int, extra, repeat: bool = False):
    dev = torch.device("cuda:0")
    args, tr = make(["--dataset", "synthetic", "--image-size", "32", "--num-classes", "10", *extra], dev)
    train, _, _ = get_dataloaders(args, 0, 1, dev)
    assert tr.graphed is not None, "graph replay is not enabled for this configuration"
    G = tr.graphed
    it = iter(train)
    for _ in range(G.warmup + 1):          # warmup + capture (+ first replay)
        x, y = next(it)
        tr.train_step(x, y)
    torch.cuda.synchronize()
    assert G.graph is not None, f"capture failed (failed={G.failed})"
    print(json.dumps({"validation": G.validation}), flush=True)
    names = [n for n in tr.ddp.arena.names] if hasattr(tr.ddp.arena, "names") else None
    worst = []
    rows = []
    for k in range(steps):
        x, y = next(it)
        s0 = _snap(tr)
        tr.train_step(x, y)                 # replay
        torch.cuda.synchronize()
        sg = _snap(tr)
        gg = tr.ddp.arena.grad_flat.detach().clone()
        _restore(tr, s0)
        _eager(G, tr, x, y)                 # eager, same stream, same state
        torch.cuda.synchronize()
        se = _snap(tr)
        ge = tr.ddp.arena.grad_flat.detach().clone()
        rep = {}
        if repeat:   # each path once more from S_k: is either one not deterministic by itself?
            for name, again in (("replay", lambda: tr.train_step(x, y)), ("eager", lambda: _eager(G, tr, x, y))):
                _restore(tr, s0)
                again()
                torch.cuda.synchronize()
                g2 = tr.ddp.arena.grad_flat.detach().clone()
                base = gg if name == "replay" else ge
                rep[name] = (g2 - base).double().norm().item() / max(base.double().norm().item(), 1e-30)
            _restore(tr, s0)
            _eager(G, tr, x, y)
            torch.cuda.synchronize()
        upd = (se["param"] - s0["param"]).double().norm().item()
        dp = (sg["param"] - se["param"]).double().norm().item()
        dg = (gg - ge).double().norm().item() / max(ge.double().norm().item(), 1e-30)
        dbuf = max(((sg[n] - se[n]).double().abs().max().item() if sg[n].is_floating_point()
                    else float((sg[n] != se[n]).any())) for n in se if n.startswith("buf:"))
        row = {"step": k, "rel_param_vs_update": dp / max(upd, 1e-30),
               "rel_param_l2": dp / se["param"].double().norm().item(), "rel_grad": dg,
               "max_buf_diff": dbuf, "metrics_g": sg["metrics"].tolist(), "metrics_e": se["metrics"].tolist()}
        # per-parameter gradient differences
        per = []
        for i, (gv_g, gv_e) in enumerate(zip(tr.ddp.arena.views(gg), tr.ddp.arena.views(ge))):
            ne = gv_e.double().norm().item()
            r = (gv_g - gv_e).double().norm().item() / max(ne, 1e-30)
            per.append((r, names[i] if names else str(i), gv_g.double().norm().item(), ne))
        per.sort(reverse=True)
        if rep:
            row["self_rel_grad"] = rep
        row["worst_grads"] = per[:5]   # (relative difference, name, |replayed grad|, |eager grad|)
        rows.append(row)
        print(json.dumps(row), flush=True)
    return rows


def free(steps: int, extra, arms=("--cuda-graph", "--no-cuda-graph"), task: str = "random"):
    """Free-running loss curves of several arms from the same init; ``arms`` may repeat a mode
    (two eager runs measure the run-to-run spread of the configuration itself)."""
    dev = torch.device("cuda:0")
    curves = {}
    for k, mode in enumerate(arms):
        data = ["--synthetic-task", task] + (["--synthetic-noise", "8"] if task == "prototypes" else [])
        args, tr = make(["--dataset", "synthetic", "--image-size", "32", "--num-classes", "10", mode, *data,
                         *extra], dev)
        train, _, _ = get_dataloaders(args, 0, 1, dev)
        losses = []
        it = iter(train)
        epoch = 0
        for _ in range(steps):
            try:
                x, y = next(it)
            except StopIteration:
                epoch += 1
                train.set_epoch(epoch)
                it = iter(train)
                x, y = next(it)
            _, loss = tr.train_step(x, y)
            losses.append(loss.detach().clone())
        torch.cuda.synchronize()
        name = mode if mode not in curves else f"{mode}#{k}"
        curves[name] = [float(v) for v in torch.stack(losses).cpu()]
        del tr
    w = 25
    names = list(curves)
    print("steps      | " + " | ".join(names), flush=True)
    for i in range(0, steps, w):
        vals = [sum(curves[n][i:i + w]) / len(curves[n][i:i + w]) for n in names]
        print(f"{i:4d}-{i + w - 1:4d}  | " + " | ".join(f"{v:.4f}" for v in vals), flush=True)
    return curves


def startup(extra):
    dev = torch.device("cuda:0")
    t0 = time.time()
    args, tr = make(["--dataset", "synthetic", "--image-size", "32", "--num-classes", "10", *extra], dev)
    train, _, _ = get_dataloaders(args, 0, 1, dev)
    torch.cuda.synchronize()
    print(f"build {time.time() - t0:.2f}s", flush=True)
    it = iter(train)
    for k in range(12):
        x, y = next(it)
        t = time.time()
        tr.train_step(x, y)
        torch.cuda.synchronize()
        g = tr.graphed
        print(f"call {k}: {1e3 * (time.time() - t):9.1f} ms  graph={'yes' if g and g.graph else 'no'}", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["teacher", "free", "startup"], default="teacher")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--extra", default="", help="extra train_ddp flags, space separated")
    ap.add_argument("--arms", default="--cuda-graph,--no-cuda-graph",
                    help="free mode: comma-separated modes, repeats allowed (spread of the configuration)")
    ap.add_argument("--repeat", action="store_true",
                    help="teacher mode: also rerun each path from the same state (self-consistency)")
    ap.add_argument("--task", default="random", choices=["random", "prototypes"])
    a = ap.parse_args()
    setup_miopen_env()
    torch.cuda.set_device(0)
    setup_tunableop()
    torch.backends.cudnn.benchmark = True
    extra = a.extra.split() if a.extra else []
    {"teacher": lambda: teacher(a.steps, extra, a.repeat), "free": lambda: free(a.steps, extra, tuple(a.arms.split(",")), a.task),
     "startup": lambda: startup(extra)}[a.mode]()


if __name__ == "__main__":
    main()
