"""Training-outcome parity: the native engine vs stock PyTorch through the reference's own script.

Runs ``train_ddp.py`` (the reference's CLI, stdout step lines and ``metrics_rank0.csv``) twice per
configuration - ``--impl native`` and ``--impl torch`` - with the same seed on the learnable
synthetic task (``--synthetic-task prototypes``: class prototype images plus fresh pixel noise every
step, held-out validation from the same prototypes), and reports per-epoch train/val loss and
accuracy side by side, plus the step-line throughput of both engines (the reference's definition,
train_ddp.py:224-242, ``--ref-throughput`` on the native side) - the same-harness table.

    python bench/train_parity.py --config r18_fp32 --epochs 5 --steps-per-epoch 100 --out profiles/...
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CONFIGS = {
    # the reference's default run (ResNet-18, 32x32, 10 classes, batch 128, fp32)
    "r18_fp32": ["--model", "resnet18", "--image-size", "32", "--num-classes", "10", "--batch-size", "128"],
    # the reference's --amp (fp16 autocast + GradScaler)
    "r18_amp_fp16": ["--model", "resnet18", "--image-size", "32", "--num-classes", "10", "--batch-size", "128",
                     "--amp"],
    # the flagship model under bf16 autocast (10 classes, lr 0.02: at 100 classes / lr 0.05 neither
    # engine left chance level in 500 steps - profiles/train_parity_r4.md)
    "r50_bf16": ["--model", "resnet50", "--image-size", "64", "--num-classes", "10", "--batch-size", "128",
                 "--amp", "--amp-dtype", "bf16", "--lr", "0.02"],
}

# pixel noise std against unit-std prototypes, per config: the classes separate only through the
# prototypes' low-frequency structure; the nearest-prototype (Bayes) accuracy is ~87 % for 10
# classes at 32x32 with noise 20 (64x64: 4x the pixels to average over, so noise 32 keeps the task
# about as hard), so the curves take hundreds of steps to flatten and the held-out accuracy
# measures generalisation.
NOISE = {"r18_fp32": 20.0, "r18_amp_fp16": 20.0, "r50_bf16": 32.0}

STEP_RE = re.compile(r"Epoch \[(\d+)\] Step \[(\d+)/(\d+)\] Loss: ([\d.]+)  Acc: ([\d.]+)%  "
                     r"Throughput: ([\d.]+) samples/s")


def run(config: str, impl: str, epochs: int, steps_per_epoch: int, out_dir: str, extra=(), timeout=1800):
    argv = CONFIGS[config]
    bs = int(argv[argv.index("--batch-size") + 1])
    cmd = [sys.executable, os.path.join(ROOT, "train_ddp.py"), "--dataset", "synthetic",
           "--synthetic-task", "prototypes", "--synthetic-train-size", str(bs * steps_per_epoch),
           "--synthetic-val-size", str(bs * 20), "--epochs", str(epochs), "--print-freq", "25",
           "--synthetic-noise", str(NOISE[config]), "--output-dir", out_dir, "--impl", impl, *argv, *extra]
    if impl == "native":
        cmd.append("--ref-throughput")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    # stream the run's lines to our stderr as they come (a long MIOpen find must not look hung)
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env, cwd=ROOT)
    lines = []
    for line in p.stdout:
        lines.append(line)
        print(f"[{config}/{impl}] {line}", end="", file=sys.stderr, flush=True)
    rc = p.wait(timeout=timeout)
    out = "".join(lines)
    if rc != 0:
        raise RuntimeError(f"{config}/{impl} failed ({rc}):\n{out[-4000:]}")
    with open(os.path.join(out_dir, "metrics_rank0.csv")) as f:
        rows = list(csv.DictReader(f))
    steps = [dict(zip(("epoch", "step", "n", "loss", "acc", "thr"), map(float, m.groups())))
             for m in STEP_RE.finditer(out)]
    return {"config": config, "impl": impl, "epochs": [{k: float(v) for k, v in row.items()} for row in rows],
            "steps": steps, "stdout": out}


def compare(config: str, epochs: int, steps_per_epoch: int, extra=()):
    out = {}
    with tempfile.TemporaryDirectory() as td:
        for impl in ("native", "torch"):
            d = os.path.join(td, impl)
            os.makedirs(d)
            out[impl] = run(config, impl, epochs, steps_per_epoch, d, extra)
            last = out[impl]["epochs"][-1]
            print(f"[train_parity] {config} {impl}: val acc {last['val_acc']:.2f} %", file=sys.stderr, flush=True)
    return out


def _thr(res, skip_epochs=1):
    """Mean step-line throughput after the first epoch (MIOpen find / capture / warm-up there)."""
    v = [s["thr"] for s in res["steps"] if s["epoch"] > skip_epochs]
    return sum(v) / len(v) if v else float("nan")


def markdown(config: str, res, extra=()) -> str:
    nat, ref = res["native"], res["torch"]
    flags = " ".join([*CONFIGS[config], *extra])
    lines = [f"## {config}: `train_ddp.py {flags} --dataset synthetic --synthetic-task prototypes`",
             "", "| epoch | train loss native / torch | train acc % native / torch | val loss native / torch | "
             "val acc % native / torch | epoch s native / torch |", "|---|---|---|---|---|---|"]
    for a, b in zip(nat["epochs"], ref["epochs"]):
        lines.append(f"| {int(a['epoch'])} | {a['train_loss']:.4f} / {b['train_loss']:.4f} | "
                     f"{a['train_acc']:.2f} / {b['train_acc']:.2f} | {a['val_loss']:.4f} / {b['val_loss']:.4f} | "
                     f"{a['val_acc']:.2f} / {b['val_acc']:.2f} | {a['epoch_time_seconds']:.2f} / "
                     f"{b['epoch_time_seconds']:.2f} |")
    tn, tt = _thr(nat), _thr(ref)
    lines += ["", f"step-line throughput after epoch 1 (reference definition, samples/s): native {tn:,.0f}, "
                  f"torch {tt:,.0f} ({tn / tt:.2f}x)", ""]
    return "\n".join(lines)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", action="append", choices=sorted(CONFIGS), required=True)
    ap.add_argument("--epochs", type=int, default=5)
    ap.add_argument("--steps-per-epoch", type=int, default=100)
    ap.add_argument("--json", default=None, help="append the raw results as JSON lines here")
    ap.add_argument("--extra", default="", help="more train_ddp.py flags, space separated (later flags win)")
    a = ap.parse_args()
    extra = a.extra.split() if a.extra else []
    for c in a.config:
        res = compare(c, a.epochs, a.steps_per_epoch, extra)
        print(markdown(c, res, extra), flush=True)
        if a.json:
            with open(a.json, "a") as f:
                for impl in ("native", "torch"):
                    r = dict(res[impl])
                    r.pop("stdout")
                    f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
