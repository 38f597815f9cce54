"""Training outcome with statistical power (VERDICT r4 next #3b): several seeds per engine.

``train_ddp.py`` (the reference's script) with ``--impl native`` and ``--impl torch`` on the
learnable synthetic task (bench/train_parity.py), one run per (seed, engine); reports every run's
final validation accuracy / loss and each engine's mean +- std, and the engine gap in units of
the pooled std.  A configuration is "stable" when no run diverges: ResNet-50 bf16 at lr 0.01 for
1,000 steps (10 epochs x 100).

    python bench/train_parity_seeds.py --config r50_bf16 --seeds 1 2 3 4 5 --epochs 10 --extra "--lr 0.01"
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import train_parity  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="r50_bf16", choices=sorted(train_parity.CONFIGS))
    ap.add_argument("--seeds", type=int, nargs="+", default=[1, 2, 3, 4, 5])
    ap.add_argument("--epochs", type=int, default=10)
    ap.add_argument("--steps-per-epoch", type=int, default=100)
    ap.add_argument("--extra", default="--lr 0.01")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    extra = a.extra.split() if a.extra else []
    res = {"native": [], "torch": []}
    for seed in a.seeds:
        for impl in ("native", "torch"):
            with tempfile.TemporaryDirectory() as td:
                r = train_parity.run(a.config, impl, a.epochs, a.steps_per_epoch, td, [*extra, "--seed", str(seed)])
            ep = r["epochs"]
            row = {"seed": seed, "impl": impl, "final_val_acc": ep[-1]["val_acc"], "final_val_loss": ep[-1]["val_loss"],
                   "final_train_loss": ep[-1]["train_loss"], "epoch1_val_loss": ep[0]["val_loss"],
                   "epoch1_val_acc": ep[0]["val_acc"], "thr": train_parity._thr(r),
                   "curve_val_acc": [e["val_acc"] for e in ep], "curve_train_loss": [e["train_loss"] for e in ep]}
            res[impl].append(row)
            print(json.dumps(row), flush=True)
            if a.json:
                with open(a.json, "a") as f:
                    f.write(json.dumps({"config": a.config, "extra": extra, **row}) + "\n")
    print(markdown(a.config, extra, res, a.epochs * a.steps_per_epoch))


def _ms(v):
    return statistics.mean(v), (statistics.stdev(v) if len(v) > 1 else 0.0)


def markdown(config, extra, res, steps) -> str:
    flags = " ".join([*train_parity.CONFIGS[config], *extra])
    lines = [f"## {config}, {steps} steps: `train_ddp.py {flags} --dataset synthetic --synthetic-task prototypes`",
             "", "| seed | native val acc % | torch val acc % | native val loss | torch val loss | "
             "native epoch-1 val loss | torch epoch-1 val loss |", "|---|---|---|---|---|---|---|"]
    for n, t in zip(res["native"], res["torch"]):
        lines.append(f"| {n['seed']} | {n['final_val_acc']:.2f} | {t['final_val_acc']:.2f} | "
                     f"{n['final_val_loss']:.4f} | {t['final_val_loss']:.4f} | {n['epoch1_val_loss']:.3f} | "
                     f"{t['epoch1_val_loss']:.3f} |")
    out = ["", "| metric | native mean +- std | torch mean +- std | gap / pooled std |", "|---|---|---|---|"]
    for key in ("final_val_acc", "final_val_loss", "final_train_loss"):
        mn, sn = _ms([r[key] for r in res["native"]])
        mt, st = _ms([r[key] for r in res["torch"]])
        pooled = ((sn ** 2 + st ** 2) / 2) ** 0.5
        out.append(f"| {key} | {mn:.4f} +- {sn:.4f} | {mt:.4f} +- {st:.4f} | "
                   f"{(mn - mt) / pooled if pooled > 0 else float('nan'):+.2f} |")
    return "\n".join(lines + out)


if __name__ == "__main__":
    main()
