"""In-step vs isolated time of every convolution pass of the ResNet-50 training step.

The kernel-trace breakdown puts the step's MFMA convolutions at 13.6 ms per step while the
isolated best-of per pass over the same shapes sums to 9.6 ms.  This tool attributes the gap:

* in-step: the training step (bench.py's configuration: ResNet-50, batch 256, bf16, channels_last,
  native engine) with ``ops.conv.profile_calls(True)``: every conv pass records a timing event
  before and after its launches on the stream, tagged (pass, shape, epilogue variant) - forward
  plain / with the BatchNorm-statistics epilogue, backward-weight (its split-K reduce deferred to the
  backward-data launch), backward-data plain / BN+ReLU statistics / block-tail statistics (+ the
  downsample statistic) / stride-2 parity classes, each carrying the backward-weight reduce;
* isolated: the same shape and pass, timed alone in a loop on fresh random tensors with the plain
  epilogue (forward with / without statistics as in the step; backward-weight with its own reduce;
  backward-data plain), median of ``--reps``.

Output: a markdown table per (pass, shape, variant) - calls per step, in-step mean, isolated,
ratio, and the per-step excess (calls x (in-step - isolated)) - sorted by excess, plus totals.
The step is also timed with the events off, so the events' own cost is visible.

    python bench/conv_instep.py --steps 4 > profiles/conv_instep_r4.md
"""
from __future__ import annotations

import argparse
import os
import statistics
import sys
import time
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from distributed_pytorch_training_amd import ops  # noqa: E402
from distributed_pytorch_training_amd.config import parse_args  # noqa: E402
from distributed_pytorch_training_amd.data import SyntheticLoader  # noqa: E402
from distributed_pytorch_training_amd.engine.trainer import Trainer  # noqa: E402
from distributed_pytorch_training_amd.models import build_model  # noqa: E402
from distributed_pytorch_training_amd.ops import conv as C  # noqa: E402
from distributed_pytorch_training_amd.utils.env import setup_miopen_env, setup_tunableop  # noqa: E402


def _step_ms(trainer, batches, n):
    torch.cuda.synchronize()
    t = time.time()
    for i in range(n):
        trainer.train_step(*batches[i % len(batches)])
    torch.cuda.synchronize()
    return 1e3 * (time.time() - t) / n


def _isolated(kind, key, variant, reps, dev):
    ci, h, w, co, r, s, p, out_hw = key
    N = 256
    x = torch.randn(N, ci, h, w, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wt = (0.05 * torch.randn(co, ci, r, r, device=dev)).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    N_ = ops.native()
    ho = out_hw[0] or (h + 2 * p - r) // s + 1
    wo = out_hw[1] or (w + 2 * p - r) // s + 1
    dy = torch.randn(N, co, ho, wo, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    if kind == "fwd":
        fn = lambda: N_.conv_fwd(x, wt, s, p, variant == "stats", *out_hw)
    elif kind == "wgrad":
        fn = lambda: N_.conv_wgrad(dy, x, list(wt.shape), s, p, False)
    elif s == 1:
        fn = lambda: N_.conv_dgrad_flip(dy, wt, p)
    else:
        fn = lambda: N_.conv_dgrad_s2(dy, wt, p, h, w)
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=6)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    setup_miopen_env()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    setup_tunableop()
    args = parse_args(["--model", "resnet50", "--dataset", "synthetic", "--batch-size", "256", "--amp",
                       "--amp-dtype", "bf16", "--channels-last", "--no-cuda-graph"])
    torch.manual_seed(0)
    model = build_model("resnet50", 1000, dev, image_size=224, channels_last=True)
    tr = Trainer(model, args, 0, 1, dev, log=lambda s: None)
    loader = SyntheticLoader(1024, 256, 224, 1000, dev, channels_last=True, pool=4, seed=0)
    batches = list(iter(loader))
    _step_ms(tr, batches, a.warmup)
    off = _step_ms(tr, batches, a.steps)

    C.profile_calls(True)
    torch.cuda.synchronize()
    agg = defaultdict(list)
    t0 = time.time()
    for i in range(a.steps):
        tr.train_step(*batches[i % len(batches)])
    torch.cuda.synchronize()
    on = 1e3 * (time.time() - t0) / a.steps
    for kind, key, variant, e0, e1 in C.take_profile():
        agg[(kind, key, variant)].append(e0.elapsed_time(e1))
    C.profile_calls(False)

    rows = []
    iso_cache = {}
    for (kind, key, variant), ts in agg.items():
        base_variant = variant if kind == "fwd" else "plain"
        ik = (kind, key, base_variant)
        if ik not in iso_cache:
            iso_cache[ik] = _isolated(kind, key, base_variant, a.reps, dev)
        calls = len(ts) / a.steps
        ins = statistics.mean(ts)
        iso = iso_cache[ik]
        rows.append((calls * (ins - iso), kind, key, variant, calls, ins, iso))
    rows.sort(key=lambda r: -r[0])
    print("# Convolutions in the ResNet-50 bf16 b256 training step vs the same pass alone\n")
    print(f"step: {off:.3f} ms/step without events, {on:.3f} ms/step with the per-call events "
          f"({a.steps} steps after {a.warmup} warm-up)\n")
    print("| pass | conv (Cin x HxW -> Cout, k, s) | variant | calls/step | in-step ms | isolated ms | ratio | "
          "excess ms/step |")
    print("|---|---|---|---|---|---|---|---|")
    tot = defaultdict(lambda: [0.0, 0.0])
    for ex, kind, key, variant, calls, ins, iso in rows:
        ci, h, w, co, r, s, p, _ = key
        print(f"| {kind} | {ci}x{h}x{w}->{co} k{r} s{s} | {variant} | {calls:.0f} | {ins:.4f} | {iso:.4f} | "
              f"{ins / iso:.2f} | {ex:+.4f} |")
        tot[kind][0] += calls * ins
        tot[kind][1] += calls * iso
    print()
    for kind, (i, s) in tot.items():
        print(f"{kind}: in-step {i:.3f} ms/step, isolated {s:.3f} ms/step, excess {i - s:+.3f}")
    i = sum(v[0] for v in tot.values())
    s = sum(v[1] for v in tot.values())
    print(f"\nall conv passes: in-step {i:.3f} ms/step, isolated {s:.3f} ms/step, excess {i - s:+.3f} "
          f"({100 * (i - s) / s:.1f} %)")


if __name__ == "__main__":
    main()
