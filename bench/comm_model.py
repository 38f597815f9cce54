"""Exposed-communication estimate for N = 2 / 4 / 8 MI355X from a measured 1-GPU backward.

One MI355X can not run RCCL at N > 1, but the part of the gradient-sync cost that depends on
the model - WHEN each bucket becomes ready during backward - is a single-GPU property.  This
tool measures it and prices the collectives with a stated link model:

1. train ``--model`` at the bench config on one GPU with the native engine, the reducer's
   collective path forced on over a 1-rank RCCL communicator (``DPT_FORCE_COLLECTIVES=1``:
   a 1-rank all-reduce is an identity, so each bucket's comm-stream start event marks the
   moment the bucket became ready) and per-bucket events on (``NativeDDP.set_profile``);
2. read, per profiled step, every bucket's ready time relative to the first gradient and the
   backward end (``Reducer.bucket_start_ms`` / ``step_times_ms``), medians over the window;
3. replay the comm stream for N ranks: bucket b starts at max(ready_b, end_{b-1}) and takes
   ``T(S, N) = 2(N-1)·alpha + 2(N-1)/N · S / busbw(N)`` (ring all-reduce); exposed comm =
   last end - backward end, busy = sum of T.

Link model: 7 xGMI links per GPU at ~153 GB/s each, fully connected.  Two
bounds are printed - ``1-link``: every ring step runs on a single link (one channel's view,
busbw = eff x 153 GB/s for every N); ``all-links``: RCCL's channels spread over all links
among the N GPUs (busbw = eff x (N-1) x 153 GB/s) - with eff = 0.7 and alpha = 5 us per ring
step.  These are estimates, not measurements; the driver's 8-GPU bench line reports the
measured ``pct_step_allreduce`` / ``pct_step_exposed_comm`` for the same quantities.

Usage (GPU): ``python bench/comm_model.py --model resnet50 --batch-size 256 --last-bucket-mb 0 1``
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

LINK_GBS = 153.0
EFF = 0.7
ALPHA_US = 5.0


def ring_ms(size_bytes: float, n: int, busbw_gbs: float, alpha_us: float = ALPHA_US) -> float:
    if n <= 1:
        return 0.0
    return 1e3 * (2 * (n - 1) * alpha_us * 1e-6 + 2 * (n - 1) / n * size_bytes / (busbw_gbs * 1e9))


def simulate(ready_ms, sizes_bytes, bwd_end_ms, n, busbw_gbs, alpha_us=ALPHA_US):
    """Serial comm stream: returns (busy_ms, exposed_ms, end_ms)."""
    end = 0.0
    busy = 0.0
    for r, s in zip(ready_ms, sizes_bytes):
        t = ring_ms(s, n, busbw_gbs, alpha_us)
        start = max(r, end)
        end = start + t
        busy += t
    return busy, max(0.0, end - bwd_end_ms), end


def busbw(n: int, mode: str) -> float:
    return EFF * LINK_GBS * (1 if mode == "1-link" else max(1, n - 1))


def measure(model_name: str, batch: int, image: int, last_mb: float, steps: int, warmup: int):
    os.environ["DPT_FORCE_COLLECTIVES"] = "1"
    import torch

    from distributed_pytorch_training_amd.config import parse_args
    from distributed_pytorch_training_amd.engine.trainer import Trainer
    from distributed_pytorch_training_amd.models import build_model
    from distributed_pytorch_training_amd.parallel.comm import make_comm
    from distributed_pytorch_training_amd.utils.env import setup_miopen_env, setup_tunableop

    setup_miopen_env()
    setup_tunableop()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    args = parse_args(["--model", model_name, "--dataset", "synthetic", "--batch-size", str(batch),
                       "--image-size", str(image), "--num-classes", "1000", "--amp", "--amp-dtype", "bf16",
                       "--channels-last", "--no-cuda-graph", "--last-bucket-mb", str(last_mb)])
    torch.manual_seed(0)
    model = build_model(model_name, 1000, dev, image_size=image, channels_last=True)
    tr = Trainer(model, args, 0, 1, dev, comm=make_comm(dev, 0, 1), log=lambda s: None)
    # the 1-rank run does not rebuild buckets by itself (no peers): rebuild like a multi-rank run
    tr.ddp.rebuild_buckets = True
    x = torch.randn(batch, 3, image, image, device=dev).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (batch,), device=dev)
    for _ in range(warmup):
        tr.train_step(x, y)
    tr.ddp.set_profile(True, slots=steps + 1)
    tr.train_step(x, y)
    torch.cuda.synchronize()
    recs = []
    for _ in range(steps):
        tr.train_step(x, y)
        torch.cuda.synchronize()
        p = tr.ddp.comm_profile()
        recs.append(p)
    B = len(recs[0]["bucket_start_ms"])
    ready = [statistics.median(r["bucket_start_ms"][b] for r in recs) for b in range(B)]
    bwd = statistics.median(r["step_ms"][0] for r in recs)
    sizes = [m * 1024 * 1024 for m in tr.ddp.bucket_sizes_mib()]
    # step time without collectives (1 GPU), for the percentage
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(steps):
        tr.train_step(x, y)
    ev1.record()
    torch.cuda.synchronize()
    step_ms = ev0.elapsed_time(ev1) / steps
    tr.close()
    return {"model": model_name, "batch": batch, "image": image, "last_bucket_mb": last_mb,
            "buckets_mib": [round(s / 2**20, 3) for s in sizes], "ready_ms": [round(r, 3) for r in ready],
            "bwd_end_ms": round(bwd, 3), "step_ms_1gpu": round(step_ms, 3)}


def table(m: dict) -> str:
    lines = [f"### {m['model']} batch {m['batch']} / {m['image']} px, last-bucket cap "
             f"{m['last_bucket_mb']} MiB",
             "",
             f"1-GPU step {m['step_ms_1gpu']:.2f} ms; first gradient -> backward end {m['bwd_end_ms']:.2f} ms",
             "",
             "| bucket | MiB | ready (ms after first grad) |",
             "|---|---|---|"]
    for b, (s, r) in enumerate(zip(m["buckets_mib"], m["ready_ms"])):
        lines.append(f"| {b} | {s:.2f} | {r:.3f} |")
    lines += ["", "| N | link model | busbw GB/s | all-reduce busy ms | % of step | exposed ms | % of step |",
              "|---|---|---|---|---|---|---|"]
    sizes = [s * 2**20 for s in m["buckets_mib"]]
    for n in (2, 4, 8):
        for mode in ("1-link", "all-links"):
            bw = busbw(n, mode)
            busy, exp, _ = simulate(m["ready_ms"], sizes, m["bwd_end_ms"], n, bw)
            step = m["step_ms_1gpu"] + exp
            lines.append(f"| {n} | {mode} | {bw:.0f} | {busy:.3f} | {100 * busy / step:.1f} | {exp:.3f} | "
                         f"{100 * exp / step:.1f} |")
    return "\n".join(lines) + "\n"


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch-size", type=int, default=256)
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--last-bucket-mb", type=float, nargs="+", default=[0.0, 1.0])
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--from-json", default=None, help="re-price a saved measurement (CPU)")
    a = ap.parse_args(argv)
    if a.from_json:
        with open(a.from_json) as f:
            ms = [json.loads(l) for l in f if l.strip()]
    else:
        ms = [measure(a.model, a.batch_size, a.image_size, c, a.steps, a.warmup) for c in a.last_bucket_mb]
        if a.json_out:
            with open(a.json_out, "a") as f:
                for m in ms:
                    f.write(json.dumps(m) + "\n")
    for m in ms:
        print(table(m))
    return 0


if __name__ == "__main__":
    sys.exit(main())
