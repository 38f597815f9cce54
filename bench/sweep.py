"""Benchmark sweeps that produce the reference README's promised tables (README.md:27-35):

* throughput vs batch size          (--table batch)
* AMP vs FP32                        (--table amp)
* native vs stock PyTorch engine     (--table impl)
* bucket-size sweep (ViT-B/16 / ResNet-50, multi-GPU under torchrun)   (--table bucket)

Each configuration runs ``bench.py`` in-process-isolated subprocesses (fresh CUDA context
per point so MIOpen/allocator state does not leak between points) and appends JSON lines to
``--out``; ``--markdown`` renders a table from such a file.

    python bench/sweep.py --table batch --out gpurun_out/sweep_batch.jsonl
    python bench/sweep.py --markdown gpurun_out/sweep_batch.jsonl
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

TABLES = {
    "batch": [["--batch-size", str(b)] for b in (64, 128, 256, 512)],
    "amp": [[], ["--no-amp"], ["--amp-dtype", "fp16"]],
    "impl": [[], ["--impl", "torch"], ["--no-fused-bn"]],
    "bucket": [["--bucket-cap-mb", str(c)] for c in (8, 25, 50, 100, 400)],
    "vit": [["--model", "vit_b_16", "--batch-size", "128", "--no-channels-last"]],
}


def run_point(extra, steps, warmup, out, timeout, launcher=None, find=True):
    # --find: MIOpen find mode (cudnn.benchmark).  Off = immediate mode over the shipped find-db
    # (bf16 shapes); fp32 shapes then use MIOpen's heuristics instead of minutes of searching.
    cmd = (launcher or [sys.executable]) + [os.path.join(ROOT, "bench.py"), "--steps", str(steps),
                                            "--warmup", str(warmup), "--json-out", out] + \
        (["--find"] if find else []) + extra
    print("+", " ".join(cmd), flush=True)
    r = subprocess.run(cmd, cwd=ROOT, timeout=timeout)
    return r.returncode


def markdown(path):
    rows = [json.loads(l) for l in open(path) if l.strip()]
    print("| model | impl | dtype | fused BN | per-GPU batch | GPUs | bucket MiB | images/s | ms/step | vs stock |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for r in rows:
        c = r["config"]
        vs = r.get("vs_baseline")
        print(f"| {c['model']} | {c['impl']} | {r['dtype']} | {c.get('fused_bn', '')} | {c['per_gpu_batch']} | "
              f"{r['n_gpus']} | {c['bucket_cap_mb']} | {r['value']:.0f} | {r['ms_per_step']:.2f} | "
              f"{'' if vs is None else f'{vs:.3f}'} |")


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--table", choices=sorted(TABLES))
    ap.add_argument("--out", default="gpurun_out/sweep.jsonl")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--timeout", type=int, default=600)
    ap.add_argument("--no-find", action="store_true", help="MIOpen immediate mode (no find-mode search)")
    ap.add_argument("--extra", default="", help="extra bench.py args for every point")
    ap.add_argument("--nproc", type=int, default=1, help=">1: launch each point with torch.distributed.run")
    ap.add_argument("--markdown", default=None)
    a = ap.parse_args(argv)
    if a.markdown:
        markdown(a.markdown)
        return 0
    launcher = None
    if a.nproc > 1:
        launcher = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.nproc}",
                    "--master-addr", "127.0.0.1", "--master-port", "29561"]
    rc = 0
    for extra in TABLES[a.table]:
        rc |= run_point(extra + a.extra.split(), a.steps, a.warmup, a.out, a.timeout, launcher, not a.no_find)
        if rc:
            break
    return rc


if __name__ == "__main__":
    sys.exit(main())
