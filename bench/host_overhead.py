"""Is the headline step host-bound anywhere?  (ResNet-50, bf16, batch 256, native engine.)

A kernel trace of the step (profiles/host_gaps_r5.md) shows the GPU idle for 0.3-0.9 ms per step
around the forward -> backward transition: the loss, the first backward kernels and the FC's GEMM
arrive 15-190 us apart.  This probe times the host side of each phase without synchronising
(forward call, loss, backward call, optimizer + metrics) against the GPU step time, then runs the
forward under cProfile to rank the Python-side cost per call site.

    python bench/host_overhead.py [--steps 20] [--profile-steps 5] [--out gpurun_out/host.txt]
"""
from __future__ import annotations

import argparse
import cProfile
import io
import os
import pstats
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--profile-steps", type=int, default=5)
    ap.add_argument("--batch-size", type=int, default=256)
    ap.add_argument("--out", default="")
    a = ap.parse_args(argv)

    from distributed_pytorch_training_amd import ops
    from distributed_pytorch_training_amd.config import parse_args
    from distributed_pytorch_training_amd.data import SyntheticLoader
    from distributed_pytorch_training_amd.engine.trainer import Trainer
    from distributed_pytorch_training_amd.models import build_model
    from distributed_pytorch_training_amd.ops import conv as native_conv
    from distributed_pytorch_training_amd.utils.env import setup_miopen_env, setup_tunableop

    setup_miopen_env()
    ops.native()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    setup_tunableop()
    args = parse_args(["--model", "resnet50", "--dataset", "synthetic", "--batch-size", str(a.batch_size),
                       "--image-size", "224", "--amp", "--amp-dtype", "bf16", "--channels-last",
                       "--no-cuda-graph", "--lr", "0.1", "--momentum", "0.9", "--weight-decay", "5e-4"])
    torch.manual_seed(0)
    model = build_model("resnet50", 1000, dev, image_size=224, channels_last=True)
    tr = Trainer(model, args, 0, 1, dev, log=lambda s: None)
    loader = SyntheticLoader(a.batch_size * 4, a.batch_size, 224, 1000, dev, channels_last=True, pool=4, seed=0)
    batches = list(iter(loader))
    for i in range(a.warmup):
        tr.train_step(*batches[i % len(batches)])
    torch.cuda.synchronize()

    # (1) GPU step time, host running free
    t0 = time.perf_counter()
    for i in range(a.steps):
        tr.train_step(*batches[i % len(batches)])
    torch.cuda.synchronize()
    gpu_ms = 1e3 * (time.perf_counter() - t0) / a.steps

    # (2) host time per phase with the GPU drained before each step (host cost alone, no
    # back-pressure from a full queue): replicate Trainer._native_step's phases
    from distributed_pytorch_training_amd.amp import autocast
    phases = {"forward": [], "loss": [], "backward": [], "optimizer+metrics": [], "total": []}
    for i in range(a.steps):
        x, y = batches[i % len(batches)]
        torch.cuda.synchronize()
        h0 = time.perf_counter()
        if tr._native_conv_cache:
            native_conv.begin_step()
        else:
            native_conv.reset_side_channels()
        with autocast(tr.device, tr.amp, tr.amp_dtype):
            out = tr.model(x)
            h1 = time.perf_counter()
            loss = tr.criterion(out, y)
        h2 = time.perf_counter()
        try:
            tr.scaler.scale(loss).backward()
        finally:
            if tr._native_conv_cache:
                native_conv.end_caching()
        h3 = time.perf_counter()
        tr.optimizer.step(tr.scaler, host_factor=tr.ddp.grad_factor, grads_checked=tr.ddp.grads_checked,
                          shadow=tr.ddp.shadow_flat, zero_grad=not tr.ddp.grads_overwritten)
        ops.accumulate_metrics(out, y, loss, tr.metrics)
        h4 = time.perf_counter()
        for k, v in zip(phases, (h1 - h0, h2 - h1, h3 - h2, h4 - h3, h4 - h0)):
            phases[k].append(1e3 * v)
    torch.cuda.synchronize()

    # (2b) the same phases with the host running free (a phase that blocks on the GPU shows up
    # as one long phase), and ATen's sync debug mode reporting synchronising calls
    free = {"forward": [], "loss": [], "backward": [], "optimizer+metrics": [], "total": []}
    import warnings
    torch.cuda.set_sync_debug_mode("warn")
    with warnings.catch_warnings(record=True) as wlist:
        warnings.simplefilter("always")
        for i in range(a.steps):
            x, y = batches[i % len(batches)]
            h0 = time.perf_counter()
            if tr._native_conv_cache:
                native_conv.begin_step()
            else:
                native_conv.reset_side_channels()
            with autocast(tr.device, tr.amp, tr.amp_dtype):
                out = tr.model(x)
                h1 = time.perf_counter()
                loss = tr.criterion(out, y)
            h2 = time.perf_counter()
            try:
                tr.scaler.scale(loss).backward()
            finally:
                if tr._native_conv_cache:
                    native_conv.end_caching()
            h3 = time.perf_counter()
            tr.optimizer.step(tr.scaler, host_factor=tr.ddp.grad_factor, grads_checked=tr.ddp.grads_checked,
                              shadow=tr.ddp.shadow_flat, zero_grad=not tr.ddp.grads_overwritten)
            ops.accumulate_metrics(out, y, loss, tr.metrics)
            h4 = time.perf_counter()
            for k, v in zip(free, (h1 - h0, h2 - h1, h3 - h2, h4 - h3, h4 - h0)):
                free[k].append(1e3 * v)
    torch.cuda.set_sync_debug_mode(0)
    torch.cuda.synchronize()
    sync_msgs = sorted({str(w.message)[:300] + " @ " + f"{w.filename}:{w.lineno}" for w in wlist})

    lines = [f"GPU step (host free-running): {gpu_ms:.3f} ms",
             "host time per phase, GPU drained before each step (median ms):"]
    for k, v in phases.items():
        lines.append(f"  {k:18s} {statistics.median(v):8.3f}")

    lines.append("host time per phase, host running free (median ms):")
    for k, v in free.items():
        lines.append(f"  {k:18s} {statistics.median(v):8.3f}   (max {max(v):.3f})")
    lines.append(f"synchronising calls reported by torch.cuda.set_sync_debug_mode: {len(sync_msgs)}")
    lines += ["  " + m for m in sync_msgs]

    # (3) cProfile of the forward + loss + backward calls (host side)
    pr = cProfile.Profile()
    for i in range(a.profile_steps):
        x, y = batches[i % len(batches)]
        torch.cuda.synchronize()
        if tr._native_conv_cache:
            native_conv.begin_step()
        pr.enable()
        with autocast(tr.device, tr.amp, tr.amp_dtype):
            out = tr.model(x)
            loss = tr.criterion(out, y)
        tr.scaler.scale(loss).backward()
        pr.disable()
        if tr._native_conv_cache:
            native_conv.end_caching()
        tr.optimizer.step(tr.scaler, host_factor=tr.ddp.grad_factor, grads_checked=tr.ddp.grads_checked,
                          shadow=tr.ddp.shadow_flat, zero_grad=not tr.ddp.grads_overwritten)
    torch.cuda.synchronize()
    s = io.StringIO()
    st = pstats.Stats(pr, stream=s)
    st.sort_stats("tottime").print_stats(35)
    s2 = io.StringIO()
    pstats.Stats(pr, stream=s2).sort_stats("cumulative").print_stats(45)
    text = "\n".join(lines) + "\n\n## cProfile, forward+loss+backward host calls, " + \
        f"{a.profile_steps} steps, by tottime\n" + s.getvalue() + "\n## by cumulative\n" + s2.getvalue()
    print(text)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text)


if __name__ == "__main__":
    main()
