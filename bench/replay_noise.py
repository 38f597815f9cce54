"""Noise floor of the fp32 hipGraph replay check.

Reproduces ``tests/test_graph_replay_gpu.py::test_fp32_resnet18_replay_matches_eager_per_parameter``
(fp32 ResNet-18, 32 px, batch 128, channels_last, MIOpen convolutions in ``cudnn.benchmark`` find
mode, random inputs x4) and, for each teacher-forced step, runs from ONE saved state:

    replay A, replay B, eager A, eager B

so the replay-vs-eager gap can be read against the two self-consistency spreads (replay-vs-replay,
eager-vs-eager).  Per pair it prints the whole-arena and the worst per-parameter relative L2.

``--db shipped`` points MIOpen at the repo's find-db (what ``train_ddp.py`` does, engine/run.py);
``--db fresh`` (default) leaves MIOpen's default user db, as the GPU test session did in r4.
Run under ``MIOPEN_LOG_LEVEL=5`` to get MIOpen's "Chosen Algorithm" lines (solver per conv and
direction) on stderr.

    MIOPEN_LOG_LEVEL=5 python bench/replay_noise.py --steps 6 2> gpurun_out/miopen.log
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def rel(a, b):
    return ((a - b).double().norm() / b.double().norm().clamp_min(1e-30)).item()


def per_param_worst(tr, a, b):
    floor = 1e-6 * b.double().norm().item()
    w = (0.0, "")
    for n, u, v in zip(tr.ddp.arena.names, tr.ddp.arena.views(a), tr.ddp.arena.views(b)):
        r = (u - v).double().norm().item() / max(v.double().norm().item(), floor, 1e-30)
        w = max(w, (r, n))
    return w


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--db", choices=["fresh", "shipped"], default="fresh")
    ap.add_argument("--benchmark", type=int, default=1)
    ap.add_argument("--amp", action="store_true")
    a = ap.parse_args()
    from distributed_pytorch_training_amd.utils.env import graph_safe_miopen, setup_miopen_env
    graph_safe_miopen()
    if a.db == "shipped":
        setup_miopen_env()
    from distributed_pytorch_training_amd.config import parse_args
    from distributed_pytorch_training_amd.engine.graph import restore, snapshot
    from distributed_pytorch_training_amd.engine.trainer import Trainer
    from distributed_pytorch_training_amd.models import build_model

    cuda = torch.device("cuda:0")
    torch.cuda.set_device(cuda)
    torch.backends.cudnn.benchmark = bool(a.benchmark)
    torch.manual_seed(0)
    model = build_model("resnet18", 10, cuda, image_size=32, channels_last=True)
    argv = ["--dataset", "synthetic", "--image-size", "32", "--num-classes", "10", "--cuda-graph"]
    if a.amp:
        argv += ["--amp", "--amp-dtype", "bf16"]
    args = parse_args(argv)
    tr = Trainer(model, args, 0, 1, cuda, log=lambda s: None)
    G = tr.graphed
    g = torch.Generator(device=cuda).manual_seed(5)

    def batch():
        x = torch.randn(128, 3, 32, 32, device=cuda, generator=g) * 4
        return x.contiguous(memory_format=torch.channels_last), torch.randint(0, 10, (128,), device=cuda, generator=g)

    os.environ["DPT_GRAPH_VALIDATE_DEBUG"] = "1"
    for _ in range(G.warmup + 1):
        tr.train_step(*batch())
    torch.cuda.synchronize()
    print(json.dumps({"validation": G.validation, "failed": G.failed}), flush=True)
    if G.graph is None or G.failed:
        return 1

    def eager(x, y):
        with G._on_stream():
            tr._native_step(x, y)
        tr.global_step -= 1

    for k in range(a.steps):
        x, y = batch()
        s0 = snapshot(tr)
        grads = {}
        for name, fn in (("replayA", lambda: tr.train_step(x, y)), ("replayB", lambda: tr.train_step(x, y)),
                         ("eagerA", lambda: eager(x, y)), ("eagerB", lambda: eager(x, y))):
            restore(tr, s0)
            fn()
            torch.cuda.synchronize()
            grads[name] = tr.ddp.arena.grad_flat.detach().clone()
        # continue from the eager result (state as after eagerB)
        row = {"step": k}
        for p, q in (("replayA", "replayB"), ("eagerA", "eagerB"), ("replayA", "eagerA"), ("replayB", "eagerB")):
            w = per_param_worst(tr, grads[p], grads[q])
            row[f"{p}-{q}"] = {"whole": rel(grads[p], grads[q]), "worst": round(w[0], 8), "param": w[1]}
        print(json.dumps(row), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
