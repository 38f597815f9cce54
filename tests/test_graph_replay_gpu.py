"""hipGraph replay vs eager, parameter by parameter (engine/graph.py replay validation).

Regression for the wrong weight gradients MIOpen's CK grouped backward-weights solver returns
under replay (utils/env.py GRAPH_UNSAFE_MIOPEN_SOLVERS): the fp32 ResNet-18 of the reference's
default workload runs every convolution on MIOpen, so a replayed step must give every parameter
the gradient an eager step gives it from the same state.
"""
import os
import warnings

import pytest
import torch

from distributed_pytorch_training_amd.config import parse_args
from distributed_pytorch_training_amd.engine.graph import restore, snapshot
from distributed_pytorch_training_amd.engine.trainer import Trainer
from distributed_pytorch_training_amd.models import build_model
from distributed_pytorch_training_amd.utils.env import GRAPH_UNSAFE_MIOPEN_SOLVERS

pytestmark = pytest.mark.gpu


def test_graph_unsafe_miopen_solvers_excluded_in_session():
    assert all(os.environ.get(k) == "0" for k in GRAPH_UNSAFE_MIOPEN_SOLVERS)


def _per_param_worst(tr, a, b):
    floor = 1e-6 * b.double().norm().item()
    w = (0.0, "")
    for n, u, v in zip(tr.ddp.arena.names, tr.ddp.arena.views(a), tr.ddp.arena.views(b)):
        r = (u - v).double().norm().item() / max(v.double().norm().item(), floor, 1e-30)
        w = max(w, (r, n))
    return w


def test_fp32_resnet18_replay_matches_eager_per_parameter(cuda):
    torch.backends.cudnn.benchmark = True
    torch.manual_seed(0)
    model = build_model("resnet18", 10, cuda, image_size=32, channels_last=True)
    args = parse_args(["--dataset", "synthetic", "--image-size", "32", "--num-classes", "10", "--cuda-graph"])
    tr = Trainer(model, args, 0, 1, cuda, log=lambda s: None)
    G = tr.graphed
    g = torch.Generator(device=cuda).manual_seed(5)

    def batch():
        x = torch.randn(128, 3, 32, 32, device=cuda, generator=g) * 4
        return x.contiguous(memory_format=torch.channels_last), torch.randint(0, 10, (128,), device=cuda, generator=g)

    for _ in range(G.warmup + 1):       # warmup, capture, validated first replay
        tr.train_step(*batch())
    torch.cuda.synchronize()
    assert G.graph is not None and not G.failed, (G.failed, G.validation)
    assert G.validation["ok"], G.validation
    # teacher-forced: three more steps, each replayed and run eagerly from the same state
    for _ in range(3):
        x, y = batch()
        s0 = snapshot(tr)
        tr.train_step(x, y)
        torch.cuda.synchronize()
        gr = tr.ddp.arena.grad_flat.clone()
        restore(tr, s0)
        with G._on_stream():
            tr._native_step(x, y)
        torch.cuda.synchronize()
        ge = tr.ddp.arena.grad_flat
        whole = ((gr - ge).double().norm() / ge.double().norm()).item()
        worst = _per_param_worst(tr, gr, ge)
        # fp32 rounding-level agreement overall; a single near-cancelling BN sum may move more
        assert whole < 1e-3 and worst[0] < 0.1, (whole, worst)


class _HostScale(torch.nn.Module):
    """Multiplies by a Python-side counter that advances every forward: eager runs see the new
    value, a replay keeps the one baked in at capture - a step that is not replay-safe."""

    def __init__(self):
        super().__init__()
        self.k = 1.0

    def forward(self, x):
        self.k += 1.0
        return x * self.k


def test_validation_rejects_a_step_that_is_not_replay_safe(cuda):
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Conv2d(3, 16, 3, padding=1), torch.nn.ReLU(), _HostScale(),
                                torch.nn.AdaptiveAvgPool2d(1), torch.nn.Flatten(), torch.nn.Linear(16, 10)).to(cuda)
    args = parse_args(["--dataset", "synthetic", "--no-channels-last", "--cuda-graph"])
    tr = Trainer(model, args, 0, 1, cuda, log=lambda s: None)
    x = torch.randn(8, 3, 16, 16, device=cuda)
    y = torch.randint(0, 10, (8,), device=cuda)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        for _ in range(tr.graphed.warmup + 1):
            tr.train_step(x, y)
    torch.cuda.synchronize()
    G = tr.graphed
    assert G.failed and G.validation is not None and not G.validation["ok"], G.validation
    assert any("not replay-safe" in str(m.message) for m in w)
    assert G.replays == 0
    assert tr.global_step == G.warmup + 1
    assert tr.metrics[2].item() == 8 * (G.warmup + 1)    # the validated call still counts one step


def test_validation_rejects_an_injected_30pct_error_on_one_parameter(cuda):
    """a replay that is wrong by 30 % on ONE parameter - what a replay-unsafe kernel
    that reads stale data produces - must fail the noise-relative validation and fall back."""
    torch.manual_seed(0)
    model = build_model("resnet18", 10, cuda, image_size=32, channels_last=True)
    args = parse_args(["--dataset", "synthetic", "--image-size", "32", "--num-classes", "10", "--cuda-graph"])
    tr = Trainer(model, args, 0, 1, cuda, log=lambda s: None)
    G = tr.graphed
    names = list(tr.ddp.arena.names)
    target = names.index("layer3.0.conv1.weight")

    def inject(grad_flat, arena):
        arena.views(grad_flat)[target].mul_(1.3)

    G.inject = inject
    g = torch.Generator(device=cuda).manual_seed(5)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        for _ in range(G.warmup + 1):
            x = torch.randn(128, 3, 32, 32, device=cuda, generator=g).contiguous(memory_format=torch.channels_last)
            tr.train_step(x, torch.randint(0, 10, (128,), device=cuda, generator=g))
    torch.cuda.synchronize()
    v = G.validation
    assert G.failed and not v["ok"] and v["worst"] == "layer3.0.conv1.weight", v
    assert any("not replay-safe" in str(m.message) for m in w)
    # without the injection the same configuration validates (the check is not simply strict)
    tr2 = Trainer(build_model("resnet18", 10, cuda, image_size=32, channels_last=True), args, 0, 1, cuda,
                  log=lambda s: None)
    for _ in range(tr2.graphed.warmup + 1):
        x = torch.randn(128, 3, 32, 32, device=cuda, generator=g).contiguous(memory_format=torch.channels_last)
        tr2.train_step(x, torch.randint(0, 10, (128,), device=cuda, generator=g))
    torch.cuda.synchronize()
    assert tr2.graphed.validation["ok"] and not tr2.graphed.failed, tr2.graphed.validation
