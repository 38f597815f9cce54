"""hipGraph replay in the configuration the reference's own script runs.

``train_ddp.py --dataset synthetic --image-size 32 --num-classes 10`` with every other flag at its
default: ResNet-18, batch 128, fp32 (no --amp), native engine, channels_last, MIOpen convolutions
with ``cudnn.benchmark = True`` (find mode), no forced split-K, no deterministic flag - and replay
on by default (launch-bound step).  Two checks (bench/graph_parity.py):

* teacher-forced: 20 replayed steps, each also run eagerly from the SAME state; the parameter
  difference must be a rounding-level fraction of the step's update (median <= 1e-5 of the update,
  every step <= 5e-3: MIOpen's find-mode algorithms are not deterministic, and an occasional ReLU /
  max-pool decision flip moves one step by ~7e-4 of its update - a replay that dropped or repeated
  work would be off by ~1);
* free-running: 300 steps replayed vs 300 eager from the same init on the learnable synthetic
  task (class prototypes + fresh noise, ``--synthetic-task prototypes``); the windowed loss curves
  must stay within a band after the first 150 steps (the lr 0.1 transient, only bounded) and both
  runs must learn the task.  (On the default 4-batch random-label pool the run is a memorisation
  race whose speed differs between two EAGER runs of this configuration by as much as between
  replay and eager - MIOpen's find-mode algorithms are not deterministic - so that task cannot
  tell replay from eager; profiles/graph_vs_eager_r4.md has both.)
"""
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench"))


@pytest.fixture
def benchmark_mode(cuda):
    from distributed_pytorch_training_amd.utils.env import setup_tunableop
    old = (torch.backends.cudnn.benchmark, torch.backends.cudnn.deterministic)
    torch.backends.cudnn.benchmark, torch.backends.cudnn.deterministic = True, False
    setup_tunableop()
    yield
    torch.backends.cudnn.benchmark, torch.backends.cudnn.deterministic = old


def test_replayed_steps_match_eager_steps_teacher_forced(benchmark_mode):
    import graph_parity

    rows = graph_parity.teacher(20, [])
    assert len(rows) == 20
    rel = sorted(r["rel_param_vs_update"] for r in rows)
    assert rel[len(rel) // 2] <= 1e-5, rel
    for r in rows:
        assert r["rel_param_vs_update"] <= 5e-3, r
        assert r["rel_grad"] <= 2e-2, r
        assert r["max_buf_diff"] <= 1e-2, r
        assert r["metrics_g"][2] == r["metrics_e"][2], r          # same sample count


def test_replayed_run_tracks_eager_run(benchmark_mode):
    import graph_parity

    curves = graph_parity.free(300, [], task="prototypes")
    g, e = curves["--cuda-graph"], curves["--no-cuda-graph"]
    w = 50
    # steps 0-149 are lr 0.1's violent transient (25-step means 2.0-3.1 against ln 10 = 2.3): its
    # path is chaotic, and which run leaves it first - and whether a second spike follows, as late
    # as steps 50-99 (0.46 / 0.34 in one eager run against 0.08 / 0.05 replayed, full-suite run of
    # round 6) - has differed between runs in both directions, so it is only checked to stay bounded
    # there; a replay that dropped or repeated work would not leave ln 10 at all
    a0, b0 = sum(g[:w]) / w, sum(e[:w]) / w
    assert a0 < 3.5 and b0 < 3.5 and max(a0, b0) <= 1.6 * min(a0, b0), (a0, b0)
    for i in range(w, 150, w):
        a = sum(g[i:i + w]) / w
        b = sum(e[i:i + w]) / w
        assert a < 1.0 and b < 1.0, (i, a, b)
    # settled: the two runs learn the task to the same loss
    for i in range(150, 300, w):
        a = sum(g[i:i + w]) / w
        b = sum(e[i:i + w]) / w
        assert abs(a - b) <= 0.1 * max(b, 0.5) + 0.05, (i, a, b)
    assert sum(g[-w:]) / w < 0.2 and sum(e[-w:]) / w < 0.2
