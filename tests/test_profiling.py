"""Sync-profile arithmetic (% of step in all-reduce, exposed communication)."""
import json

import torch

from distributed_pytorch_training_amd.profiling.timeline import StepTimeline, roctx_range


def test_summary_math(tmp_path):
    tl = StepTimeline(torch.device("cpu"), enabled=False)
    tl.records = [
        {"fwd_ms": 10.0, "bwd_ms": 20.0, "opt_ms": 1.0, "step_ms": 31.0, "allreduce_busy_ms": 99.0},  # skipped
        {"fwd_ms": 10.0, "bwd_ms": 20.0, "opt_ms": 1.0, "step_ms": 40.0, "allreduce_busy_ms": 8.0,
         "exposed_comm_ms": 2.0, "comm_span_ms": 15.0},
        {"fwd_ms": 12.0, "bwd_ms": 22.0, "opt_ms": 1.0, "step_ms": 40.0, "allreduce_busy_ms": 8.0,
         "exposed_comm_ms": 2.0, "comm_span_ms": 15.0},
    ]
    s = tl.summary(skip=1)
    assert s["pct_step_allreduce"] == 20.0
    assert s["pct_step_exposed_comm"] == 5.0
    assert s["steps_profiled"] == 2 and s["fwd_ms"] == 11.0
    out = tmp_path / "p.json"
    tl.dump(str(out), {"world_size": 4})
    d = json.loads(out.read_text())
    assert d["world_size"] == 4 and len(d["steps"]) == 3


def test_disabled_on_cpu_and_roctx_is_harmless():
    tl = StepTimeline(torch.device("cpu"), enabled=True)
    assert not tl.enabled
    tl.mark("start")
    tl.end_step(None)
    assert tl.summary() == {}
    with roctx_range("x", enabled=True):
        pass


def test_trainer_gives_the_reducer_one_event_slot_per_unresolved_step():
    """--profile-sync: a step's per-bucket comm events are read max_pending steps
    later, so the reducer must keep at least max_pending + 1 event slots or the deferred reader
    sees the NEXT step's (incomplete) events."""
    from distributed_pytorch_training_amd.config import parse_args
    from distributed_pytorch_training_amd.engine.trainer import Trainer
    from distributed_pytorch_training_amd.models import build_model

    args = parse_args(["--model", "resnet18", "--dataset", "synthetic", "--image-size", "32", "--num-classes", "10",
                       "--profile-sync"])
    tr = Trainer(build_model("resnet18", 10), args, 0, 1, torch.device("cpu"), log=lambda s: None)
    assert tr.ddp._profile_slots >= tr.timeline.max_pending + 1
