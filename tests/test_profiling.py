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
