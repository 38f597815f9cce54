"""Gradient-sync profiling: hipEvent timeline + roctx ranges.

The reference README promises "gradient sync profiling" and "At 4 GPUs, gradient
synchronization accounts for ~X% of step time" (reference README.md:6,35) but measures
nothing beyond wall clock.  This module measures it:

* per step, hipEvents on the compute stream at start / after forward / after backward /
  after the optimizer (``StepTimeline.mark``);
* per bucket, hipEvents recorded by the C++ reducer on the RCCL stream around each
  all-reduce (+ fused non-finite check), plus "backward end -> last bucket done" (the
  *exposed* communication that overlap failed to hide) and the comm span;
* derived: forward / backward / optimizer ms, all-reduce busy ms, exposed ms, and
  "% of step in all-reduce" (busy / step) and "% of step exposed" (exposed / step).

Event reads are deferred: a step's events are resolved ``max_pending`` steps later (they are
complete by then), and the reducer keeps one event set per step of the window (event slots),
so profiling does not serialise the pipeline.
``roctx_range`` emits markers for ``rocprofv3 --marker-trace`` when roctx is loadable.
"""
from __future__ import annotations

import collections
import contextlib
import ctypes
import json
import statistics
from typing import Deque, Dict, List, Optional

import torch


class StepTimeline:
    def __init__(self, device: torch.device, enabled: bool = False) -> None:
        self.enabled = enabled and torch.device(device).type == "cuda"
        self.device = device
        self._marks: Dict[str, torch.cuda.Event] = {}
        self._pending: Deque[tuple] = collections.deque()
        # steps whose events may stay unread; must stay below the reducer's profile slots
        self.max_pending = 1
        self.records: List[Dict[str, float]] = []

    def mark(self, name: str) -> None:
        if not self.enabled:
            return
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        self._marks[name] = ev

    def discard(self) -> None:
        """Drop the marks of a step that did not run the optimizer (accumulation micro-batch)."""
        self._marks = {}

    def end_step(self, comm_profile=None) -> None:
        """``comm_profile``: None, a dict, or a zero-argument callable returning the reducer's
        per-bucket times for THIS step (``NativeDDP.comm_profile_ref()``: bound to the step's
        event slot).  Nothing is read now: up to ``max_pending`` steps stay unresolved, so a
        profiled window has no per-step host synchronisation when the reducer keeps at least
        ``max_pending + 1`` event slots; older steps are resolved (their events are long
        complete) as new ones arrive."""
        if not self.enabled:
            return
        self._pending.append((dict(self._marks), comm_profile))
        self._marks = {}
        while len(self._pending) > self.max_pending:
            self._resolve_one()

    def _resolve_one(self) -> None:
        marks, comm = self._pending.popleft()
        marks["opt"].synchronize()
        if callable(comm):
            comm = comm()
        rec = {"fwd_ms": marks["start"].elapsed_time(marks["fwd"]),
               "bwd_ms": marks["fwd"].elapsed_time(marks["bwd"]),
               "opt_ms": marks["bwd"].elapsed_time(marks["opt"]),
               "step_ms": marks["start"].elapsed_time(marks["opt"])}
        if comm and comm.get("bucket_ms"):
            b = [x for x in comm["bucket_ms"] if x >= 0]
            rec["allreduce_busy_ms"] = float(sum(b))
            rec["buckets"] = len(b)
            if len(comm.get("step_ms", [])) == 3:
                rec["exposed_comm_ms"] = comm["step_ms"][1]
                rec["comm_span_ms"] = comm["step_ms"][2]
        self.records.append(rec)

    def _resolve_pending(self) -> None:
        while self._pending:
            self._resolve_one()

    def flush(self) -> None:
        if self.enabled:
            torch.cuda.synchronize()
            self._resolve_pending()

    def summary(self, skip: int = 1) -> Dict[str, float]:
        self.flush()
        recs = self.records[skip:] if len(self.records) > skip else self.records
        if not recs:
            return {}
        keys = sorted({k for r in recs for k in r if k != "buckets"})
        out = {k: statistics.median([r[k] for r in recs if k in r]) for k in keys}
        if "allreduce_busy_ms" in out and out.get("step_ms"):
            out["pct_step_allreduce"] = 100.0 * out["allreduce_busy_ms"] / out["step_ms"]
        if "exposed_comm_ms" in out and out.get("step_ms"):
            out["pct_step_exposed_comm"] = 100.0 * out["exposed_comm_ms"] / out["step_ms"]
        out["steps_profiled"] = len(recs)
        return out

    def dump(self, path: str, extra: Optional[dict] = None) -> None:
        with open(path, "w") as f:
            json.dump({"summary": self.summary(), "steps": self.records, **(extra or {})}, f, indent=1)


_roctx = None


def _load_roctx():
    global _roctx
    if _roctx is None:
        _roctx = False
        for name in ("libroctx64.so", "libroctx64.so.4"):
            try:
                lib = ctypes.CDLL(name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                _roctx = lib
                break
            except OSError:
                continue
    return _roctx or None


@contextlib.contextmanager
def roctx_range(name: str, enabled: bool = True):
    lib = _load_roctx() if enabled else None
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib is not None:
            lib.roctxRangePop()
