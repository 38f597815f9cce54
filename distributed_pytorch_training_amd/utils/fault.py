"""Fault injection for the failure-detection and elastic-restart tests.

One flag, one spec, one exit status::

    --fault-inject rank=R,step=S    rank R dies before global optimizer step S
    --fault-inject rank=R,epoch=E   rank R dies at the start of (0-based) epoch E

The rank leaves with ``os._exit(FAULT_EXIT_CODE)`` - abruptly, no teardown, no collective -
which is what its peers must survive (watchdog / abort path) and what ``--resume auto``
must recover from.

* A **step** fault fires every time the rank reaches step S (no state on disk), so re-running
  the same fault test in the same output directory always injects it.
* An **epoch** fault fires once per output directory (a marker file there): it exists for the
  restart case, where the job a restart policy relaunches with the same command line resumes
  at that epoch and must run through.  When the marker suppresses it, a warning says so once.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from pathlib import Path
from typing import Optional

FAULT_EXIT_CODE = 17
_SUPPRESSED: set = set()


@dataclass(frozen=True)
class FaultSpec:
    rank: int
    step: Optional[int] = None
    epoch: Optional[int] = None

    @classmethod
    def parse(cls, text: Optional[str]) -> Optional["FaultSpec"]:
        if not text:
            return None
        fields = {}
        for part in str(text).split(","):
            k, sep, v = part.partition("=")
            k = k.strip()
            if not sep or k not in ("rank", "step", "epoch") or k in fields:
                raise ValueError(f"--fault-inject: expected rank=R,step=S or rank=R,epoch=E, got {text!r}")
            fields[k] = int(v)
        if "rank" not in fields or (("step" in fields) == ("epoch" in fields)):
            raise ValueError(f"--fault-inject: expected rank=R,step=S or rank=R,epoch=E, got {text!r}")
        return cls(**fields)

    def marker(self, output_dir: str) -> Path:
        what = f"step{self.step}" if self.step is not None else f"epoch{self.epoch}"
        return Path(output_dir) / f".fault_injected_rank{self.rank}_{what}"

    def fire(self, output_dir: str, log=print) -> None:
        """Die now: the caller has decided this is the fault point (epoch faults: once per
        output dir)."""
        if self.epoch is not None:
            m = self.marker(output_dir)
            key = (self, str(m))
            if key in _SUPPRESSED:
                return
            if m.exists():
                _SUPPRESSED.add(key)    # decided once per process: no file check on later calls
                log(f"rank {self.rank}: fault at epoch {self.epoch} NOT injected - it already fired for "
                    f"this output dir (marker {m}; delete it to re-arm)")
                return
            m.parent.mkdir(parents=True, exist_ok=True)
            m.touch()
        where = f"step {self.step}" if self.step is not None else f"epoch {self.epoch}"
        log(f"rank {self.rank}: injected fault at {where}")
        import sys
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(FAULT_EXIT_CODE)
