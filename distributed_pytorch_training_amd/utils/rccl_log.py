"""What RCCL actually opened, read back from its own init log.

RCCL has no API that reports a communicator's channel count.  With ``NCCL_DEBUG=INFO``
(subsystem ``INIT``) every communicator's initialisation logs, in order,

    ... NCCL INFO 16 coll channels, 0 collnet channels, 0 nvls channels, 16 p2p channels, 2 p2p channels per peer
    ... NCCL INFO ncclCommInitRank comm 0x55d0c6a1e2f0 rank 0 nranks 8 cudaDev 0 ... - Init COMPLETE

so the channel line that precedes a communicator's "Init COMPLETE" line is that
communicator's.  Several communicators live in one process (torch's process group creates its
own before the framework's, ``parallel/comm.py``); ``channels_by_comm`` keys the counts by the
``comm 0x...`` handle, which ``RcclComm.handle`` exposes for the framework's one.

``NCCL_DEBUG_FILE`` sends the log to a file (``%h`` host, ``%p`` pid), so the bench's stdout
contract (one JSON line) is untouched.
"""
from __future__ import annotations

import os
import re
from typing import Dict, Optional

_CHANNELS = re.compile(r"NCCL INFO (\d+) coll channels")
_COMPLETE = re.compile(r"NCCL INFO .*\bcomm (0x[0-9a-fA-F]+) rank (\d+) nranks (\d+) .*Init COMPLETE")
_RING = re.compile(r"NCCL INFO Channel (\d+)/(\d+) :")


def channels_by_comm(text: str) -> Dict[int, Dict[str, int]]:
    """``{comm handle: {"coll_channels": n, "rank": r, "nranks": N}}`` from an RCCL INFO log."""
    out: Dict[int, Dict[str, int]] = {}
    pending: Optional[int] = None
    ring_total: Optional[int] = None
    for line in text.splitlines():
        m = _CHANNELS.search(line)
        if m:
            pending = int(m.group(1))
            continue
        m = _RING.search(line)
        if m:
            ring_total = int(m.group(2))
            continue
        m = _COMPLETE.search(line)
        if m:
            n = pending if pending is not None else ring_total
            if n is not None:
                out[int(m.group(1), 16)] = {"coll_channels": n, "rank": int(m.group(2)),
                                            "nranks": int(m.group(3))}
            pending = ring_total = None
    return out


def debug_env(path_prefix: str) -> Dict[str, str]:
    """Environment that makes RCCL write its init log to ``<prefix>.<pid>.log`` (set BEFORE the
    first communicator of the process is created: RCCL reads it once)."""
    return {"NCCL_DEBUG": "INFO", "NCCL_DEBUG_SUBSYS": "INIT", "NCCL_DEBUG_FILE": f"{path_prefix}.%p.log"}


def opened_channels(handle: int, path_prefix: str) -> Optional[int]:
    """Channel count of the communicator ``handle`` from this process's log file, or None."""
    path = f"{path_prefix}.{os.getpid()}.log"
    try:
        with open(path, errors="replace") as f:
            text = f.read()
    except OSError:
        return None
    rec = channels_by_comm(text).get(int(handle))
    return rec["coll_channels"] if rec else None
