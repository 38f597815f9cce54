"""Communicator bootstrap: the framework-owned collective for the gradient hot path.

Control plane: torch's process group (``env://`` TCPStore rendezvous, reference
train_ddp.py:65) carries the 128-byte RCCL unique id from rank 0 to every rank.  Data
plane: a C++ ``Collective`` (csrc/comm.h) that the C++ reducer enqueues bucket all-reduces
on, one of

* ``"rccl"`` - ``RcclComm`` (csrc/rccl_comm.cpp): RCCL over xGMI on a dedicated
  high-priority HIP stream, guarded by a watchdog thread (csrc/watchdog.cpp) that enforces
  ``--dist-timeout`` and polls ``ncclCommGetAsyncError``;
* ``"c10d"`` - ``ProcessGroupComm`` (csrc/pg_comm.cpp): the same contract served by torch's
  default process group on device memory (RCCL through ProcessGroupNCCL, torch's watchdog).
  The fallback when the framework communicator cannot be created, and its A/B arm;
* ``"host"`` - ``HostBridgeComm`` (csrc/host_comm.cpp): the same device-pointer contract
  served by ``torch.distributed`` over gloo through pinned host staging.  Several ranks can
  then share one GPU and still run the whole multi-rank GPU data path (tests/
  test_multirank_gpu.py); it is a verification / debug transport, not a fast one.
* ``"host-async"`` - the same bridge enqueued like RCCL (D2H, a HIP host function running the
  gloo collective, H2D on the caller's stream; the caller never blocks), so backward overlaps
  the in-flight collective and the exposed-comm measurement means something on one GPU.  Its
  collectives use a gloo group of their own, driven from C++ on HIP's host-function thread
  without the GIL; they never interleave with the main thread's collectives on the default group.

On CPU (gloo) there is no device collective; ``make_comm`` returns ``None`` and the reducer
drives ``torch.distributed`` through a Python callback instead.

RCCL channel count: ``rccl_channels`` > 0 creates the framework communicator with
``ncclCommInitRankConfig`` and ``ncclConfig_t.minCTAs = maxCTAs = rccl_channels`` - a
per-communicator setting, so it applies no matter what torch's own process-group
communicator (created earlier, eagerly, by ``init_process_group(device_id=...)``) read from
the process-wide ``NCCL_MIN/MAX_NCHANNELS`` environment.  The environment is not touched.
On an 8x MI355X node every GPU has 7 point-to-point xGMI links and a ring uses one outgoing
link per channel, so a bucket reaches the aggregate link bandwidth only with >= 7 channels
(SURVEY.md §5.8).  0 keeps RCCL's topology-derived choice, which already opens more than 7
channels on a fully connected xGMI node; the knob exists to bound the CUs RCCL's kernels
take from the overlapped backward (docs/DESIGN.md §3.2).  tests/test_comm_gpu.py parses
RCCL's init log to check the communicator got what was asked.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.distributed as dist

from .. import ops

COMM_KINDS = ("rccl", "c10d", "host", "host-async")
_HOST_GROUP = None
_ASYNC_GROUP = None
# Why the last ``make_comm(kind="rccl")`` of this process ended on the c10d fallback (None: it did
# not).  NativeDDP copies it to ``comm_fallback_reason``; bench.py fails closed on it.
LAST_FALLBACK_REASON: Optional[str] = None
# Upper bound of the RCCL init wait; tied to the process-group timeout (``init_timeout_for``).
MAX_INIT_TIMEOUT_S = 300.0


def init_timeout_for(pg_timeout_s: Optional[float]) -> float:
    """How long a rank waits inside ``ncclCommInitRank`` before giving up.

    A rank whose own init failed goes straight to the post-init MIN agreement, a control-plane
    collective bounded by the process-group timeout (``--dist-timeout``).  Its peers must reach
    that agreement first, so their init wait has to end well inside that timeout: half of it,
    capped at ``MAX_INIT_TIMEOUT_S``."""
    if pg_timeout_s is None or pg_timeout_s <= 0:
        return MAX_INIT_TIMEOUT_S
    return min(MAX_INIT_TIMEOUT_S, 0.5 * float(pg_timeout_s))


def _host_group():
    """A gloo group for the host bridge (the default group when it already is gloo)."""
    global _HOST_GROUP
    if _HOST_GROUP is None:
        _HOST_GROUP = dist.group.WORLD if dist.get_backend() == "gloo" else dist.new_group(backend="gloo")
    return _HOST_GROUP


def _async_group():
    """A gloo group of its own for the asynchronous bridge (its collectives run on another
    thread, concurrently with the main thread's).  Collective creation: every rank, same point."""
    global _ASYNC_GROUP
    if _ASYNC_GROUP is None:
        _ASYNC_GROUP = dist.new_group(backend="gloo")
    return _ASYNC_GROUP


def _host_all_reduce(t: torch.Tensor) -> None:
    dist.all_reduce(t, group=_host_group())


def _host_broadcast(t: torch.Tensor, root: int) -> None:
    dist.broadcast(t, root, group=_host_group())


def make_comm(device: torch.device, rank: int, world_size: int, kind: str = "rccl",
              timeout_s: Optional[float] = None, rccl_channels: int = 0,
              exit_grace_s: float = 30.0, init_timeout_s: Optional[float] = None):
    """Create the device collective on ``device`` (GPU) or return None (CPU/gloo path).

    ``init_timeout_s`` defaults to ``init_timeout_for(timeout_s)``."""
    global LAST_FALLBACK_REASON
    LAST_FALLBACK_REASON = None
    if init_timeout_s is None:
        init_timeout_s = init_timeout_for(timeout_s)
    if device.type != "cuda":
        if kind == "rccl" and world_size > 1 and "DPT_TEST_FAIL_COMM_INIT_RANK" in os.environ:
            _cpu_rehearsal(rank, world_size)
        return None
    if kind not in COMM_KINDS:
        raise ValueError(f"unknown communicator kind {kind!r}; expected one of {COMM_KINDS}")
    C = ops.native()
    dev = device.index if device.index is not None else 0
    if kind in ("host", "host-async"):
        if world_size > 1 and not dist.is_initialized():
            raise RuntimeError("the host-bridge communicator needs an initialised process group")
        if kind == "host-async":
            # collective group creation: every rank, same point.  The bridge calls the group's
            # C++ ProcessGroup from HIP's host-function thread, without the GIL.
            pg = _async_group() if world_size > 1 else None
            return C.HostBridgeComm(_host_all_reduce, _host_broadcast, rank, world_size, dev, True, pg)
        if world_size > 1:
            _host_group()
        return C.HostBridgeComm(_host_all_reduce, _host_broadcast, rank, world_size, dev)
    if kind == "c10d":
        return _pg_comm(C, dev)
    n_ch = max(0, int(rccl_channels or 0))
    comm = rccl_or_fallback(
        new_uid=C.RcclComm.new_unique_id,
        create=lambda uid: C.RcclComm(uid, rank, world_size, dev, n_ch, n_ch, float(init_timeout_s)),
        fallback=lambda: _pg_comm(C, dev), rank=rank, world_size=world_size, flag_device=device)
    if timeout_s and timeout_s > 0 and world_size > 1 and comm.kind == "rccl":
        comm.enable_watchdog(float(timeout_s), 0.5, float(exit_grace_s))
    return comm


def _cpu_rehearsal(rank: int, world_size: int) -> None:
    """Testing (``DPT_TEST_FAIL_COMM_INIT_RANK`` set, gloo ranks on the CPU): run the bootstrap
    agreement of ``rccl_or_fallback`` with a stand-in unique id, so the fallback decision and
    ``LAST_FALLBACK_REASON`` (what bench.py fails closed on) are exercised without a GPU.  The
    CPU path has no device collective either way: the reducer keeps its gloo callback."""
    rccl_or_fallback(new_uid=lambda: b"\0" * 128, create=lambda uid: "cpu-stand-in",
                     fallback=lambda: None, rank=rank, world_size=world_size,
                     flag_device=torch.device("cpu"))


def _agree(ok: bool, flag_device) -> bool:
    on = flag_device if dist.get_backend() == "nccl" else "cpu"
    flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=on)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    return bool(flag.item())


def rccl_or_fallback(new_uid, create, fallback, rank: int, world_size: int, flag_device):
    """Create the framework communicator on every rank, or fall back on every rank.

    RCCL's initialisation is collective and blocking: a rank that fails BEFORE it (no unique id,
    a failed precondition) would leave its peers blocked inside ``ncclCommInitRank`` and never
    reach an agreement afterwards.  So the ranks agree three times over the control plane:

    1. rank 0's unique id travels with its creation status (a failed ``ncclGetUniqueId`` is a
       ``None`` every rank sees, and nobody enters RCCL);
    2. before init, a MIN all-reduce of "ready" (the test hook ``DPT_TEST_FAIL_COMM_INIT_RANK``
       makes one rank not ready) - any rank not ready: nobody enters RCCL;
    3. after init, a MIN all-reduce of "created" - a communicator some ranks built and others did
       not would hang the first collective, so the built ones are aborted.

    Every fallback records its reason in ``LAST_FALLBACK_REASON``.

    A failure INSIDE ``ncclCommInitRank`` on some ranks only is bounded by the communicator's
    init timeout (csrc/rccl_comm.cpp: the blocked ranks give up and reach step 3), then every
    rank takes the fallback.  ``world_size == 1`` skips the agreements."""
    import warnings

    err = None
    uid = None
    if world_size > 1:
        box = [None]
        if rank == 0:
            try:
                box = [new_uid()]
            except RuntimeError as e:
                err = e
        dist.broadcast_object_list(box, src=0)
        uid = box[0]
        ready = uid is not None and os.environ.get("DPT_TEST_FAIL_COMM_INIT_RANK") != str(rank)
        if uid is None and err is None:
            err = RuntimeError("rank 0 could not create an RCCL unique id")
        elif not ready and err is None:
            err = RuntimeError("injected pre-init failure (DPT_TEST_FAIL_COMM_INIT_RANK)")
        if not _agree(ready, flag_device):
            reason = f"framework RCCL communicator not created on any rank ({err or 'another rank was not ready'})"
            warnings.warn(reason + "; falling back to --comm c10d")
            return _fell_back(reason, fallback)
    else:
        uid = new_uid()
    comm = None
    try:
        comm = create(uid)
    except RuntimeError as e:
        err = e
    ok = comm is not None
    if world_size > 1:
        ok = _agree(ok, flag_device)
    if not ok:
        if comm is not None:
            # its peers never finished (or gave up on) the collective init: ncclCommDestroy could
            # block on them, ncclCommAbort does not
            (comm.abort if hasattr(comm, "abort") else comm.destroy)()
        reason = f"framework RCCL communicator unavailable on some rank ({err if err is not None else 'another rank'})"
        warnings.warn(reason + "; falling back to --comm c10d")
        return _fell_back(reason, fallback)
    return comm


def _fell_back(reason: str, fallback):
    global LAST_FALLBACK_REASON
    LAST_FALLBACK_REASON = reason
    return fallback()


def _pg_comm(C, dev: int):
    """ProcessGroupComm over the default group: a device backend (nccl = RCCL) is required."""
    if not dist.is_initialized():
        raise RuntimeError("--comm c10d needs an initialised torch.distributed process group")
    if dist.get_backend() != "nccl":
        raise RuntimeError(f"--comm c10d needs the nccl (RCCL) backend, not {dist.get_backend()!r}")
    return C.ProcessGroupComm(dist.group.WORLD, dev)


def broadcast_(tensor: torch.Tensor, comm, src: int = 0) -> None:
    """Broadcast on the current stream through the device comm (GPU) or torch.distributed."""
    if comm is not None:
        comm.broadcast(tensor, src)
    elif dist.is_initialized() and dist.get_world_size() > 1:
        dist.broadcast(tensor, src)


def all_reduce_(tensor: torch.Tensor, comm=None) -> None:
    if comm is not None:
        comm.all_reduce(tensor, True)
    elif dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(tensor)


def check(comm) -> None:
    """Host touch point: raise if the communicator's watchdog tripped (no-op without one)."""
    if comm is not None:
        comm.check()
