"""hipGraph capture of the whole native training step (``--cuda-graph``).

The native step has no host synchronisation (device-resident scaler, fused optimizer,
device metrics, C++ reducer with event-ordered RCCL), so forward + backward (+ bucketed
all-reduce on the comm stream) + optimizer can be captured once and replayed: one
``hipGraphLaunch`` per step instead of ~750 kernel launches.  That matters when the step is
launch-bound (the reference's own ResNet-18 / 32x32 CIFAR workload), not for GPU-bound
ResNet-50 at batch 256.

Stream discipline: autograd runs each AccumulateGrad node on the stream that was current
when the node was created, and the C++ reducer keeps those nodes alive from construction
(on the default stream).  A capture on a side stream would then need a default-stream sync
inside the capture (illegal).  So graph mode owns ONE stream: the reducer is rebuilt under
it (recreating the accumulator nodes there), and the warmup steps, the capture and every
replay run on it, ordered against the caller's stream with wait_stream.

Rules (checked or documented):
* ``warmup`` eager steps run first - MIOpen kernels get compiled/found, the reducer
  rebuilds its buckets, the optimizer allocates its state;
* shapes are static: a batch of another shape (the short last batch) runs eagerly;
* hyper-parameters are baked into the graph (constant LR, as in the reference);
* the profiling timeline is incompatible (it reads events on the host) and disables replay;
* any capture failure falls back to eager execution with a warning;
* the communicator watchdog gets one completion marker per replay (``Collective.track``),
  since the captured collectives never pass through ``RcclComm::all_reduce``.

Default (``--cuda-graph`` not given): on for launch-bound steps only - per-GPU batch x
pixels <= ``AUTO_GRAPH_MAX_PIXELS`` (the reference's own ResNet-18 / 32x32 / batch 128 is
131k; ResNet-50 / 224 / 256 is 12.8M and GPU-bound) - and only at world size 1: replayed RCCL
collectives have run on no multi-GPU node yet, so N > 1 replays only when asked for
(``--cuda-graph``).  ``--no-cuda-graph`` turns it off.

Multi-rank capture: every rank must take the same path (a rank replaying while another runs
eagerly still pairs its collectives, but the steps would no longer be the same program), so
after its capture each rank contributes "captured OK" to a MIN all-reduce over the control
plane and all fall back to eager together if any failed.  The synchronous host bridge
(``--comm host``) cannot be captured (it blocks on the stream) and is refused up front; the
asynchronous one records its host collectives as graph host nodes (csrc/host_comm.cpp).
"""
from __future__ import annotations

import contextlib
import gc
import warnings

import torch


AUTO_GRAPH_MAX_PIXELS = 1 << 18


def auto_enabled(args, device, world_size: int = 1) -> bool:
    """The ``--cuda-graph`` default: replay when the step is launch-bound."""
    if torch.device(device).type != "cuda" or getattr(args, "impl", "native") != "native":
        return False
    if getattr(args, "profile_sync", False) or getattr(args, "grad_accum", 1) != 1:
        return False
    if world_size > 1:
        return False
    return int(args.batch_size) * int(args.image_size) ** 2 <= AUTO_GRAPH_MAX_PIXELS


class GraphedStep:
    def __init__(self, trainer, warmup: int = 3) -> None:
        self.trainer = trainer
        self.warmup = warmup
        self.graph = None
        self.failed = False
        self.calls = 0
        self.replays = 0
        self.stream = None
        self.static_x = self.static_y = None
        self.out = self.loss = None

    @contextlib.contextmanager
    def _on_stream(self):
        caller = torch.cuda.current_stream()
        self.stream.wait_stream(caller)
        with torch.cuda.stream(self.stream):
            yield
        caller.wait_stream(self.stream)

    def _own_stream(self) -> None:
        t = self.trainer
        torch.cuda.synchronize()
        self.stream = torch.cuda.Stream(device=t.device)
        with torch.cuda.stream(self.stream):
            t.ddp._build_reducer()      # accumulator nodes (re)created on the graph stream

    def __call__(self, x: torch.Tensor, y: torch.Tensor):
        t = self.trainer
        if self.failed or t.timeline.enabled:
            return t._native_step(x, y)
        if self.stream is None:
            self._own_stream()
        if self.graph is None:
            if self.calls < self.warmup:
                self.calls += 1
                with self._on_stream():
                    return t._native_step(x, y)
            self._capture(x, y)
            if self.failed:
                with self._on_stream():
                    return t._native_step(x, y)
        if x.shape != self.static_x.shape or y.shape != self.static_y.shape:
            with self._on_stream():
                return t._native_step(x, y)
        with self._on_stream():
            self.static_x.copy_(x)
            self.static_y.copy_(y)
            self.graph.replay()
            if t.ddp.comm is not None:
                # the replayed all-reduces bypass RcclComm::all_reduce: give the watchdog a
                # completion marker behind them so --dist-timeout covers graph steps too
                t.ddp.comm.track()
        self.replays += 1
        t.global_step += 1
        return self.out, self.loss

    def _capture(self, x: torch.Tensor, y: torch.Tensor) -> None:
        t = self.trainer
        torch.cuda.synchronize()
        self.static_x = x.clone()
        self.static_y = y.clone()
        g = torch.cuda.CUDAGraph()
        comm = t.ddp.comm if t.ddp is not None else None
        ok = True
        if comm is not None and comm.kind == "host":
            warnings.warn("hipGraph replay disabled: the synchronous host bridge (--comm host) blocks on "
                          "the stream and cannot be captured; use --comm host-async")
            ok = False
        else:
            # No Python garbage collection while the stream is captured: a cycle collected there
            # runs destructors (graphs, allocator pools, extension objects of earlier trainers)
            # whose HIP calls are illegal during capture - one such collection aborted the
            # process in a GPU test run.  torch.cuda.graph collects once before it starts.
            gc_was = gc.isenabled()
            gc.disable()
            try:
                with torch.cuda.graph(g, stream=self.stream):
                    out, loss = t._native_step(self.static_x, self.static_y)
                t.global_step -= 1          # the captured call counted a step that did not run
                torch.cuda.synchronize()
            except Exception as e:  # capture is an optimisation: never fatal
                warnings.warn(f"hipGraph capture failed, running eagerly: {e!r}")
                ok = False
                torch.cuda.synchronize()
            finally:
                if gc_was:
                    gc.enable()
        if t.world_size > 1 and not agree(ok, t.device):
            if ok:
                warnings.warn("hipGraph capture failed on another rank: every rank runs eagerly")
            ok = False
        if not ok:
            self.failed = True
            return
        self.graph, self.out, self.loss = g, out, loss


def agree(ok: bool, device) -> bool:
    """All ranks' capture outcomes, MIN-reduced over the control-plane process group."""
    import torch.distributed as dist
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return ok
    on = device if dist.get_backend() == "nccl" else "cpu"
    flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=on)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    return bool(flag.item())
