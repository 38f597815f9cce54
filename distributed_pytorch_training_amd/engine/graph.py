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
* the first replay is validated (``validate``): from one saved training state the step runs
  eagerly twice and is replayed twice; the whole gradient and every parameter's gradient must
  agree (replay vs eager and replay vs replay) within ``VALIDATE_NOISE_K`` x the measured
  eager-vs-eager / replay-vs-replay spread of that state, floored per dtype (``check_replay``),
  or the trainer falls back to eager with a warning naming the parameter.
  MIOpen's graph-unsafe CK backward-weights solver (utils/env.py ``GRAPH_UNSAFE_MIOPEN_SOLVERS``,
  excluded when the GraphedStep is built) produced per-parameter errors of 1e5-1e37;
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
import os
import warnings

import torch


AUTO_GRAPH_MAX_PIXELS = 1 << 18
# Replay validation (check_replay): relative L2 differences ||g_a - g_b|| / ||g_b||, over the whole
# gradient arena and per parameter, judged against the noise measured from the SAME state: two
# eager steps and two replays.  A replayed gradient may differ from eager by at most
# VALIDATE_NOISE_K x the larger self-spread (eager-vs-eager, replay-vs-replay) of that parameter,
# and never less than the per-dtype floor below - the rounding a correct replay of a deterministic
# step shows (eager and replay run the same kernels: the capture's split-K policy is used for the
# eager steps too).  Measured on the fp32 ResNet-18 default path (bench/replay_noise.py,
# profiles/replay_noise_r5.md): replay-vs-eager 8e-7..4e-6 whole, <= 1.2e-5 per parameter.  A
# replay-unsafe kernel (MIOpen's CK grouped backward solvers: 1e5..1e37) or a stale read (O(1))
# is far outside; tests/test_graph_replay_gpu.py injects a 30 % error into one parameter.
VALIDATE_NOISE_K = 4.0
VALIDATE_FLOOR = {True: (1e-4, 1e-3), False: (1e-3, 1e-2)}   # fp32?: (whole, per parameter)
# Eager steps that are not reproducible from the saved state beyond this (whole arena, any single
# parameter) depend on state outside the snapshot (host-side values read by forward: exactly what
# a captured graph bakes in) - the step is not replay-safe whatever the replays show.
VALIDATE_NOISE_CAP = (1e-2, 1e-1)


def step_state(trainer) -> dict:
    """Every tensor one native training step reads and writes, restorable in place: fp32 master
    parameters, optimizer state and step counter, module buffers (BN running statistics), 16-bit
    weight shadows, device-side AMP scaler state and the device metrics."""
    t = trainer
    out = {"param": t.ddp.arena.param_flat, "step": t.optimizer._step, "metrics": t.metrics}
    for i, st in enumerate(t.optimizer.arena_state() if hasattr(t.optimizer, "arena_state") else []):
        if st is not None:
            out[f"opt{i}"] = st
    for n, b in t.module.named_buffers():
        out["buf:" + n] = b
    if t.ddp.shadow_flat is not None:
        out["shadow"] = t.ddp.shadow_flat
    for k in ("scale_tensor", "growth_tracker", "found_inf"):
        v = getattr(t.scaler, k, None)
        if isinstance(v, torch.Tensor):
            out["scaler:" + k] = v
    return out


def snapshot(trainer) -> dict:
    return {k: v.detach().clone() for k, v in step_state(trainer).items()}


def restore(trainer, snap: dict) -> None:
    with torch.no_grad():
        for k, v in step_state(trainer).items():
            v.copy_(snap[k])


@contextlib.contextmanager
def _graph_splitk_policy():
    """Run an eager step with the K-loop splits a capture chooses (ops/conv split-K policy, mode 2):
    eager launches split fewer small grids than captured ones, which changes the summation order,
    and bf16 steps of a small-batch network amplify that past any useful tolerance (24 % of the
    gradient at batch 32, both paths equally far from fp32: profiles/graph_replay_miopen_r4.md).
    With the same splits, eager and replay run the same kernels and must agree to rounding."""
    from .. import ops
    if not ops.native_available():
        yield
        return
    C = ops.native()
    old = C.conv_get_splitk()
    if old == 1:
        C.conv_set_splitk(2)
    try:
        yield
    finally:
        C.conv_set_splitk(old)


def _has_randomness(module) -> bool:
    """Dropout-like modules draw fresh random numbers per run: eager and replay differ legitimately."""
    return any(isinstance(m, torch.nn.modules.dropout._DropoutNd) and m.p > 0 for m in module.modules())


# communicators whose collectives a hipGraph can hold: the framework's RCCL communicator (captured
# ncclAllReduce on its comm stream, tests/test_graph_rccl_gpu.py) and the asynchronous host bridge
# (host-function nodes).  The synchronous bridge blocks on the stream; torch's c10d communicator
# is not captured by default.
GRAPH_COMMS = ("rccl", "host-async")


def auto_enabled(args, device, world_size: int = 1, comm_kind: str | None = None) -> bool:
    """The ``--cuda-graph`` default: replay when the step is launch-bound - at any world size
    whose communicator can be captured (``comm_kind``: the communicator actually created, else
    ``--comm``).  At N > 1 the capture outcome is MIN-agreed over the ranks and the first replay
    is validated against eager steps on every rank (``GraphedStep``), so a rank whose capture or
    replay disagrees puts every rank back on eager steps."""
    if torch.device(device).type != "cuda" or getattr(args, "impl", "native") != "native":
        return False
    if getattr(args, "profile_sync", False) or getattr(args, "grad_accum", 1) != 1:
        return False
    if world_size > 1 and (comm_kind or getattr(args, "comm", "rccl")) not in GRAPH_COMMS:
        return False
    return int(args.batch_size) * int(args.image_size) ** 2 <= AUTO_GRAPH_MAX_PIXELS


class GraphedStep:
    def __init__(self, trainer, warmup: int = 3, validate: bool | None = None) -> None:
        from ..utils.env import graph_safe_miopen
        # effective only if no convolution has run in this process yet (MIOpen reads it once);
        # engine/run.py and the GPU test session call it at process start
        graph_safe_miopen()
        self.trainer = trainer
        self.warmup = warmup
        if validate is None:
            validate = os.environ.get("DPT_GRAPH_VALIDATE", "1") != "0"
        self.validate = validate
        self.validation = None     # check_replay's record once run
        self.inject = None         # testing: callable(grad_flat, arena) applied to each validation replay
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
        if self.validate and self.validation is None:
            return self._validated_first_replay(x, y)
        return self._replay(x, y)

    def reset(self) -> None:
        """Drop the captured graph, then free what the communicator kept alive for it (the
        asynchronous host bridge's host-node jobs and pinned staging buffers).  Called when the
        step falls back to eager and by ``Trainer.close`` (before the communicator is destroyed)."""
        if self.graph is None:
            return
        torch.cuda.synchronize()
        self.graph.reset()
        self.graph = None
        comm = self.trainer.ddp.comm if self.trainer.ddp is not None else None
        release = getattr(comm, "release_graph_resources", None)
        if release is not None:
            release()

    def _replay(self, x: torch.Tensor, y: torch.Tensor):
        t = self.trainer
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

    def _validated_first_replay(self, x: torch.Tensor, y: torch.Tensor):
        """From one saved state: two eager steps, then two replays; compare every parameter's
        gradient against the measured noise of the same state (``check_replay``).  Leaves the
        state of the last replay (the step this call stands for)."""
        t = self.trainer
        arena = t.ddp.arena
        names = list(getattr(arena, "names", [])) or [str(i) for i in range(len(arena.params))]
        if _has_randomness(t.module):
            self.validation = {"ok": True, "skipped": "model draws random numbers (dropout)"}
            return self._replay(x, y)
        torch.cuda.synchronize()
        s0 = snapshot(t)
        g = {}
        for name in ("eager1", "eager2"):
            restore(t, s0)
            with self._on_stream(), _graph_splitk_policy():
                t._native_step(x, y)
            t.global_step -= 1
            torch.cuda.synchronize()
            g[name] = arena.grad_flat.detach().clone()
        out = None
        for name in ("replay1", "replay2"):
            restore(t, s0)
            out = self._replay(x, y)
            if name == "replay1":
                t.global_step -= 1
                self.replays -= 1
            torch.cuda.synchronize()
            g[name] = arena.grad_flat.detach().clone()
            if self.inject is not None:      # testing: a replay-unsafe kernel's wrong gradient
                self.inject(g[name], arena)
        fp32 = not getattr(t, "amp", False)
        self.validation = check_replay(g, arena.views, names, fp32)
        ok = self.validation["ok"]
        if t.world_size > 1:
            ok = agree(ok, t.device)
            self.validation["ok"] = ok
        if os.environ.get("DPT_GRAPH_VALIDATE_DEBUG") == "1":   # diagnostics
            plan = t.ddp.plan
            rep2, eager = g["replay2"], g["eager1"]
            self.validation["bucket_replay_vs_eager"] = [
                round(((rep2[o:o + n] - eager[o:o + n]).double().norm() /
                       eager[o:o + n].double().norm().clamp_min(1e-30)).item(), 4)
                for o, n in zip(plan.offsets, plan.numels)]
            print(f"[graph validate] rank {t.rank}: {self.validation}", flush=True)
        if not ok:
            v = self.validation
            why = ("" if v["eager_reproducible"] else
                   "eager steps from the same saved state are not reproducible (forward reads state outside "
                   "the step's tensors, which a graph bakes in); ")
            warnings.warn(
                why + f"hipGraph replay disagrees with eager execution beyond the measured noise "
                f"(whole gradient: replay-vs-eager {v['replay_vs_eager']:.3g}, replay-vs-replay "
                f"{v['replay_vs_replay']:.3g}, eager-vs-eager {v['eager_vs_eager']:.3g}, tolerance "
                f"{v['tol_whole']:.3g}; worst parameter {v['worst']}: {v['worst_ratio']:.3g} x its tolerance); "
                "a kernel in the step is not replay-safe - running eagerly from now on"
                + (" (torch.backends.cudnn.deterministic is set: MIOpen then picks its CK grouped "
                   "backward-data solver, which is wrong under replay)" if torch.backends.cudnn.deterministic else ""))
            self.failed = True
            t.global_step -= 1
            self.replays -= 1
            restore(t, s0)
            self.reset()
            with self._on_stream():
                return t._native_step(x, y)
        return out

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
            # every failure path (this rank's capture raised, or another rank's did): drop what
            # was captured and the host-bridge jobs / pinned staging it kept alive
            self.failed = True
            try:
                g.reset()
            except Exception:       # nothing was captured
                pass
            torch.cuda.synchronize()
            release = getattr(comm, "release_graph_resources", None)
            if release is not None:
                release()
            return
        self.graph, self.out, self.loss = g, out, loss


def check_replay(g: dict, views, names, fp32: bool) -> dict:
    """Noise-relative replay check over gradients ``g`` = {eager1, eager2, replay1, replay2}, all
    taken from one saved state.  Over the whole arena and for every parameter:

    * replay-vs-replay <= max(VALIDATE_NOISE_K x eager-vs-eager, floor): a replay may be no less
      reproducible than eager execution (a stale or racy read varies between replays);
    * replay-vs-eager <= max(VALIDATE_NOISE_K x max(eager-vs-eager, replay-vs-replay), floor):
      a replay that is reproducibly wrong differs from eager beyond either path's own spread.

    The floor is per dtype (VALIDATE_FLOOR)."""
    fw, fp = VALIDATE_FLOOR[bool(fp32)]

    def rel(a, b, scale):
        r = (a - b).double().norm().item() / max(b.double().norm().item(), scale)
        return r if r == r else float("inf")     # NaN anywhere is a failure

    e1, e2, r1, r2 = g["eager1"], g["eager2"], g["replay1"], g["replay2"]
    K = VALIDATE_NOISE_K

    def verdict(ee, rr, re_, floor_):
        """Largest (difference / its tolerance) of the two conditions."""
        return max(rr / max(K * ee, floor_), re_ / max(K * max(ee, rr), floor_))

    ee, rr, re_ = rel(e2, e1, 1e-30), rel(r2, r1, 1e-30), rel(r2, e1, 1e-30)
    whole_ratio = verdict(ee, rr, re_, fw)
    # a parameter whose gradient is ~0 compares against the arena's scale
    scale = max(1e-6 * e1.double().norm().item(), 1e-30)
    worst, worst_name, worst_abs, param_ee = 0.0, "", 0.0, 0.0
    for n, a1, a2, b1, b2 in zip(names, views(e1), views(e2), views(r1), views(r2)):
        pe, pr, pre = rel(a2, a1, scale), rel(b2, b1, scale), rel(b2, a1, scale)
        param_ee = max(param_ee, pe)
        v = verdict(pe, pr, pre, fp)
        if v > worst or v != v:
            worst, worst_name, worst_abs = (float("inf") if v != v else v), n, max(pr, pre)
    ok = whole_ratio <= 1.0 and worst <= 1.0
    reproducible = ee <= VALIDATE_NOISE_CAP[0] and param_ee <= VALIDATE_NOISE_CAP[1]
    ok = ok and reproducible
    tol = max(K * max(ee, rr), fw)
    return {"ok": ok, "replay_vs_eager": re_, "replay_vs_replay": rr, "eager_vs_eager": ee, "tol_whole": tol,
            "worst": worst_name, "worst_ratio": worst, "param_worst_rel": worst_abs,
            "eager_reproducible": reproducible, "param_eager_vs_eager": param_ee}


def agree(ok: bool, device) -> bool:
    """All ranks' capture outcomes, MIN-reduced over the control-plane process group."""
    import torch.distributed as dist
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return ok
    on = device if dist.get_backend() == "nccl" else "cpu"
    flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=on)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    return bool(flag.item())
