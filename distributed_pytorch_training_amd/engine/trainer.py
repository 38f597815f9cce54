"""Training / validation engine.

Output contract (byte-identical to the reference):
* step line every ``print_freq`` steps on rank 0 (reference train_ddp.py:228-244);
* epoch train metrics = SUM-all-reduced (loss*bs, correct, total) (reference :247-263);
* validation over the full, unsharded split on every rank (reference :266-300).

Two engines share that contract:
* ``impl="torch"`` - the reference's exact mechanics on PyTorch-ROCm: torch DDP with
  defaults, ``torch.amp.GradScaler``, foreach SGD/Adam, two ``.item()`` host syncs per
  step.  This is the stock baseline the native engine is measured against.
* ``impl="native"`` - the MI355X path: ``NativeDDP`` (flat arenas + C++ reducer over RCCL),
  ``DeviceGradScaler``, one fused HIP optimizer launch, device-side metric accumulation;
  zero host synchronisations per step.  The host syncs at print boundaries only, so the
  throughput window is timed from sync to sync (the reference's window times each step
  after the loader yields; with on-device loaders the loader wait is a kernel launch).
"""
from __future__ import annotations

import contextlib
import os
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from .. import ops
from ..amp import DeviceGradScaler, autocast
from ..ops import conv as native_conv
from ..profiling.timeline import StepTimeline, roctx_range
from ..utils.dist import all_reduce_


def format_step_line(epoch: int, i: int, n: int, avg_loss: float, avg_acc: float, thr: float) -> str:
    return (f"Epoch [{epoch+1}] Step [{i+1}/{n}] "
            f"Loss: {avg_loss:.4f}  "
            f"Acc: {avg_acc:.2f}%  "
            f"Throughput: {thr:.2f} samples/s (global)")


def format_epoch_line(epoch: int, epochs: int, tl: float, ta: float, vl: float, va: float, et: float) -> str:
    return (f"[Epoch {epoch+1}/{epochs}] "
            f"Train: loss={tl:.4f}, acc={ta:.2f}% | "
            f"Val: loss={vl:.4f}, acc={va:.2f}% | "
            f"Epoch time: {et:.2f}s")


@dataclass
class EpochStats:
    loss: Optional[float]
    acc: Optional[float]
    epoch_time: float
    steps: int = 0
    samples: int = 0
    windows: List[Dict[str, float]] = field(default_factory=list)


def _sync(device: torch.device) -> None:
    if device.type == "cuda":
        torch.cuda.synchronize(device)


class Trainer:
    """Owns model/optimizer/scaler wiring for one of the two engines."""

    def __init__(self, model: nn.Module, args, rank: int, world_size: int, device: torch.device,
                 comm=None, log: Callable[[str], None] = print) -> None:
        self.args, self.rank, self.world_size, self.device = args, rank, world_size, device
        self.impl = args.impl
        self.log = log
        self.amp = bool(args.amp)
        self.amp_dtype = getattr(args, "amp_dtype", "fp16")
        self.criterion = nn.CrossEntropyLoss().to(device)
        self.timeline = StepTimeline(device, enabled=getattr(args, "profile_sync", False))
        self.global_step = 0
        self.grad_accum = max(1, getattr(args, "grad_accum", 1))
        self._accum_fresh = True
        self.roctx = bool(getattr(args, "roctx", False))
        self.graphed = None
        self._native_conv_cache = False
        if self.impl == "native":
            self._init_native(model, comm)
        else:
            self._init_torch(model)

    # ------------------------------------------------------------------ construction
    def _init_native(self, model: nn.Module, comm) -> None:
        from ..models.layers import fuse_native_layers, set_conv_routing
        from ..optim import build_optimizer
        from ..parallel.ddp import NativeDDP

        args = self.args
        from ..models.vit import set_native as vit_set_native
        vit_set_native(model, self.device.type == "cuda")   # fused ViT encoder (no-op for other models)
        gpu_cl = self.device.type == "cuda" and bool(getattr(args, "channels_last", False))
        # MFMA convs need channels_last bf16/fp16 activations; routing is per model
        use_native_conv = gpu_cl and bool(getattr(args, "native_conv", True)) and native_conv.ENABLED
        if use_native_conv:
            from .. import ops
            sk = {"off": 0, "auto": 1, "all": 2}[getattr(args, "conv_streamk", "off")]
            ops.native().conv_set_streamk(sk)   # process-wide, like the other conv policies
            self._streamk = bool(sk)
            if sk:
                ops.native().conv_sk_prepare()  # workspace before any graph capture
        # every supported conv runs native: small tile grids split their K loop (split-K,
        # conv_kernels.hip), which made the MFMA path faster than MIOpen on ResNet-18 / 32x32
        # under hipGraph too; DPT_CONV_MIN_PIXELS still routes tiny convs to MIOpen
        min_px = None
        # --native-conv-fp32: this model's fp32 convs on the fp32 MFMA kernels (routing stored per
        # conv module, never process-wide: ADVICE r5)
        f32 = True if getattr(args, "native_conv_fp32", False) else None
        if f32 and not use_native_conv:
            import warnings
            warnings.warn("--native-conv-fp32 has no effect: the MFMA conv kernels need a GPU, channels_last "
                          "activations and native convs (no --no-native-conv)")
        if f32 and self.amp:
            import warnings
            warnings.warn("--native-conv-fp32 only affects fp32 convolutions; under --amp the 16-bit MFMA "
                          "kernels run")
        if getattr(args, "fused_bn", True) and gpu_cl:
            fuse_native_layers(model, native_conv=use_native_conv, min_pixels=min_px, native_f32=f32)
        else:
            set_conv_routing(model, use_native_conv, min_px, f32)
        # per-step flip cache of the stride-1 backward-data weights (ops/conv.py)
        self._native_conv_cache = use_native_conv
        params_in_order = [p for p in model.parameters() if p.requires_grad]
        self.scaler = DeviceGradScaler(self.device, enabled=self.amp)
        shadow = None
        if (self.amp and getattr(args, "weight_shadow", True) and self.grad_accum == 1
                and self.device.type == "cuda"):
            shadow = torch.bfloat16 if self.amp_dtype == "bf16" else torch.float16
        self.ddp = NativeDDP(model, rank=self.rank, world_size=self.world_size, device=self.device,
                             bucket_cap_mb=args.bucket_cap_mb, first_bucket_mb=args.first_bucket_mb,
                             last_bucket_mb=getattr(args, "last_bucket_mb", 0.0),
                             broadcast_buffers=args.broadcast_buffers, grad_dtype=args.grad_dtype,
                             found_inf=self.scaler.found_inf, scale=self.scaler.scale_tensor,
                             check_inf=self.amp, profile=self.timeline.enabled,
                             # a step's comm events are read max_pending steps later: they must
                             # still be that step's (one event slot per unresolved step + 1)
                             profile_slots=self.timeline.max_pending + 1, comm=comm,
                             weight_shadow=shadow, comm_kind=getattr(args, "comm", "rccl"),
                             timeout_s=getattr(args, "dist_timeout", None),
                             rccl_channels=getattr(args, "rccl_channels", 0),
                             debug=bool(getattr(args, "ddp_debug", False)))
        self.model = self.ddp
        self.module = model
        self.optimizer = build_optimizer(args.optimizer, self.ddp.arena, args, params_in_order)
        self.metrics = torch.zeros(3, dtype=torch.float64, device=self.device)
        self.graphed = None
        from .graph import GraphedStep, auto_enabled
        cg = getattr(args, "cuda_graph", False)
        if cg is None:      # default: replay launch-bound steps (engine/graph.py)
            comm = self.ddp.comm
            cg = auto_enabled(args, self.device, self.world_size, comm.kind if comm is not None else None)
        if cg and self.device.type == "cuda":
            self.graphed = GraphedStep(self)

    def _init_torch(self, model: nn.Module) -> None:
        args = self.args
        self.module = model
        if self.world_size > 1:
            kw = dict(device_ids=[self.device.index], output_device=self.device.index) \
                if self.device.type == "cuda" else {}
            self.model = nn.parallel.DistributedDataParallel(
                model, find_unused_parameters=False, bucket_cap_mb=args.bucket_cap_mb,
                broadcast_buffers=args.broadcast_buffers, **kw)
        else:
            self.model = model
        params = model.parameters()
        if args.optimizer == "sgd":
            self.optimizer = torch.optim.SGD(params, lr=args.lr, momentum=args.momentum,
                                             weight_decay=args.weight_decay,
                                             nesterov=getattr(args, "nesterov", False))
        elif args.optimizer == "adam":
            self.optimizer = torch.optim.Adam(params, lr=args.lr, betas=args.betas, eps=args.eps,
                                              weight_decay=args.weight_decay)
        else:
            self.optimizer = torch.optim.AdamW(params, lr=args.lr, betas=args.betas, eps=args.eps,
                                               weight_decay=args.weight_decay)
        self.scaler = torch.amp.GradScaler(self.device.type, enabled=self.amp and self.device.type == "cuda")
        self.ddp = None

    # ------------------------------------------------------------------ one step
    def train_step(self, images: torch.Tensor, targets: torch.Tensor, sync: bool = True):
        """Forward + backward (+ optimizer when ``sync``) for one batch; returns (outputs, loss).

        ``sync=False`` is a gradient-accumulation micro-batch (``--grad-accum``): no
        all-reduce (``no_sync``), no optimizer step, gradients keep accumulating.
        """
        if self.impl == "native":
            if self.graphed is not None and sync and self.grad_accum == 1:
                return self.graphed(images, targets)
            return self._native_step(images, targets, sync)
        return self._torch_step(images, targets, sync)

    def _native_step(self, images, targets, sync: bool = True):
        tl = self.timeline
        tl.mark("start")
        if self._native_conv_cache:
            native_conv.begin_step()  # weights changed since the last step: new flip cache
        else:
            native_conv.reset_side_channels()
        ctx = self.ddp.no_sync() if not sync else contextlib.nullcontext()
        rx = self.roctx
        with ctx:
            with roctx_range("forward", rx), autocast(self.device, self.amp, self.amp_dtype):
                outputs = self.model(images)
                loss = self.criterion(outputs, targets)
            tl.mark("fwd")
            scaled = loss / self.grad_accum if self.grad_accum > 1 else loss
            with roctx_range("backward+allreduce", rx):
                try:
                    (self.scaler.scale(scaled) if self.amp else scaled).backward()
                except BaseException:
                    native_conv.reset_side_channels()  # no stale BN-backward partials survive
                    raise
                finally:
                    if self._native_conv_cache:
                        native_conv.end_caching()
        tl.mark("bwd")
        if not sync:
            ops.accumulate_metrics(outputs, targets, loss, self.metrics)
            tl.discard()
            return outputs, loss
        if self.ddp.maybe_rebuild_buckets(self.optimizer) and self.rank == 0 and getattr(self.args, "verbose", False):
            self.log(f"rebuilt buckets: {self.ddp.bucket_sizes_mib()}")
        with roctx_range("optimizer", rx):
            self.optimizer.step(self.scaler if self.amp else None, host_factor=self.ddp.grad_factor,
                                grads_checked=self.ddp.grads_checked, shadow=self.ddp.shadow_flat,
                                zero_grad=not self.ddp.grads_overwritten)
        tl.mark("opt")
        ops.accumulate_metrics(outputs, targets, loss, self.metrics)
        tl.end_step(self.ddp.comm_profile_ref() if tl.enabled else None)
        self.global_step += 1
        return outputs, loss

    def _torch_step(self, images, targets, sync: bool = True):
        if self._accum_fresh:
            self.optimizer.zero_grad(set_to_none=True)
        use_scaler = self.amp and self.scaler.is_enabled()
        ctx = self.model.no_sync() if (not sync and hasattr(self.model, "no_sync")) else contextlib.nullcontext()
        with ctx:
            with autocast(self.device, self.amp, self.amp_dtype):
                outputs = self.model(images)
                loss = self.criterion(outputs, targets)
            scaled = loss / self.grad_accum if self.grad_accum > 1 else loss
            (self.scaler.scale(scaled) if use_scaler else scaled).backward()
        self._accum_fresh = sync
        if not sync:
            return outputs, loss
        if use_scaler:
            self.scaler.step(self.optimizer)
            self.scaler.update()
        else:
            self.optimizer.step()
        self.global_step += 1
        return outputs, loss

    # ------------------------------------------------------------------ epochs
    def _fault(self):
        """``--fault-inject rank=R,step=S`` for this rank (utils/fault.py), else None."""
        from ..utils.fault import FaultSpec
        spec = FaultSpec.parse(getattr(self.args, "fault_inject", None))
        return spec if spec is not None and spec.step is not None and spec.rank == self.rank else None

    def check_consistency(self) -> None:
        """Debug: parameters must be bit-identical across ranks; with
        ``--ddp-debug`` the device collective sequences must match too."""
        if self.world_size <= 1:
            return
        if self.ddp is not None:
            self.ddp.check_comm()
            flat = self.ddp.arena.param_flat
        else:
            flat = torch.cat([p.detach().reshape(-1) for p in self.module.parameters()])
        s = flat.double().sum().reshape(1)
        lo, hi = s.clone(), s.clone()
        all_reduce_(lo, op=dist.ReduceOp.MIN)
        all_reduce_(hi, op=dist.ReduceOp.MAX)
        if float(hi - lo) != 0.0:
            raise RuntimeError(f"parameters diverged across ranks: checksum range {float(lo)}..{float(hi)}")
        if self.ddp is not None and getattr(self.args, "ddp_debug", False):
            self.ddp.verify_sequence()

    def _host_touch(self) -> None:
        """Host touch point: surface a tripped communicator watchdog, or a stream-K conv whose
        consumer gave up waiting for a contributor (its tile was poisoned with NaN), as an
        exception."""
        if self.ddp is not None:
            self.ddp.check_comm()
        if getattr(self, "_streamk", False):
            from .. import ops
            n = ops.native().conv_sk_errors()
            if n:
                raise RuntimeError(f"stream-K convolution: {n} tile(s) gave up waiting for a contributing "
                                   "block (results poisoned with NaN); rerun with --conv-streamk off")

    def train_one_epoch(self, epoch: int, loader, train_sampler=None) -> EpochStats:
        """One epoch with the reference's stdout contract (train_ddp.py:170-263).

        Throughput windows: native default = sync-to-sync wall time over the window (no
        per-step host sync exists to time individual steps); ``--ref-throughput`` (and the torch
        engine always) = the reference's definition, the sum of per-step times measured from
        after the loader yields to after the step's host sync (train_ddp.py:196,224).
        ``--warmup-steps N``: the first N steps of the first epoch this trainer runs are left
        out of every window."""
        args, rank, ws = self.args, self.rank, self.world_size
        self.model.train()
        if train_sampler is not None:
            train_sampler.set_epoch(epoch)
        if hasattr(loader, "set_epoch") and train_sampler is None:
            loader.set_epoch(epoch)
        n = len(loader)
        native = self.impl == "native"
        ref_thr = (not native) or bool(getattr(args, "ref_throughput", False))
        warm = 0
        if not getattr(self, "_warmed", False):
            warm = max(0, int(getattr(args, "warmup_steps", 0) or 0))
            self._warmed = True
        check_every = int(getattr(args, "check_consistency", 0) or 0)
        fault = self._fault()
        if native:
            self.metrics.zero_()
        epoch_loss, epoch_correct, epoch_total = 0.0, 0, 0
        windows = []
        _sync(self.device)
        start_epoch = time.time()
        accum_time, accum_samples = 0.0, 0
        win_start = time.time()
        steps = 0
        for i, (images, targets) in enumerate(loader):
            if fault is not None and self.global_step >= fault.step:
                fault.fire(getattr(args, "output_dir", "."), self.log)   # dies; peers must not hang
            sync = (i + 1) % self.grad_accum == 0 or i + 1 == n
            batch_start = time.time()
            outputs, loss = self.train_step(images, targets, sync)
            bs = images.size(0)
            if native:
                if ref_thr:
                    _sync(self.device)
            else:
                epoch_loss += loss.item() * bs
                _, preds = outputs.max(1)
                epoch_correct += preds.eq(targets).sum().item()
                epoch_total += bs
            steps += 1
            if i < warm:
                if i + 1 == warm:          # warmup over: the windows start now
                    _sync(self.device)
                    win_start, accum_time, accum_samples = time.time(), 0.0, 0
                continue
            accum_time += time.time() - batch_start
            accum_samples += bs * ws
            if sync and check_every and self.global_step % check_every == 0:
                self.check_consistency()
            if rank == 0 and (i + 1) % args.print_freq == 0:
                if native:
                    _sync(self.device)
                    self._host_touch()
                    if not ref_thr:
                        accum_time = time.time() - win_start
                    m = self.metrics.tolist()
                    avg_loss, avg_acc = m[0] / m[2], 100.0 * m[1] / m[2]
                else:
                    avg_loss, avg_acc = epoch_loss / epoch_total, 100.0 * epoch_correct / epoch_total
                thr = accum_samples / accum_time if accum_time > 0 else 0.0
                self.log(format_step_line(epoch, i, n, avg_loss, avg_acc, thr))
                windows.append({"step": i + 1, "seconds": accum_time, "samples": accum_samples,
                                "throughput": thr})
                accum_time, accum_samples = 0.0, 0
                win_start = time.time()
        # ---- epoch reduction (one float64[3] all-reduce instead of three scalars)
        if native:
            tot = self.metrics.clone()
        else:
            tot = torch.tensor([epoch_loss, float(epoch_correct), float(epoch_total)],
                               dtype=torch.float64, device=self.device)
        if ws > 1:
            all_reduce_(tot)
        _sync(self.device)
        self._host_touch()
        epoch_time = time.time() - start_epoch
        t = tot.tolist()
        samples = int(t[2])
        if rank == 0 and t[2] > 0:
            return EpochStats(t[0] / t[2], 100.0 * t[1] / t[2], epoch_time, steps, samples, windows)
        return EpochStats(None, None, epoch_time, steps, samples, windows)

    @torch.no_grad()
    def validate(self, loader) -> EpochStats:
        """Full unsharded pass on every rank (reference train_ddp.py:266-300).  fp32 like the
        reference - no autocast even under ``--amp`` - unless ``--amp-val`` opts in."""
        self.model.eval()
        acc = torch.zeros(3, dtype=torch.float64, device=self.device)
        t0 = time.time()
        amp_val = self.amp and bool(getattr(self.args, "amp_val", False))
        for images, targets in loader:
            with autocast(self.device, amp_val, self.amp_dtype):
                outputs = self.model(images)
                loss = self.criterion(outputs, targets)
            if self.impl == "native":
                ops.accumulate_metrics(outputs, targets, loss, acc)
            else:
                bs = images.size(0)
                acc[0] += loss.item() * bs
                _, preds = outputs.max(1)
                acc[1] += preds.eq(targets).sum().item()
                acc[2] += bs
        if self.world_size > 1:
            all_reduce_(acc)
        t = acc.tolist()
        if self.rank == 0 and t[2] > 0:
            return EpochStats(t[0] / t[2], 100.0 * t[1] / t[2], time.time() - t0)
        return EpochStats(None, None, time.time() - t0)

    def sync_weights(self) -> None:
        """After externally loading parameters: refresh the 16-bit weight shadows."""
        if self.ddp is not None:
            self.ddp.refresh_shadow()

    def close(self) -> None:
        if self.graphed is not None:
            self.graphed.reset()        # before the communicator its host nodes may reference
        if self.ddp is not None:
            self.ddp.close()

    def abort(self) -> None:
        """Failure path: abort the RCCL communicator so peers blocked in a
        collective error out instead of hanging until the process-group timeout."""
        comm = getattr(self.ddp, "comm", None) if self.ddp is not None else None
        if comm is not None:
            comm.abort()

    # ------------------------------------------------------------------ checkpoint glue
    def model_state(self):
        return self.module.state_dict()

    def optimizer_state(self):
        return self.optimizer.state_dict()

    def scaler_state(self):
        return self.scaler.state_dict()
