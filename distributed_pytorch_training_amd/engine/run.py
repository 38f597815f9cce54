"""Orchestration: the reference's ``main()`` (reference train_ddp.py:314-386) on the native stack.

Sequence: parse args -> mkdir output dir -> distributed bootstrap ->
seed(seed + rank) -> rank-0 banner -> cudnn.benchmark -> data -> model -> DDP wrap ->
criterion / optimizer / scaler -> rank-0 CSV header (only if the file is absent) -> epochs
(train -> validate -> rank-0 epoch line + CSV row) -> teardown.  The CSV schema and the
stdout lines are the reference's, byte for byte.  Extensions (perf CSV, sync profile,
checkpoints) write to separate files so the reference artefacts are untouched.
"""
from __future__ import annotations

import json
import os
from pathlib import Path
from typing import Optional, Sequence

import torch

from ..config import parse_args
from ..data import get_dataloaders
from ..models import build_model
from ..utils.checkpoint import load_checkpoint, save_checkpoint
from ..utils.dist import cleanup_distributed, init_distributed, set_seed
from ..utils.env import graph_safe_miopen, setup_miopen_env, setup_tunableop
from ..utils.fault import FaultSpec
from .trainer import Trainer, format_epoch_line

CSV_HEADER = "epoch,train_loss,train_acc,val_loss,val_acc,epoch_time_seconds\n"
PERF_HEADER = "epoch,step,window_seconds,window_samples,throughput_samples_per_s\n"


def csv_row(epoch: int, tl: float, ta: float, vl: float, va: float, et: float) -> str:
    return f"{epoch},{tl:.4f},{ta:.2f},{vl:.4f},{va:.2f},{et:.4f}\n"


def main(argv: Optional[Sequence[str]] = None) -> int:
    args = parse_args(argv)
    Path(args.output_dir).mkdir(parents=True, exist_ok=True)
    setup_miopen_env()
    shared = bool(getattr(args, "rehearse_shared_gpu", False))
    if shared and args.comm not in ("host", "host-async"):
        raise SystemExit("--rehearse-shared-gpu needs --comm host or --comm host-async (RCCL needs one GPU per rank)")
    info = init_distributed(args.backend, args.dist_timeout, shared_gpu=shared)
    rank, world_size, device = info.rank, info.world_size, info.device
    if args.impl == "native" and device.type == "cuda":
        setup_tunableop()
        from .graph import auto_enabled
        cg = args.cuda_graph if args.cuda_graph is not None else auto_enabled(args, device, world_size)
        if cg:
            graph_safe_miopen()     # before the first convolution (utils/env.py)
    set_seed(args.seed, rank)

    if rank == 0:
        print(f"Using device: {device}, world_size={world_size}, amp={args.amp}", flush=True)
    torch.backends.cudnn.benchmark = True

    train_loader, val_loader, train_sampler = get_dataloaders(args, rank, world_size, device)
    model = build_model(args.model, args.num_classes, device, image_size=args.image_size,
                        channels_last=args.channels_last)
    trainer = Trainer(model, args, rank, world_size, device,
                      log=lambda s: print(s, flush=True))

    start_epoch = 0
    resume = args.resume
    if resume == "auto":   # elastic restart: the last checkpoint of this output dir, if any
        ck = Path(args.output_dir) / "checkpoint.pt"
        resume = str(ck) if ck.exists() else None
    if resume:
        start_epoch = load_checkpoint(resume, trainer)
        if rank == 0:
            print(f"Resumed from {resume} at epoch {start_epoch}", flush=True)

    metrics_path = Path(args.output_dir) / "metrics_rank0.csv"
    perf_path = Path(args.output_dir) / "metrics_perf_rank0.csv"
    if rank == 0:
        if not metrics_path.exists():
            with metrics_path.open("w") as f:
                f.write(CSV_HEADER)
        if not perf_path.exists():
            with perf_path.open("w") as f:
                f.write(PERF_HEADER)

    try:
        _epochs(args, trainer, train_loader, val_loader, train_sampler, start_epoch, rank, world_size,
                metrics_path, perf_path)
    except BaseException as e:
        if world_size <= 1:
            raise
        # abort the device communicator (peers stuck in a collective error out
        # instead of hanging), then leave non-zero without waiting on collectives a dead peer
        # will never join (destroy_process_group / atexit handlers could block).
        trainer.abort()
        import traceback
        traceback.print_exc()
        print(f"rank {rank}: training failed ({type(e).__name__}: {e}); exiting", flush=True)
        import sys
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(1)
    g = trainer.graphed
    if g is not None:   # stderr: the reference's stdout lines stay byte-identical
        import sys
        v = g.validation or {}
        print(f"[dpt] rank {rank}: hipGraph captured={g.graph is not None} failed={g.failed} replays={g.replays} "
              f"validation_ok={v.get('ok')} replay_vs_eager={v.get('replay_vs_eager')} "
              f"param_checksum={trainer.ddp.arena.param_flat.double().sum().item():.17g}", file=sys.stderr, flush=True)
    trainer.close()
    cleanup_distributed()
    return 0


def _epochs(args, trainer, train_loader, val_loader, train_sampler, start_epoch, rank, world_size,
            metrics_path, perf_path) -> None:
    fault = FaultSpec.parse(args.fault_inject)
    for epoch in range(start_epoch, args.epochs):
        if fault is not None and fault.epoch == epoch and fault.rank == rank:
            fault.fire(args.output_dir, lambda s: print(s, flush=True))  # once per output dir
        st = trainer.train_one_epoch(epoch, train_loader, train_sampler)
        if args.validate:
            vs = trainer.validate(val_loader)
            vl, va = vs.loss, vs.acc
        else:
            vl, va = float("nan"), float("nan")
        if args.check_consistency:
            trainer.check_consistency()
        if rank == 0:
            print(format_epoch_line(epoch, args.epochs, st.loss, st.acc, vl, va, st.epoch_time), flush=True)
            with metrics_path.open("a") as f:
                f.write(csv_row(epoch + 1, st.loss, st.acc, vl, va, st.epoch_time))
            with perf_path.open("a") as f:
                wins = st.windows or [{"step": st.steps, "seconds": st.epoch_time,
                                       "samples": st.samples, "throughput": st.samples / max(st.epoch_time, 1e-9)}]
                for w in wins:
                    f.write(f"{epoch+1},{w['step']},{w['seconds']:.6f},{w['samples']},{w['throughput']:.2f}\n")
            if args.save_every and (epoch + 1) % args.save_every == 0:
                save_checkpoint(str(Path(args.output_dir) / "checkpoint.pt"), trainer, epoch + 1, args)
        if args.save_every and (epoch + 1) % args.save_every == 0 and world_size > 1:
            # nobody starts the next epoch before the checkpoint is on disk: a failure from here on
            # restarts (--resume auto) from this epoch, never from an older one
            import torch.distributed as dist
            dist.barrier()

    if trainer.timeline.enabled and rank == 0:
        out = args.profile_out or str(Path(args.output_dir) / "sync_profile.json")
        extra = {"world_size": world_size, "model": args.model, "batch_size": args.batch_size,
                 "amp": args.amp, "amp_dtype": args.amp_dtype,
                 "buckets_mib": trainer.ddp.bucket_sizes_mib() if trainer.ddp else []}
        trainer.timeline.dump(out, extra)
        print("sync-profile " + json.dumps(trainer.timeline.summary()), flush=True)
