"""Command-line contract.

The first eleven flags reproduce the reference's CLI exactly: names, types, defaults and
help strings (reference ``train_ddp.py:19-46``).  Everything after them is
additive, and every additive default reproduces the reference's behaviour
(resnet18 / CIFAR-10 / fp16 autocast / SGD / 25 MiB buckets / BN-buffer broadcast), except
``--impl``: the default ``native`` engine keeps the same semantics but runs the MI355X hot
path (HIP fused optimizer + device-resident scaler + RCCL reducer).
"""
from __future__ import annotations

import argparse
import os
from typing import Optional, Sequence


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="DDP training of ResNet-18 on CIFAR-10")

    # ---- reference flags (train_ddp.py:22-43) -------------------------------------------
    p.add_argument("--data-dir", default="./data", type=str,
                   help="directory to store CIFAR-10")
    p.add_argument("--epochs", default=10, type=int,
                   help="number of total epochs to run")
    p.add_argument("--batch-size", default=128, type=int,
                   help="mini-batch size *per GPU*")
    p.add_argument("--workers", default=4, type=int,
                   help="number of data loading workers per process")
    p.add_argument("--lr", default=0.1, type=float,
                   help="initial learning rate")
    p.add_argument("--momentum", default=0.9, type=float,
                   help="SGD momentum")
    p.add_argument("--weight-decay", default=5e-4, type=float,
                   help="weight decay")
    p.add_argument("--amp", action="store_true",
                   help="use automatic mixed precision (AMP)")
    p.add_argument("--print-freq", default=50, type=int,
                   help="print frequency (in steps)")
    p.add_argument("--output-dir", default="./experiments", type=str,
                   help="directory to save logs")
    p.add_argument("--seed", default=42, type=int,
                   help="random seed")

    # ---- additive flags ---------------------------------------------------
    g = p.add_argument_group("MI355X extensions (defaults reproduce the reference)")
    g.add_argument("--model", default="resnet18",
                   choices=["resnet18", "resnet34", "resnet50", "resnet101", "vit_b_16"],
                   help="model architecture")
    g.add_argument("--dataset", default="cifar10", choices=["cifar10", "synthetic"],
                   help="cifar10 reads local CIFAR-10 files; synthetic generates on-device data")
    g.add_argument("--image-size", default=None, type=int,
                   help="input resolution (default 32 for cifar10, 224 for synthetic)")
    g.add_argument("--num-classes", default=None, type=int,
                   help="number of classes (default 10 for cifar10, 1000 for synthetic)")
    g.add_argument("--synthetic-train-size", default=50000, type=int,
                   help="samples per epoch for --dataset synthetic")
    g.add_argument("--synthetic-val-size", default=10000, type=int,
                   help="validation samples for --dataset synthetic")
    g.add_argument("--synthetic-task", default="random", choices=["random", "prototypes"],
                   help="--dataset synthetic: random = a pool of 4 random batches with random labels "
                        "(benchmark input, memorisation only); prototypes = class prototype images plus "
                        "pixel noise, fresh every step, learnable and with a held-out validation split")
    g.add_argument("--synthetic-noise", default=2.0, type=float,
                   help="pixel noise std of --synthetic-task prototypes (prototypes have unit std)")
    g.add_argument("--amp-dtype", default="fp16", choices=["fp16", "bf16"],
                   help="autocast dtype when --amp is set (reference: fp16)")
    g.add_argument("--optimizer", default="sgd", choices=["sgd", "adam", "adamw"],
                   help="optimizer (reference: sgd)")
    g.add_argument("--nesterov", action="store_true", help="Nesterov momentum (SGD)")
    g.add_argument("--betas", default="0.9,0.999", type=str, help="Adam betas")
    g.add_argument("--eps", default=1e-8, type=float, help="Adam epsilon")
    g.add_argument("--impl", default="native", choices=["native", "torch"],
                   help="native: MI355X engine (HIP kernels, RCCL reducer); torch: stock DDP/foreach SGD/GradScaler")
    g.add_argument("--backend", default="auto", choices=["auto", "rccl", "nccl", "gloo"],
                   help="process-group backend (auto: rccl on GPUs, gloo on CPU)")
    g.add_argument("--bucket-cap-mb", default=25.0, type=float,
                   help="gradient bucket size cap in MiB")
    g.add_argument("--first-bucket-mb", default=1.0, type=float,
                   help="first (last-layer) bucket cap in MiB")
    g.add_argument("--last-bucket-mb", default=0.0, type=float,
                   help="native impl: cap of the bucket that becomes ready last (its all-reduce can not "
                        "overlap backward); 0 (default) = torch DDP's plan, where it is whatever is left "
                        "over; bench.py passes 1.0")
    g.add_argument("--no-broadcast-buffers", dest="broadcast_buffers", action="store_false",
                   help="do not broadcast BN buffers from rank 0 before each forward")
    g.add_argument("--grad-dtype", default="fp32", choices=["fp32", "bf16"],
                   help="all-reduce wire dtype (bf16 = gradient compression, native only)")
    g.add_argument("--channels-last", dest="channels_last", action="store_true", default=None,
                   help="NHWC activations/weights (default: on for the native engine on a GPU - the "
                        "layout every fused gfx950 kernel and MIOpen's fast convs use; same math)")
    g.add_argument("--no-channels-last", dest="channels_last", action="store_false",
                   help="keep the reference's NCHW layout")
    g.add_argument("--no-fused-bn", dest="fused_bn", action="store_false",
                   help="native impl: keep MIOpen BatchNorm + separate ReLU/add instead of the fused "
                        "gfx950 BN(+add)(+ReLU) kernels (channels_last GPU runs)")
    g.add_argument("--no-native-conv", dest="native_conv", action="store_false",
                   help="native impl: run convolutions on MIOpen instead of the hand-written MFMA "
                        "implicit-GEMM kernels (which also fuse the BatchNorm statistics pass)")
    g.add_argument("--native-conv-fp32", action="store_true",
                   help="native impl, fp32 (no --amp): run the convolutions on the hand-written fp32 MFMA "
                        "kernels (exact, bitwise deterministic, replay-safe) instead of MIOpen (faster on "
                        "ResNet-50: profiles/conv_f32_r5.md)")
    g.add_argument("--conv-streamk", choices=("off", "auto", "all"),
                   default=os.environ.get("DPT_CONV_STREAMK", "off"),
                   help="native impl: stream-K grids for the MFMA convs whose tiles spread unevenly over the "
                        "256 CUs (auto), for every eligible conv (all), or never (off; env DPT_CONV_STREAMK)")
    g.add_argument("--no-weight-shadow", dest="weight_shadow", action="store_false",
                   help="native impl: let autocast cast fp32 weights every forward instead of keeping "
                        "16-bit weight shadows updated by the fused optimizer")
    g.add_argument("--max-steps", default=0, type=int,
                   help="stop each epoch after this many steps (0 = full epoch)")
    g.add_argument("--warmup-steps", default=0, type=int,
                   help="the first N steps of the first epoch run but are excluded from the throughput "
                        "windows (step lines and metrics_perf_rank0.csv)")
    g.add_argument("--profile-sync", action="store_true",
                   help="hipEvent timeline: per-step forward/backward/all-reduce/optimizer times")
    g.add_argument("--profile-out", default=None, type=str,
                   help="JSON file for the --profile-sync report (default output-dir/sync_profile.json)")
    g.add_argument("--roctx", action="store_true", help="emit roctx ranges for rocprofv3 --marker-trace")
    g.add_argument("--grad-accum", default=1, type=int,
                   help="micro-batches per optimizer step (all-reduce only on the last)")
    g.add_argument("--save-every", default=0, type=int,
                   help="write a checkpoint every N epochs (0 = never, the reference default)")
    g.add_argument("--resume", default=None, type=str,
                   help="checkpoint file to resume from, or 'auto': output-dir/checkpoint.pt when it "
                        "exists (a job restarted by torchrun --max-restarts picks up its last epoch)")
    g.add_argument("--no-val", dest="validate", action="store_false", help="skip validation")
    g.add_argument("--dist-timeout", default=1800, type=int,
                   help="process-group timeout in seconds")
    g.add_argument("--check-consistency", default=0, type=int,
                   help="debug: every N optimizer steps (and at every epoch end) verify that parameters "
                        "are identical across ranks")
    g.add_argument("--comm", default="rccl", choices=["rccl", "c10d", "host", "host-async"],
                   help="device collective of the native reducer: rccl (the framework's own RCCL "
                        "communicator over xGMI; falls back to c10d if it cannot be created), c10d "
                        "(RCCL through torch's default process group), host (gloo through pinned host "
                        "staging - lets several ranks share one GPU; debug only); host-async enqueues "
                        "the host collective on the comm stream like RCCL, so backward overlaps it")
    g.add_argument("--rehearse-shared-gpu", action="store_true",
                   help="testing: every rank runs on cuda:0 with a gloo process group (needs --comm host or "
                        "host-async) - the N > 1 GPU code path (bucketed collectives, hipGraph capture, "
                        "consistency checks) on a one-GPU box; timings are not xGMI's")
    g.add_argument("--rccl-channels", default=0, type=int,
                   help="RCCL channels (CTAs) of the framework's gradient communicator, set per "
                        "communicator through ncclConfig_t minCTAs/maxCTAs (0 = RCCL's topology default; "
                        ">= 7 spans all xGMI links of an MI355X)")
    g.add_argument("--ddp-debug", action="store_true",
                   help="debug: reducer assertions (double ready-mark, a gradient arriving after its "
                        "bucket was already all-reduced) and a "
                        "cross-rank collective-sequence check at every consistency check")
    g.add_argument("--amp-val", action="store_true",
                   help="run validation under autocast too (the reference validates in fp32)")
    g.add_argument("--ref-throughput", action="store_true",
                   help="native impl: time each step from after the loader yields to after a host sync "
                        "(the reference's step-line definition, train_ddp.py:196,224) instead of the "
                        "default sync-to-sync window, which has no per-step host sync")
    g.add_argument("--fault-inject", default=None, type=str, metavar="rank=R,step=S|rank=R,epoch=E",
                   help="testing: rank R exits abruptly with status 17 before global optimizer step S (every "
                        "run), or at the start of 0-based epoch E (once per output dir: a marker file there "
                        "lets a restarted job run through)")
    g.add_argument("--cuda-graph", dest="cuda_graph", action="store_true", default=None,
                   help="capture the training step in a hipGraph (static shapes, native impl); "
                        "default: on when the step is launch-bound (per-GPU batch x pixels <= 2^18, "
                        "e.g. the reference's ResNet-18 / CIFAR), off otherwise")
    g.add_argument("--no-cuda-graph", dest="cuda_graph", action="store_false",
                   help="never replay the step as a hipGraph")
    return p


def parse_args(argv: Optional[Sequence[str]] = None) -> argparse.Namespace:
    args = build_parser().parse_args(argv)
    return finalize(args)


def finalize(args: argparse.Namespace) -> argparse.Namespace:
    """Fill the data-dependent defaults."""
    if args.channels_last is None:
        import torch

        args.channels_last = args.impl == "native" and torch.cuda.is_available()
    if args.image_size is None:
        args.image_size = 32 if args.dataset == "cifar10" else 224
    if args.num_classes is None:
        args.num_classes = 10 if args.dataset == "cifar10" else 1000
    if args.backend == "nccl":
        args.backend = "rccl"
    b = [float(v) for v in str(args.betas).split(",")]
    if len(b) != 2:
        raise ValueError("--betas expects two comma-separated floats")
    args.betas = tuple(b)
    if args.grad_accum < 1:
        raise ValueError("--grad-accum must be >= 1")
    from .utils.fault import FaultSpec
    FaultSpec.parse(args.fault_inject)   # reject a malformed spec at start-up, not mid-run
    return args
