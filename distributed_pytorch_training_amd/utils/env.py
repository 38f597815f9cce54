"""Runtime environment for MI355X runs.

MIOpen's find step (triggered by ``cudnn.benchmark = True``, reference train_ddp.py:329)
costs minutes per new convolution configuration on a fresh box (measured: 2-4 min for
ResNet-50 at one batch size).  Its results are a small text database keyed by problem
shape and device; this repo carries the databases tuned on MI355X under ``miopen_db/``
and points ``MIOPEN_USER_DB_PATH`` at a writable copy, so a fresh box starts with the
tuned kernels and the timed window never includes find-mode tuning.
"""
from __future__ import annotations

import os
import shutil
from pathlib import Path

REPO = Path(__file__).resolve().parents[2]
SHIPPED_DB = REPO / "miopen_db"
SHIPPED_GEMM_DB = REPO / "gemm_db" / "tunableop_results.csv"

# MIOpen solvers whose kernels compute wrong results under hipGraph replay.  Measured on MIOpen
# 3.5 / ROCm 7.2 (profiles/graph_replay_miopen_r4.md): the CK grouped backward-weights solver
# (ConvHipImplicitGemmGroupWrwXdlops) and the CK grouped backward-data solver (...GroupBwdXdlops)
# return gradients wrong by up to 1e36 relative on replays of a captured conv backward, while
# eager calls of the same solvers are correct (the CK grouped forward solver is replay-safe).
# Find mode picks them on timing (they win some shapes by ~15%), so which boxes hit them varies
# from run to run.  Only the backward-weights one honours a switch: neither
# MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_HIP_GROUP_BWD_XDLOPS nor MIOPEN_DEBUG_GROUP_CONV_IMPLICIT_GEMM_HIP_BWD_XDLOPS
# keeps the backward-data solver out of find (measured).  Against that one: the shipped find-db
# pins the replay-safe ASM solver for the default fp32 ResNet-18 shapes, and engine/graph.py
# validates the first replay and falls back to eager.  MIOpen reads these switches once, at the
# first convolution of the process: graph_safe_miopen() must run before any MIOpen call.
#
# The second switch is about determinism, not replay safety (round 5, profiles/replay_noise_r5.md):
# the ASM implicit-GEMM forward solver for NHWC (ConvAsmImplicitGemmGTCDynamicFwdXdlopsNHWC, find's
# choice for 7 of the 12 fp32 ResNet-18 convolutions) reduces over K with atomics, so two forwards
# of the same input differ by ~1e-6.  That flips the ReLU mask of activations within 1e-6 of zero,
# which moves a BatchNorm parameter's gradient by O(1/batch): eager-vs-eager (and replay-vs-eager)
# differed by 3e-3 of the whole gradient on some steps (the round-4 driver failure of
# tests/test_graph_replay_gpu.py).  Without it find picks the CK grouped forward solver (replay-
# safe, deterministic: bench/determinism_probe.py, logits bitwise equal run to run), and the
# remaining noise is the rounding of the backward solvers' atomics (~7e-7, no discrete step after
# it).  Excluding the ASM backward-weights solver as well would leave only the naive one.
GRAPH_MIOPEN_EXCLUDE = {
    "MIOPEN_DEBUG_GROUP_CONV_IMPLICIT_GEMM_HIP_WRW_XDLOPS": "CK grouped backward-weights: wrong under replay",
    "MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_FWD_GTC_XDLOPS_NHWC": "ASM NHWC forward: non-deterministic (atomics)",
}
GRAPH_UNSAFE_MIOPEN_SOLVERS = tuple(GRAPH_MIOPEN_EXCLUDE)


def graph_safe_miopen() -> bool:
    """Exclude the graph-unsafe and the non-deterministic-forward MIOpen solvers
    (``GRAPH_MIOPEN_EXCLUDE``; unless the user set the switches explicitly).  True when all of
    them are excluded.  Processes that may capture a hipGraph call this before their first
    convolution (its first replay is validated against eager steps, which needs a reproducible
    step); eager-only processes keep the full solver set."""
    for k in GRAPH_UNSAFE_MIOPEN_SOLVERS:
        os.environ.setdefault(k, "0")
    return all(os.environ.get(k) == "0" for k in GRAPH_UNSAFE_MIOPEN_SOLVERS)


def setup_miopen_env(scratch: str | None = None) -> str:
    """Point MIOpen's user find-db / kernel cache at writable dirs seeded from the repo."""
    if "MIOPEN_USER_DB_PATH" in os.environ:
        return os.environ["MIOPEN_USER_DB_PATH"]
    # one directory per local rank: N ranks starting together never read a database another
    # rank is still copying, and never contend for MIOpen's sqlite kernel-cache lock
    lr = os.environ.get("LOCAL_RANK", "0")
    base = Path(scratch or os.environ.get("DPT_SCRATCH", "/tmp")) / f"dpt_miopen_{os.getuid()}_r{lr}"
    db = base / "db"
    cache = base / "cache"
    db.mkdir(parents=True, exist_ok=True)
    cache.mkdir(parents=True, exist_ok=True)
    if SHIPPED_DB.is_dir():
        for f in SHIPPED_DB.iterdir():
            if not f.is_file():
                continue
            # find/perf databases (text) seed the user db; the compiled-kernel cache (.ukdb)
            # seeds the kernel cache so a fresh box does not recompile MIOpen's kernels.
            dst = (cache if f.suffix == ".ukdb" else db) / f.name
            if not dst.exists():
                tmp = dst.with_name(f"{dst.name}.{os.getpid()}.tmp")
                shutil.copy2(f, tmp)
                os.replace(tmp, dst)       # atomic: readers see all or nothing
    os.environ["MIOPEN_USER_DB_PATH"] = str(db)
    os.environ.setdefault("MIOPEN_CUSTOM_CACHE_DIR", str(cache))
    return str(db)


def export_miopen_db(dest: str | None = None) -> int:
    """Copy the (text) find/perf databases MIOpen wrote back into ``miopen_db/``."""
    src = Path(os.environ.get("MIOPEN_USER_DB_PATH", ""))
    if not src.is_dir():
        return 0
    out = Path(dest) if dest else SHIPPED_DB
    out.mkdir(parents=True, exist_ok=True)
    n = 0
    for f in src.iterdir():
        if f.is_file() and f.name.endswith(".txt"):
            shutil.copy2(f, out / f.name)
            n += 1
    cache = Path(os.environ.get("MIOPEN_CUSTOM_CACHE_DIR", ""))
    if cache.is_dir():
        for f in cache.glob("*.ukdb"):
            shutil.copy2(f, out / f.name)
            n += 1
    return n


def setup_tunableop() -> bool:
    """Use the shipped MI355X GEMM tunings (PyTorch TunableOp over hipBLASLt/rocBLAS).

    hipBLASLt's default heuristic picks non-split-K kernels for the long-K weight-gradient
    GEMMs of ViT ([3072 x 768] outputs with K = tokens = 25,216): 36 workgroups on a 256-CU
    chip.  ``gemm_db/tunableop_results.csv`` holds the measured-fastest solution per GEMM
    shape (tuned on MI355X by ``bench/gpu_tune_gemm.sh``); TunableOp looks shapes up there and
    falls back to the default heuristic for unknown ones.  Read-only: tuning stays off unless
    the caller set ``PYTORCH_TUNABLEOP_*`` itself.  ``DPT_TUNABLEOP=0`` disables.
    """
    if os.environ.get("DPT_TUNABLEOP", "1") == "0" or "PYTORCH_TUNABLEOP_ENABLED" in os.environ:
        return False
    if not SHIPPED_GEMM_DB.is_file():
        return False
    import torch

    if not torch.cuda.is_available():
        return False
    t = torch.cuda.tunable
    t.enable(True)
    t.tuning_enable(False)
    t.record_untuned_enable(False)
    t.set_filename(str(SHIPPED_GEMM_DB), False)
    return True
