"""Headline benchmark: ResNet-50 bf16 AMP data-parallel training throughput (images/s, whole job).

    python bench.py [--gpus N --steps K --warmup W]       # N ranks, launched by this script
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W

Run directly with ``--gpus N > 1`` (no launcher environment), the script is its own launcher:
the parent process spawns N rank processes (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=
127.0.0.1 / a free MASTER_PORT - the env:// contract of reference train_ddp.py:50,61-65)
before anything touches the GPU, waits for them and exits with the worst rank's status.  It
fails (non-zero) instead of running fewer ranks: fewer than N visible GPUs, a dead rank, or
a launcher WORLD_SIZE that differs from ``--gpus`` are errors.  The JSON line records the
rank count the framework communicator was created with (``comm.world_size``), each rank's
device (``comm.rank_devices``), the launcher and every DPT_/NCCL_/RCCL_/MIOPEN_/HIP_ variable
in effect (``config.env``), so a record can be reproduced from itself.

Metric/config from BASELINE.json: "images/sec (whole node) ResNet-50 bf16 at 1/2/4/8
MI355X; % step in all-reduce".  Synthetic ImageNet-shape data (3x224x224, 1000 classes),
random-init weights, the full training step inside the timed window: forward (bf16
autocast, channels_last), loss, loss scaling, backward with the bucketed RCCL all-reduce,
fused SGD (lr 0.1, momentum 0.9, wd 5e-4) with the device-resident scaler, device metrics.
W untimed warmup steps, then EXACTLY K steps bracketed by barrier + device synchronize on
both sides; the MAX step time over ranks is reported.  Per-GPU batch is fixed as N grows
(weak scaling).  The reference publishes no numbers, so the baseline is stock PyTorch-ROCm
running the reference's mechanics (torch DDP, foreach SGD, torch.amp.GradScaler: ``--impl
torch``) on the SAME box: after the native run, a fresh child job measures it with the same
model, batch, dtype and steps (``--stock-baseline``), and ``vs_baseline`` = value / that number.
The round-1 constant from another box stays in the record as
``baseline.stock_reference_constant`` and is the divisor only when the child job fails.
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import signal
import socket
import subprocess
import sys
import time

import torch
import torch.distributed as dist

# Stock PyTorch-ROCm (torch DDP defaults, foreach SGD, torch.amp.GradScaler, bf16 autocast,
# channels_last) on one MI355X, ResNet-50, 224px: images/s per GPU at the per-GPU batch.
STOCK_TORCH_1GPU = {128: 5736.1, 256: 6381.7}


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch-size", type=int, default=256, help="per-GPU batch")
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--num-classes", type=int, default=1000)
    ap.add_argument("--impl", default="native", choices=["native", "torch"])
    ap.add_argument("--amp-dtype", default="bf16", choices=["bf16", "fp16"])
    ap.add_argument("--no-amp", action="store_true", help="fp32 (AMP-vs-FP32 table)")
    ap.add_argument("--no-channels-last", action="store_true")
    ap.add_argument("--optimizer", default="sgd", choices=["sgd", "adam", "adamw"])
    ap.add_argument("--bucket-cap-mb", type=float, default=25.0)
    ap.add_argument("--first-bucket-mb", type=float, default=1.0)
    ap.add_argument("--last-bucket-mb", type=float, default=1.0,
                    help="cap of the bucket that becomes ready last (0 = torch DDP's plan)")
    ap.add_argument("--grad-dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--no-fused-bn", action="store_true", help="A/B: MIOpen BN + separate ReLU/add")
    ap.add_argument("--find", action="store_true",
                    help="cudnn.benchmark=True: run MIOpen find (minutes on a fresh box). Default is "
                         "immediate mode, which reads the find-db shipped in miopen_db/ (tuned on MI355X "
                         "for this config) and skips the search")
    ap.add_argument("--cuda-graph", action="store_true", help="replay the captured step as a hipGraph")
    ap.add_argument("--no-native-conv", action="store_true", help="A/B: MIOpen convolutions")
    ap.add_argument("--native-conv-fp32", action="store_true",
                    help="with --no-amp: the fp32 MFMA conv kernels instead of MIOpen's fp32 solvers")
    ap.add_argument("--conv-streamk", choices=("off", "auto", "all"), default=None,
                    help="stream-K grids for unevenly spread MFMA conv tile grids (default: the "
                         "framework's, env DPT_CONV_STREAMK)")
    ap.add_argument("--no-weight-shadow", action="store_true",
                    help="A/B: autocast casts fp32 weights every forward (no optimizer-kept bf16 copy)")
    ap.add_argument("--profile-steps", type=int, default=8,
                    help="a SECOND timed window of this many steps, after the headline window, with "
                         "per-bucket hipEvents on the comm stream (one event slot per step, read after "
                         "the window: no host sync inside it) -> BASELINE's second metric, %% of step "
                         "in all-reduce, plus exposed comm; 0 = off")
    ap.add_argument("--comm", default="rccl", choices=["rccl", "c10d", "host", "host-async"],
                    help="native reducer collective (host / host-async = gloo staging, debug only)")
    ap.add_argument("--rccl-channels", type=int, default=0,
                    help="NCCL_MIN/MAX_NCHANNELS for the framework's RCCL communicator (0 = RCCL default)")
    ap.add_argument("--rehearse-shared-gpu", action="store_true",
                    help="testing: the ranks share cuda:0 over a gloo process group and the asynchronous "
                         "host-bridge collective (--comm host-async: enqueued like RCCL, so backward "
                         "overlaps it) - the N > 1 path of this script on a 1-GPU box (RCCL itself is not "
                         "exercised; timings are gloo's, not xGMI's)")
    ap.add_argument("--fake-pg", action="store_true",
                    help="testing: run as rank 0 of a --gpus-rank job on torch's fake process group (CPU)")
    ap.add_argument("--fail-rank", type=int, default=-1,
                    help="testing: this rank exits with status 17 right after the process group is up")
    ap.add_argument("--allow-comm-fallback", action="store_true",
                    help="N > 1: publish a record even when the framework RCCL communicator could not be "
                         "created and the reducer fell back to torch's c10d communicator (default: exit 4 "
                         "without measuring - a headline must come from the framework's RCCL reducer)")
    ap.add_argument("--stock-baseline", default="auto", choices=["auto", "on", "off"],
                    help="after the native run, measure stock PyTorch-ROCm (--impl torch: torch DDP, foreach "
                         "SGD, torch.amp.GradScaler) with the same model/batch/dtype/steps in a FRESH child "
                         "job on the same GPUs; vs_baseline is then value / that number (auto: on for the "
                         "native engine on GPUs)")
    ap.add_argument("--stock-timeout", type=float, default=420.0,
                    help="seconds the stock child job may take before it is killed (then no same-box number)")
    ap.add_argument("--extra-windows", default="auto", choices=["auto", "on", "off"],
                    help="after the headline (and the stock job), fresh child jobs on the same GPUs for "
                         "BASELINE.json configs 4 and 5: at 1 GPU the ViT-B/16 bf16 AdamW step and the fp32 "
                         "ResNet-50 step, at 4 GPUs the fp32 ResNet-50 run (AMP vs FP32 with the sync "
                         "profile), at 8 GPUs ViT-B/16 at several bucket caps; recorded under extra_windows, "
                         "never part of the headline (auto: on for the native ResNet-50 bf16 engine on 1, 4 "
                         "or 8 GPUs)")
    ap.add_argument("--extra-timeout", type=float, default=240.0,
                    help="seconds each extra-window child job may take")
    ap.add_argument("--extra-steps", type=int, default=10,
                    help="timed steps of each extra-window job (3 warm-up steps, a 6-step sync-profile window)")
    ap.add_argument("--extra-budget", type=float, default=300.0,
                    help="seconds all extra-window child jobs together may take (later windows are "
                         "skipped and recorded as such once it is spent)")
    ap.add_argument("--deadline", type=float, default=480.0,
                    help="seconds from the start of the job by which rank 0 has printed the record: the "
                         "same-box stock job and the extra windows only get the time that is left (each "
                         "child job runs in its own process group and is killed whole at its limit), so a "
                         "hung child can never cost the headline line")
    ap.add_argument("--vit-buckets", default="25,400,100",
                    help="bucket caps (MB) of the 8-GPU ViT-B/16 extra windows")
    ap.add_argument("--extra-rccl-channels", default="8,16",
                    help="per-communicator RCCL channel bounds of the 8-GPU ResNet-50 extra windows (how many "
                         "CUs RCCL's kernels take from the overlapped backward; the headline uses RCCL's choice)")
    ap.add_argument("--json-out", default=None)
    return ap.parse_args(argv)


ENV_PREFIXES = ("DPT_", "NCCL_", "RCCL_", "MIOPEN_", "HIP_", "HSA_", "AMD_", "GPU_MAX_HW_QUEUES",
                "PYTORCH_TUNABLEOP", "TORCH_NCCL", "OMP_NUM_THREADS")
CHILD_MARK = "DPT_BENCH_LAUNCHER"
DEADLINE_MARK = "DPT_BENCH_DEADLINE_AT"   # absolute epoch deadline, handed from a launcher to its ranks
RECORD_MARK = "DPT_BENCH_RECORD_FILE"     # a file rank 0 creates once its record is written (launcher)
CHILD_JOB_MARK = "DPT_BENCH_CHILD_JOB"     # set in the stock / extra-window child jobs


def _process_start() -> float:
    """Creation time of this process (the --deadline clock starts before the torch import)."""
    try:
        import psutil
        return float(psutil.Process().create_time())
    except Exception:
        return time.time()


T_START = _process_start()
rccl_log = None  # distributed_pytorch_training_amd.utils.rccl_log, imported by the ranks only


def env_in_effect() -> dict:
    return {k: v for k, v in sorted(os.environ.items())
            if k.startswith(ENV_PREFIXES) and k not in (CHILD_MARK, DEADLINE_MARK, CHILD_JOB_MARK, RECORD_MARK)}


def _sig(v: float, digits: int = 6) -> float:
    """Round to significant figures (a fixed number of decimals loses all precision on a slow
    CPU run: 0.107 img/s -> 0.11)."""
    return float(f"{v:.{digits}g}")


def deadline_at(a) -> float:
    """Absolute deadline of this job: a launcher's (inherited by its ranks) or start + --deadline."""
    v = os.environ.get(DEADLINE_MARK)
    return float(v) if v else T_START + a.deadline


def _kill_group(p: subprocess.Popen, grace: float = 5.0) -> None:
    """SIGTERM the whole process group of ``p`` (a child job started with start_new_session: its
    self-launched ranks are in that group too), then SIGKILL whatever is left after ``grace``."""
    pgid = p.pid          # start_new_session: the child leads its own process group
    for sig in (signal.SIGTERM, signal.SIGKILL):
        try:
            os.killpg(pgid, sig)
        except OSError:
            break         # nothing left in the group
        t_end = time.time() + grace
        while time.time() < t_end:
            p.poll()      # reap the leader (a zombie still counts as a group member)
            try:
                os.killpg(pgid, 0)
            except OSError:
                return
            time.sleep(0.1)
    p.poll()


_LIVE_CHILDREN = []   # child-job Popen objects of this process, for the signal handler


def run_group(cmd: list, env: dict, timeout: float):
    """Run ``cmd`` as a child job in its own session / process group; on timeout kill the whole
    group (its ranks included) and raise ``subprocess.TimeoutExpired``.  Returns (rc, stderr)."""
    import tempfile
    with tempfile.TemporaryFile(mode="w+") as err:
        p = subprocess.Popen(cmd, env=env, stdout=subprocess.DEVNULL, stderr=err, text=True,
                             start_new_session=True)
        _LIVE_CHILDREN.append(p)
        try:
            try:
                rc = p.wait(timeout=max(1.0, timeout))
            except subprocess.TimeoutExpired:
                _kill_group(p)
                raise
            # the launcher exited; anything left in its group is an orphaned rank: end it
            try:
                os.killpg(p.pid, 0)
                _kill_group(p)
            except OSError:
                pass
        finally:
            _LIVE_CHILDREN.remove(p)
        err.seek(0)
        return rc, err.read()


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _visible_gpus() -> int:
    """GPU count WITHOUT touching the GPU runtime in this (launcher) process.

    A launcher must not initialise HIP before it starts its ranks, and ``torch.cuda.device_count()``
    can fall back to a HIP call (``_cuda_getDeviceCount``) when amdsmi discovery fails.  So a
    throwaway child process counts (whatever HIP state it creates dies with it; it sees the same
    device cgroup and visibility variables the ranks will).  If the child cannot run, the KFD
    topology in sysfs (GPU nodes have a non-zero ``gpu_id``) bounded by a ``ROCR_/HIP_/
    CUDA_VISIBLE_DEVICES`` list is the fallback."""
    try:
        r = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                           capture_output=True, text=True, timeout=180)
        if r.returncode == 0 and r.stdout.strip():
            return int(r.stdout.strip().splitlines()[-1])
    except (subprocess.SubprocessError, ValueError, OSError):
        pass
    n = _kfd_gpu_count() or 0
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([t for t in v.split(",") if t.strip() != ""]))
    return n


def _kfd_gpu_count(root: str = "/sys/class/kfd/kfd/topology/nodes"):
    """GPU nodes in the KFD topology, or None when it cannot be read."""
    try:
        names = os.listdir(root)
    except OSError:
        return None
    n = 0
    for d in names:
        try:
            with open(os.path.join(root, d, "gpu_id")) as f:
                n += int(f.read().strip() or 0) != 0
        except (OSError, ValueError):
            continue
    return n


def launch_ranks(a, argv, grace_s: float = 30.0) -> int:
    """Spawn ``--gpus`` rank processes of this script (self-launch, no torchrun needed).

    Nothing here touches the GPU: the children are fresh interpreters.  Returns the worst
    child exit status; when one rank fails, the survivors get ``grace_s`` to finish (they
    normally error out of their collective) and are then terminated, so a dead peer can not
    leave the node hanging.  The ranks stay in this process's group (a ``killpg`` of the job
    reaches them) and inherit the job's absolute deadline; a SIGTERM to this launcher is passed on
    to them, and once rank 0 has written its record, ranks still alive 60 s past the deadline (a
    teardown that hangs: 60 s after the record and past the deadline) are ended - a headline window
    still being measured is never cut."""
    import tempfile
    n = a.gpus
    t_dead = deadline_at(a)
    fd, mark = tempfile.mkstemp(prefix="dpt_bench_record_")
    os.close(fd)
    os.remove(mark)
    ngpu = _visible_gpus()
    if a.rehearse_shared_gpu:
        if ngpu < 1:
            print("error: --rehearse-shared-gpu needs one visible GPU", file=sys.stderr)
            return 2
    elif ngpu == 0:
        print(f"bench: no GPU visible - {n} gloo ranks on the CPU", file=sys.stderr)
    elif ngpu < n:
        print(f"error: --gpus {n} but only {ngpu} GPU(s) are visible; refusing to run fewer ranks",
              file=sys.stderr)
        return 2
    port = _free_port()
    script = os.path.abspath(__file__)
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", ROLE_RANK=str(r), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env[CHILD_MARK] = "self"
        env[DEADLINE_MARK] = repr(t_dead)
        env[RECORD_MARK] = mark
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, script, *argv], env=env))
    rcs = [None] * n

    def _forward(signum, _frame):
        for p in procs:
            if p.poll() is None:
                p.send_signal(signum)
        t_end = time.time() + 10
        for p in procs:
            try:
                p.wait(timeout=max(0.1, t_end - time.time()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        os._exit(128 + signum)

    old = {s: signal.signal(s, _forward) for s in (signal.SIGTERM,)}
    failed_at = None
    try:
        while any(rc is None for rc in rcs):
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    rcs[i] = p.poll()
                    if rcs[i] not in (None, 0) and failed_at is None:
                        failed_at = time.time()
                        print(f"bench: rank {i} exited with status {rcs[i]}", file=sys.stderr)
            if failed_at is None and time.time() > t_dead + 60 and os.path.exists(mark) and \
                    time.time() > os.path.getmtime(mark) + 60:
                failed_at = time.time() - grace_s - 1   # end them now
                print("bench: ranks still running 60 s after the record, past the deadline; terminating them",
                      file=sys.stderr)
            if failed_at is not None and time.time() - failed_at > grace_s:
                for i, p in enumerate(procs):
                    if rcs[i] is None:
                        p.terminate()
                deadline = time.time() + 10
                for i, p in enumerate(procs):
                    if rcs[i] is None:
                        try:
                            rcs[i] = p.wait(timeout=max(0.1, deadline - time.time()))
                        except subprocess.TimeoutExpired:
                            p.kill()
                            rcs[i] = p.wait()
                break
            time.sleep(0.1)
    except KeyboardInterrupt:
        for p in procs:
            if p.poll() is None:
                p.send_signal(signal.SIGINT)
        for p in procs:
            p.wait()
        return 130
    finally:
        for s, h in old.items():
            signal.signal(s, h)
        try:
            os.remove(mark)
        except OSError:
            pass
    rcs = [124 if rc is None else rc for rc in rcs]
    bad = [rc for rc in rcs if rc != 0]
    if not bad:
        return 0
    rc = bad[0]
    return 128 - rc if rc < 0 else rc


def _red_dev(device):
    """Where to all-reduce a host-read scalar: gloo reduces host tensors (its device path is
    not used here), RCCL device tensors."""
    return "cpu" if dist.is_initialized() and dist.get_backend() == "gloo" else device


def _rccl_log_prefix() -> str:
    import tempfile
    return os.path.join(tempfile.gettempdir(), f"dpt_bench_rccl_{os.environ.get('MASTER_PORT', '0')}_"
                                               f"r{os.environ.get('RANK', '0')}")


def verify_job(trainer, device, ws: int, rank: int, ms_per_step: float) -> dict:
    """Self-verification of an N > 1 record: after the timed window
    * parameters bit-identical on every rank (``Trainer.check_consistency``: fp64 checksum
      MIN == MAX across ranks);
    * one all-reduce of ``rank + 1``-filled data through the framework communicator (the
      device collective the gradients used; the process group where there is none) equals
      ``N (N + 1) / 2`` exactly;
    * every rank's own ms/step (the headline is the max);
    * the channel count RCCL actually opened for the framework communicator (its init log).
    ``ok`` is the AND over ranks of the checks; ``main`` exits non-zero when it is false."""
    if dist.get_backend() == "fake":      # every collective is a no-op: nothing to verify
        return {"skipped": "fake process group", "ok": None, "selftest_ok": None,
                "rccl_channels_opened": None}
    out = {}
    try:
        trainer.check_consistency()
        params_ok = True
    except RuntimeError as e:
        params_ok = False
        out["consistency_error"] = str(e)[:300]
    comm = trainer.ddp.comm if trainer.ddp is not None else None
    if comm is not None:
        t = torch.full((4096,), float(rank + 1), dtype=torch.float32, device=device)
        comm.all_reduce(t, True)
        torch.cuda.synchronize(device)
        comm.check()
        via = comm.kind
    else:
        t = torch.full((4096,), float(rank + 1), dtype=torch.float32, device=_red_dev(device))
        dist.all_reduce(t)
        via = "process-group:" + dist.get_backend()
    want = ws * (ws + 1) / 2
    self_ok = bool((t == want).all().item())
    flag = torch.tensor([int(params_ok and self_ok)], dtype=torch.int32, device=_red_dev(device))
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    per_rank = [None] * ws
    dist.all_gather_object(per_rank, round(ms_per_step, 3))
    opened = None
    if comm is not None and hasattr(comm, "handle") and os.environ.get("NCCL_DEBUG_FILE", "").startswith(
            _rccl_log_prefix()):
        opened = rccl_log.opened_channels(int(comm.handle), _rccl_log_prefix())
    gathered = [None] * ws
    dist.all_gather_object(gathered, opened)
    out.update({"ok": bool(flag.item()), "params_consistent": params_ok, "selftest_ok": self_ok,
                "selftest_via": via, "selftest_expected": want, "per_rank_ms_per_step": per_rank,
                "rccl_channels_opened": gathered})
    return out


def _rccl_version():
    try:
        from distributed_pytorch_training_amd import ops
        return ops.native().rccl_version() if ops.native_available() else None
    except Exception:
        return None


def _rank_devices(device, ws):
    """Every rank's device (index and PCI bus id): proves N distinct GPUs took part."""
    mine = {"device": str(device)}
    if device.type == "cuda":
        p = torch.cuda.get_device_properties(device)
        mine["pci_bus_id"] = getattr(p, "pci_bus_id", None)
        mine["name"] = p.name
    if ws > 1 and dist.is_initialized() and dist.get_backend() != "fake":
        out = [None] * ws
        dist.all_gather_object(out, mine)
        return out
    return [mine]


def _stock_argv(a, _unused=None) -> list:
    """The same benchmark on the stock engine: same model, per-GPU batch, dtype, layout, steps."""
    argv = ["--gpus", str(a.gpus), "--impl", "torch", "--steps", str(a.steps), "--warmup", str(a.warmup),
            "--model", a.model, "--batch-size", str(a.batch_size), "--image-size", str(a.image_size),
            "--num-classes", str(a.num_classes), "--amp-dtype", a.amp_dtype, "--optimizer", a.optimizer,
            "--bucket-cap-mb", str(a.bucket_cap_mb), "--profile-steps", "0", "--stock-baseline", "off",
            "--extra-windows", "off"]
    for flag in ("no_amp", "no_channels_last", "find"):
        if getattr(a, flag):
            argv.append("--" + flag.replace("_", "-"))
    return argv


def _child_env() -> dict:
    """This job's environment minus its launcher variables (a child picks its own rendezvous and
    self-launches its ranks), marked as a child job."""
    drop = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK", "MASTER_ADDR",
            "MASTER_PORT", "GROUP_WORLD_SIZE", "ROLE_WORLD_SIZE", CHILD_MARK, DEADLINE_MARK, RECORD_MARK, "NCCL_DEBUG",
            "NCCL_DEBUG_FILE", "NCCL_DEBUG_SUBSYS")
    env = {k: v for k, v in os.environ.items() if k not in drop and not k.startswith("TORCHELASTIC_")}
    env[CHILD_JOB_MARK] = "1"
    return env


def _run_child(argv: list, timeout: float) -> dict:
    """A fresh child ``bench.py`` job (new interpreter in its own process group, launcher
    variables stripped); returns its JSON record or the reason there is none.  At ``timeout``
    the whole group - the child's ranks included - is killed."""
    import tempfile
    fd, out = tempfile.mkstemp(prefix="dpt_child_", suffix=".json")
    os.close(fd)
    # the child's own deadline: its record must be written before this job gives up on it
    cmd = [sys.executable, os.path.abspath(__file__), *argv, "--json-out", out,
           "--deadline", f"{max(10.0, timeout - 5):.0f}"]
    t0 = time.time()
    try:
        rc, err = run_group(cmd, _child_env(), timeout)
        with open(out) as f:
            lines = [json.loads(l) for l in f if l.startswith("{")]
        if rc != 0 or not lines:
            return {"error": f"child job exited {rc}: {err[-400:]}", "wall_s": round(time.time() - t0, 1)}
        rec = lines[-1]
        rec["wall_s"] = round(time.time() - t0, 1)
        return rec
    except subprocess.TimeoutExpired:
        return {"error": f"child job exceeded {timeout:.0f} s (process group killed)",
                "wall_s": round(time.time() - t0, 1)}
    except (OSError, ValueError) as e:
        return {"error": repr(e)[:400]}
    finally:
        try:
            os.remove(out)
        except OSError:
            pass


def _window(rec: dict, argv: list) -> dict:
    """The fields of a child record that the extra windows keep."""
    if "error" in rec:
        return {"error": rec["error"], "cmd": "bench.py " + " ".join(argv)}
    cfg = rec.get("config", {})
    return {"value": rec.get("value"), "unit": rec.get("unit"), "ms_per_step": rec.get("ms_per_step"),
            "n_gpus": rec.get("n_gpus"), "steps": rec.get("steps"), "dtype": rec.get("dtype"),
            "model": cfg.get("model"), "impl": cfg.get("impl"), "per_gpu_batch": cfg.get("per_gpu_batch"),
            "bucket_cap_mb": cfg.get("bucket_cap_mb"), "optimizer": cfg.get("optimizer"),
            "pct_step_allreduce": rec.get("pct_step_allreduce"),
            "pct_step_exposed_comm": rec.get("pct_step_exposed_comm"),
            "sync_profile_window": rec.get("sync_profile_window"),
            "comm_kind": rec.get("comm", {}).get("kind"), "buckets_mib": rec.get("comm", {}).get("buckets_mib"),
            "wall_s": rec.get("wall_s"), "cmd": "bench.py " + " ".join(argv)}


def extra_windows_plan(a, ws: int, forced: bool = False) -> list:
    """(name, argv) of the extra windows for a ``ws``-GPU headline job (BASELINE.json configs 4/5);
    ``forced`` (--extra-windows on) adds the fp32 window at any world size."""
    common = ["--gpus", str(ws), "--stock-baseline", "off", "--extra-windows", "off", "--comm", a.comm,
              "--bucket-cap-mb", str(a.bucket_cap_mb)]
    steps = ["--steps", str(a.extra_steps), "--warmup", "3", "--profile-steps", "6"]
    r50_shape = ["--model", a.model, "--batch-size", str(a.batch_size), "--image-size", str(a.image_size)]
    plan = []
    vit1 = ("vit_b16_bucket25mb", common[:-1] + ["25", "--model", "vit_b_16", "--batch-size", "128",
                                                 "--optimizer", "adamw"] + steps)
    if ws == 1 and not a.no_amp and a.model == "resnet50" and a.image_size == 224:
        # one GPU, headline config: the ViT-B/16 step (BASELINE.json config 5's model, native and
        # stock engines) beside the fp32 ResNet-50 step (config 4's AMP-vs-FP32 pair)
        plan.append(vit1)
        plan.append(("vit_b16_stock", vit1[1] + ["--impl", "torch"]))
    if (ws in (1, 4) or forced) and not a.no_amp:
        plan.append(("resnet50_fp32", common + r50_shape + ["--no-amp"] + steps))
    if ws == 8:
        vit = [(f"vit_b16_bucket{float(cap):g}mb",
                common + ["--model", "vit_b_16", "--batch-size", "128", "--optimizer", "adamw",
                          "--bucket-cap-mb", cap.strip()] + steps)
               for cap in a.vit_buckets.split(",") if cap.strip()]
        r50 = [(f"resnet50_rccl_channels{int(ch)}", common + r50_shape + ["--rccl-channels", ch.strip()] + steps)
               for ch in a.extra_rccl_channels.split(",") if ch.strip()]
        # interleaved, the first two ViT caps first: what the time budget cuts is the least informative
        order = vit[:2] + r50[:1] + vit[2:] + r50[1:]
        plan.extend(order)
    return plan


def run_stock_baseline(a, timeout: float) -> dict:
    """Stock PyTorch-ROCm on the same box ("same MI355X box ... same harness"), in a
    fresh child job started AFTER this job's GPU work is done and its memory released: a new
    interpreter in its own process group (this process keeps running; nothing is exec'd over a
    process that touched the GPU) that self-launches ``--gpus`` ranks of ``--impl torch``.
    Returns its record's numbers or the reason there are none."""
    rec = _run_child(_stock_argv(a, None), timeout)
    if "error" in rec:
        return rec
    try:
        return {"img_s": rec["value"], "ms_per_step": rec["ms_per_step"], "n_gpus": rec["n_gpus"],
                "steps": rec["steps"], "warmup": rec["warmup"], "impl": rec["config"]["impl"],
                "wall_s": rec["wall_s"], "cmd": "bench.py " + " ".join(_stock_argv(a, None))}
    except KeyError as e:
        return {"error": repr(e)[:400]}


def train_args(a):
    from distributed_pytorch_training_amd.config import parse_args

    argv = ["--model", a.model, "--dataset", "synthetic", "--batch-size", str(a.batch_size),
            "--image-size", str(a.image_size), "--num-classes", str(a.num_classes),
            "--impl", a.impl, "--amp-dtype", a.amp_dtype, "--optimizer", a.optimizer,
            "--bucket-cap-mb", str(a.bucket_cap_mb), "--first-bucket-mb", str(a.first_bucket_mb),
            "--last-bucket-mb", str(a.last_bucket_mb),
            "--grad-dtype", a.grad_dtype, "--lr", "0.1", "--momentum", "0.9", "--weight-decay", "5e-4",
            "--comm", a.comm, "--rccl-channels", str(a.rccl_channels)]
    if not a.no_amp:
        argv.append("--amp")
    argv.append("--no-channels-last" if a.no_channels_last else "--channels-last")
    if a.no_fused_bn:
        argv.append("--no-fused-bn")
    # the headline bench keeps hipGraph replay opt-in (the framework default turns it on for
    # launch-bound steps only; the profiled window needs eager steps)
    argv.append("--cuda-graph" if a.cuda_graph else "--no-cuda-graph")
    if a.no_weight_shadow:
        argv.append("--no-weight-shadow")
    if a.no_native_conv:
        argv.append("--no-native-conv")
    if a.native_conv_fp32:
        argv.append("--native-conv-fp32")
    if a.conv_streamk:
        argv += ["--conv-streamk", a.conv_streamk]
    return parse_args(argv)


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    a = parse(argv)
    env_ws = os.environ.get("WORLD_SIZE")
    if a.fake_pg:
        pass
    elif env_ws is None:
        if a.gpus > 1:
            return launch_ranks(a, argv)
    elif int(env_ws) != a.gpus:
        print(f"error: --gpus {a.gpus} but the launcher started WORLD_SIZE={env_ws} ranks", file=sys.stderr)
        return 2
    if os.environ.get(CHILD_JOB_MARK) and os.environ.get("DPT_TEST_HANG_CHILD"):
        while True:         # testing: a child job whose ranks never finish (bench deadline test)
            time.sleep(3600)
    global rccl_log
    from distributed_pytorch_training_amd.utils import rccl_log
    launcher = ("fake" if a.fake_pg else os.environ.get(CHILD_MARK) or
                ("torchrun" if env_ws is not None else "none"))
    from distributed_pytorch_training_amd.data import SyntheticLoader
    from distributed_pytorch_training_amd.engine.trainer import Trainer
    from distributed_pytorch_training_amd.models import build_model
    from distributed_pytorch_training_amd.utils.dist import init_distributed, set_seed
    from distributed_pytorch_training_amd.utils.env import setup_miopen_env, setup_tunableop

    if a.rehearse_shared_gpu and a.comm == "rccl":
        a.comm = "host-async"   # RCCL needs one device per rank
    setup_miopen_env()
    args = train_args(a)
    if a.rehearse_shared_gpu:
        from distributed_pytorch_training_amd.utils.dist import DistInfo
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        dist.init_process_group("gloo", init_method="env://")
        info = DistInfo(dist.get_rank(), dist.get_world_size(), 0, "gloo", dev)
    elif a.fake_pg:
        from torch.testing._internal.distributed.fake_pg import FakeStore

        from distributed_pytorch_training_amd.utils.dist import DistInfo
        dist.init_process_group("fake", store=FakeStore(), rank=0, world_size=a.gpus)
        info = DistInfo(0, a.gpus, 0, "fake", torch.device("cpu"))
    else:
        # a rank may touch the GPU runtime (it is about to use it): count directly
        ngpu = torch.cuda.device_count() if env_ws is not None and int(env_ws) > 1 else 0
        if ngpu > 0 and ngpu < int(os.environ.get("LOCAL_WORLD_SIZE", env_ws)):
            print(f"error: {os.environ.get('LOCAL_WORLD_SIZE', env_ws)} local ranks but only "
                  f"{ngpu} GPU(s) visible", file=sys.stderr)
            return 2
        if (env_ws is not None and int(env_ws) > 1 and a.impl == "native" and a.comm == "rccl"
                and "NCCL_DEBUG" not in os.environ):
            # RCCL's init log, to a file (stdout stays one JSON line): the channel count the
            # framework communicator actually opened is read back from it after the run
            os.environ.update(rccl_log.debug_env(_rccl_log_prefix()))
        info = init_distributed("auto")
    gemm_db = setup_tunableop() if (a.impl == "native" and info.device.type == "cuda") else False
    rank, ws, device = info.rank, info.world_size, info.device
    if ws != a.gpus:
        print(f"error: --gpus {a.gpus} but the process group has {ws} rank(s)", file=sys.stderr)
        return 2
    if a.fail_rank == rank:
        os._exit(17)
    set_seed(0, rank)
    torch.backends.cudnn.benchmark = bool(a.find)

    model = build_model(args.model, args.num_classes, device, image_size=args.image_size,
                        channels_last=args.channels_last)
    trainer = Trainer(model, args, rank, ws, device, log=lambda s: None)
    fallback = getattr(trainer.ddp, "comm_fallback_reason", None) if trainer.ddp is not None else None
    if fallback and not a.allow_comm_fallback:
        # fail closed: every rank took the same branch (parallel/comm.py agreement), so every rank
        # exits here and the job's status is non-zero - no record of the wrong engine
        print(f"bench: rank {rank}: --comm {a.comm} requested but the job fell back to torch's c10d "
              f"communicator: {fallback} (pass --allow-comm-fallback to measure it anyway)", file=sys.stderr)
        trainer.close()
        if ws > 1:
            dist.destroy_process_group()
        return 4
    trainer.model.train()
    loader = SyntheticLoader(a.batch_size * 4, a.batch_size, args.image_size, args.num_classes, device,
                             channels_last=args.channels_last, pool=4, seed=rank)
    batches = list(iter(loader))

    def run(n):
        for i in range(n):
            x, y = batches[i % len(batches)]
            trainer.train_step(x, y)

    def fence():
        if ws > 1:
            dist.barrier()
        torch.cuda.synchronize(device) if device.type == "cuda" else None

    t_w = time.time()
    run(a.warmup)
    fence()
    warm_s = time.time() - t_w
    t0 = time.time()
    run(a.steps)
    fence()
    dt = own_dt = time.time() - t0
    if ws > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=_red_dev(device))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ms = 1e3 * dt / max(a.steps, 1)
    value = a.batch_size * ws * a.steps / dt
    verify = verify_job(trainer, device, ws, rank, 1e3 * own_dt / max(a.steps, 1)) if ws > 1 else None

    prof, prof_window = {}, None
    collective = ws > 1 and a.impl == "native" and trainer.ddp is not None and trainer.ddp.comm is not None
    if a.profile_steps > 0 and collective and device.type == "cuda" and trainer.graphed is None:
        # second timed window, per-bucket comm events on: one event slot per step, everything
        # read after the window (every rank runs the same steps)
        trainer.timeline.enabled = True
        trainer.timeline.max_pending = a.profile_steps + 1
        trainer.ddp.set_profile(True, slots=a.profile_steps + 2)
        run(2)                      # events/slots live; not timed
        fence()
        trainer.timeline.records.clear()
        trainer.timeline._pending.clear()
        t1 = time.time()
        run(a.profile_steps)
        fence()
        pdt = time.time() - t1
        if ws > 1:
            t = torch.tensor([pdt], dtype=torch.float64, device=_red_dev(device))
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            pdt = float(t.item())
        prof = trainer.timeline.summary(skip=0)
        prof_window = {"steps": a.profile_steps, "ms_per_step": round(1e3 * pdt / a.profile_steps, 3),
                       "value": _sig(a.batch_size * ws * a.profile_steps / pdt)}

    const = STOCK_TORCH_1GPU.get(a.batch_size) if (args.model == "resnet50" and args.amp and
                                                   args.amp_dtype == "bf16" and args.image_size == 224) else None
    rec = {
        "metric": "images/sec (whole node) ResNet-50 bf16 training" if args.model == "resnet50"
                  else f"images/sec (whole node) {args.model} training",
        "value": _sig(value), "unit": "images/s", "n_gpus": ws, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(value / (const * ws), 4) if const else None,   # replaced below when the
                                                                            # same-box stock run succeeds
        "dtype": (args.amp_dtype if args.amp else "fp32"), "data": "synthetic",
        "config": {"model": args.model, "global_batch": a.batch_size * ws, "per_gpu_batch": a.batch_size,
                   "seq_len": None, "image_size": args.image_size, "parallelism": f"dp{ws}",
                   "impl": a.impl, "optimizer": a.optimizer, "channels_last": bool(args.channels_last),
                   "bucket_cap_mb": a.bucket_cap_mb, "grad_dtype": a.grad_dtype,
                   "fused_bn": bool(args.fused_bn and a.impl == "native" and args.channels_last
                                     and device.type == "cuda"),
                   "native_conv": bool(args.native_conv and args.fused_bn and a.impl == "native"
                                       and args.channels_last and args.amp and device.type == "cuda"),
                   "miopen": "find" if a.find else "immediate(find-db)",
                   "gemm_db": bool(gemm_db),
                   "weight_shadow": bool(trainer.ddp is not None and trainer.ddp.shadow_flat is not None),
                   "cuda_graph": bool(a.cuda_graph and trainer.graphed is not None
                                      and trainer.graphed.graph is not None)},
        "baseline": {"stock_reference_constant": (round(const * ws, 2) if const else None),
                     "stock_reference_constant_source": "BASELINE.md round-1 stock run x N (another box)",
                     "stock_same_box_img_s": None, "vs_baseline_source": "stock_reference_constant"},
        "warmup_seconds": round(warm_s, 1),
    }
    # BASELINE's second headline number, measured in the second (profiled) window; null when
    # there is no collective (one GPU: the reducer runs local) or it was not measured
    rec["pct_step_allreduce"] = round(prof["pct_step_allreduce"], 2) if "pct_step_allreduce" in prof else None
    rec["pct_step_exposed_comm"] = (round(prof["pct_step_exposed_comm"], 2)
                                    if "pct_step_exposed_comm" in prof else None)
    rec["sync_profile_window"] = prof_window
    if prof:
        rec["sync_profile"] = {k: round(v, 4) if isinstance(v, float) else v for k, v in prof.items()}
    ddp = trainer.ddp
    comm = ddp.comm if ddp is not None else None
    rec["comm"] = {"kind": (comm.kind if comm is not None else
                            ("gloo" if ws > 1 and a.impl == "native" else
                             ("torch-ddp" if ws > 1 else "none"))),
                   # rank count of the framework communicator itself (the process group's when
                   # there is none: gloo / torch DDP)
                   "world_size": int(comm.world_size) if comm is not None else ws,
                   "pg_backend": dist.get_backend() if dist.is_initialized() else None,
                   "rank_devices": _rank_devices(device, ws),
                   "buckets_mib": [round(v, 3) for v in ddp.bucket_sizes_mib()] if ddp is not None else None,
                   "bucket_cap_mb": a.bucket_cap_mb, "first_bucket_mb": a.first_bucket_mb,
                   "last_bucket_mb": a.last_bucket_mb,
                   "grad_dtype": a.grad_dtype,
                   # requested per-communicator bound (None = RCCL's own choice) and what RCCL
                   # opened per rank (its init log; None where it could not be read)
                   "rccl_channels": (int(comm.max_ctas) or None) if comm is not None and hasattr(comm, "max_ctas")
                                    else None,
                   "rccl_channels_opened": verify["rccl_channels_opened"] if verify else None,
                   "selftest_ok": verify["selftest_ok"] if verify else None,
                   "rccl_version": _rccl_version(),
                   "requested": a.comm if a.impl == "native" and ws > 1 else None,
                   "fallback_reason": fallback}
    rec["verify"] = verify
    rec["config"]["launcher"] = launcher
    rec["config"]["env"] = env_in_effect()
    if ws > 1:
        dist.barrier()
    trainer.close()
    stock_on = a.stock_baseline == "on" or (a.stock_baseline == "auto" and a.impl == "native"
                                            and device.type == "cuda" and not a.rehearse_shared_gpu
                                            and not a.fake_pg)
    extra_on = a.extra_windows == "on" or (a.extra_windows == "auto" and a.impl == "native"
                                            and device.type == "cuda" and not a.rehearse_shared_gpu
                                            and not a.fake_pg and a.model == "resnet50" and not a.no_amp
                                            and ws in (1, 4, 8))
    extra_plan = extra_windows_plan(a, ws, forced=a.extra_windows == "on") if extra_on else []
    t_dead = deadline_at(a)
    printed = []
    t_headline = time.time()

    def emit():
        """Print rank 0's ONE JSON line (and append it to --json-out) exactly once."""
        if rank != 0 or printed:
            return
        printed.append(True)
        # wall-clock bookkeeping of the job (epoch seconds): when the headline window was done,
        # the --deadline, and when this record was written
        rec["timing"] = {"process_start": round(T_START, 3), "headline_done": round(t_headline, 3),
                         "deadline": round(t_dead, 3), "record": round(time.time(), 3)}
        line = json.dumps(rec)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "a") as f:
                f.write(line + "\n")
        if os.environ.get(RECORD_MARK):
            try:
                open(os.environ[RECORD_MARK], "w").close()
            except OSError:
                pass

    if stock_on or extra_plan:
        if rank == 0:
            # the headline is measured: whatever happens to the child jobs from here on, a SIGTERM
            # (the driver's time limit) kills their process groups and still prints the record
            def _on_term(signum, _frame):
                for p in list(_LIVE_CHILDREN):
                    _kill_group(p, grace=2.0)
                if stock_on and "stock_same_box" not in rec["baseline"]:
                    rec["baseline"]["stock_same_box"] = {"error": f"not measured: signal {signum} first"}
                emit()
                os._exit(0 if (verify is None or verify["ok"] is not False) else 3)

            signal.signal(signal.SIGTERM, _on_term)
            print("bench: headline measured (provisional record, before the child jobs): "
                  + json.dumps({k: rec[k] for k in ("value", "ms_per_step", "n_gpus", "steps", "warmup")}),
                  file=sys.stderr, flush=True)
        # free this job's GPU memory, then rank 0 runs the child jobs on the same GPUs while the
        # other ranks wait on the TCPStore (host side: no collective kernel spinning on a GPU)
        del trainer, model, batches, loader, ddp, comm
        import gc
        gc.collect()
        if device.type == "cuda":
            torch.cuda.synchronize(device)
            torch.cuda.empty_cache()
        if ws > 1:
            dist.barrier()
        reserve = 15.0      # seconds kept back for printing the record before the deadline

        def left() -> float:
            return t_dead - reserve - time.time()

        def take_stock(stock):
            """Put the stock job's result into the record (as soon as it exists: a SIGTERM later
            still prints it)."""
            rec["baseline"]["stock_same_box"] = stock
            if stock.get("img_s"):
                rec["baseline"]["stock_same_box_img_s"] = stock["img_s"]
                rec["baseline"]["vs_baseline_source"] = "stock_same_box (fresh child job, --impl torch)"
                rec["vs_baseline"] = round(value / stock["img_s"], 4)

        if rank == 0 and stock_on:
            if left() >= 20:
                take_stock(run_stock_baseline(a, min(a.stock_timeout, left())))
            else:
                take_stock({"error": f"skipped: {max(0.0, left() + reserve):.0f} s left before the --deadline"})
        extra = {}
        if rank == 0 and extra_plan:
            rec["extra_windows"] = extra    # filled window by window (a SIGTERM prints what is done)
        if rank == 0:
            t_extra = time.time()
            for name, argv in extra_plan:
                budget = min(a.extra_budget - (time.time() - t_extra), left())
                if budget < 30:
                    why = ("--extra-budget spent" if a.extra_budget - (time.time() - t_extra) < 30
                           else "the --deadline is near")
                    extra[name] = {"error": f"skipped: {why}", "cmd": "bench.py " + " ".join(argv)}
                    continue
                extra[name] = _window(_run_child(argv, min(a.extra_timeout, budget)), argv)
        if ws > 1:
            store = dist.distributed_c10d._get_default_store()
            key = "dpt_bench_stock_done"
            if rank == 0:
                store.set(key, "1")
            else:
                store.wait([key], datetime.timedelta(seconds=max(60.0, t_dead - time.time() + 60)))
    emit()
    if ws > 1:
        dist.barrier()
        dist.destroy_process_group()
    if verify is not None and verify["ok"] is False:
        print(f"bench: rank {rank}: self-verification FAILED: {json.dumps(verify)}", file=sys.stderr)
        return 3
    return 0


if __name__ == "__main__":
    sys.exit(main())
