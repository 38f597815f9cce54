"""Failure detection and debug checks of the distributed path.

* a rank that dies mid-epoch (``--fault-inject``) must not hang its peer: the survivor exits
  non-zero within the timeout (+ slack) - the reference has no timeout handling at all
  (train_ddp.py:65 takes the PG defaults, no watchdog settings);
* ranks whose bucket plans differ must raise at construction instead of deadlocking in the
  first backward (collective-sequence check, parallel/ddp.py ``_verify_plan``);
* the reducer's debug assertions (double ready-mark) raise.

Ranks are plain subprocesses with the env:// variables set by hand (not torchrun: its agent
would tear the survivor down itself and hide what the framework does)."""
import os
import socket
import subprocess
import sys
import time

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COMMON = ["--dataset", "synthetic", "--image-size", "32", "--num-classes", "10",
          "--synthetic-train-size", "2048", "--synthetic-val-size", "64", "--batch-size", "16",
          "--print-freq", "1000", "--epochs", "1", "--model", "resnet18"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.slow
def test_dead_peer_survivor_exits_nonzero(tmp_path):
    timeout_s = 20
    port = _free_port()
    procs = []
    t0 = time.time()
    for r in range(2):
        env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2", WORLD_SIZE="2", RANK=str(r),
                   LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        cmd = [sys.executable, os.path.join(ROOT, "train_ddp.py"), *COMMON, "--output-dir", str(tmp_path),
               "--dist-timeout", str(timeout_s), "--fault-inject", "rank=1,step=3"]
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                      text=True, cwd=ROOT))
    try:
        out1, _ = procs[1].communicate(timeout=300)
        t_dead = time.time()
        out0, _ = procs[0].communicate(timeout=timeout_s + 60)
        t_survivor = time.time()
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert procs[1].returncode == 17, out1          # the injected fault
    assert procs[0].returncode != 0, out0           # the survivor did not pretend success
    assert t_survivor - t_dead < timeout_s + 10, (t_survivor - t_dead, out0)
    assert "training failed" in out0, out0
    assert time.time() - t0 < 400


def _plan_worker(rank, ws, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    from distributed_pytorch_training_amd.models import build_model
    from distributed_pytorch_training_amd.parallel.ddp import NativeDDP
    torch.manual_seed(0)
    m = build_model("resnet18", 10)
    msg = "ok"
    try:
        # rank 1 buckets differently: the plans (and the collective sequence) would not pair up
        NativeDDP(m, rank=rank, world_size=ws, bucket_cap_mb=25.0 if rank == 0 else 5.0)
    except RuntimeError as e:
        msg = str(e)
    with open(os.path.join(out_dir, f"r{rank}.txt"), "w") as f:
        f.write(msg)
    dist.destroy_process_group()


@pytest.mark.slow
def test_bucket_plan_mismatch_raises_on_every_rank(tmp_path):
    mp.start_processes(_plan_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, start_method="spawn")
    for r in range(2):
        msg = (tmp_path / f"r{r}.txt").read_text()
        assert "bucket plans differ" in msg, msg


def _double_mark_worker(rank, ws, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    from distributed_pytorch_training_amd.parallel.ddp import NativeDDP
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(8, 8), torch.nn.ReLU(), torch.nn.Linear(8, 2))
    ddp = NativeDDP(m, rank=rank, world_size=ws, debug=True)
    x = torch.randn(4, 8)
    loss = ddp(x).sum()
    loss.backward(retain_graph=True)
    msg = "no error"
    try:
        loss.backward()      # second backward without a forward: every parameter marked twice
    except RuntimeError as e:
        msg = str(e)
    with open(os.path.join(out_dir, f"r{rank}.txt"), "w") as f:
        f.write(msg)
    dist.destroy_process_group()


@pytest.mark.slow
def test_reducer_debug_double_mark_raises(tmp_path):
    mp.start_processes(_double_mark_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2,
                       start_method="spawn")
    for r in range(2):
        msg = (tmp_path / f"r{r}.txt").read_text()
        assert "marked ready twice" in msg, msg
