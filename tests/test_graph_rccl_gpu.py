"""RCCL inside a hipGraph.

The reference's multi-GPU run (ResNet-18 / 32 px / batch 128, reference train_ddp.py:26-27,154,
195-244) is launch-bound, so at N > 1 the framework replays its step as a hipGraph whose backward
holds the bucket all-reduces of the framework's RCCL communicator.  On one GPU that path runs with
a forced one-rank ``RcclComm`` (``DPT_FORCE_COLLECTIVES=1``: the reducer issues every bucket's
``ncclAllReduce`` although N = 1, an identity): the captured graph must contain them, the first
replay is validated against eager steps from the same state (``engine/graph.py check_replay``),
and the watchdog must retire the completion marker each replay hands it (``Collective.track``).
"""
import os
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_rccl_allreduce_captured_and_replayed_in_graph():
    code = textwrap.dedent("""
        import time, torch
        from distributed_pytorch_training_amd.config import parse_args
        from distributed_pytorch_training_amd.engine.trainer import Trainer
        from distributed_pytorch_training_amd.models import build_model
        from distributed_pytorch_training_amd.parallel.comm import make_comm
        from distributed_pytorch_training_amd.utils.env import graph_safe_miopen, setup_miopen_env
        graph_safe_miopen()
        setup_miopen_env()
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        torch.manual_seed(0)
        model = build_model("resnet18", 10, dev, image_size=32, channels_last=True)
        args = parse_args(["--dataset", "synthetic", "--batch-size", "128", "--image-size", "32",
                           "--num-classes", "10", "--amp", "--amp-dtype", "bf16", "--channels-last",
                           "--cuda-graph"])
        # the framework communicator, forced at N = 1 (make_comm only builds one for N > 1 itself)
        tr = Trainer(model, args, 0, 1, dev, comm=make_comm(dev, 0, 1), log=lambda s: None)
        comm = tr.ddp.comm
        assert comm is not None and comm.kind == "rccl" and comm.world_size == 1, comm
        comm.enable_watchdog(60.0, 0.02, -1.0)
        g = torch.Generator(device=dev).manual_seed(1)
        batches = [(torch.randn(128, 3, 32, 32, device=dev, generator=g).contiguous(memory_format=torch.channels_last),
                    torch.randint(0, 10, (128,), device=dev, generator=g)) for _ in range(3)]
        ops0 = comm.ops
        for i in range(4):                     # 3 eager warm-up steps, then the capture step
            tr.train_step(*batches[i % 3])
        torch.cuda.synchronize()
        gs = tr.graphed
        assert gs is not None and gs.graph is not None and not gs.failed, (gs.failed, gs.validation)
        captured_ops = comm.ops - ops0
        assert captured_ops >= 4 * tr.ddp.plan.num_buckets, (captured_ops, tr.ddp.plan.num_buckets)
        tracked0 = comm.watchdog_tracked
        n = 6
        for i in range(n):
            tr.train_step(*batches[i % 3])
        v = gs.validation
        assert v is not None and v["ok"], v
        # the capture call validated (eager x2 + replay x2 from one saved state) and stands for one
        # replayed step; every later call is a plain replay
        assert gs.replays == n + 1, gs.replays
        # each replay handed the watchdog one marker (the validation's eager steps track their own
        # collectives: RcclComm tracks outside capture)
        assert comm.watchdog_tracked - tracked0 >= n, (comm.watchdog_tracked, tracked0)
        torch.cuda.synchronize()
        t0 = time.time()
        while comm.watchdog_outstanding and time.time() - t0 < 5.0:
            time.sleep(0.02)
        assert comm.watchdog_outstanding == 0 and not comm.watchdog_tripped
        comm.check()
        assert torch.isfinite(tr.ddp.arena.param_flat).all()
        print("ok", {"replays": gs.replays, "validation": {k: v[k] for k in ("replay_vs_eager", "eager_vs_eager",
                                                                               "tol_whole")},
                     "tracked": comm.watchdog_tracked - tracked0, "captured_ops": captured_ops}, flush=True)
        tr.close()
    """)
    env = dict(os.environ, DPT_FORCE_COLLECTIVES="1")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, env=env, timeout=300)
    print(r.stdout[-2000:])
    assert r.returncode == 0 and "ok" in r.stdout, (r.stdout + r.stderr)[-4000:]
