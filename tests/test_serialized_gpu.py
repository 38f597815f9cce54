"""``AMD_SERIALIZE_KERNEL=3`` tier: the HIP runtime waits for every kernel
(and copy) to finish before and after launching it, which turns a missing stream/event
dependency - a kernel on the comm stream reading a bucket before the compute stream wrote
it, an optimizer launch racing the last all-reduce - into a DIFFERENT result from the
normal, overlapped run.  Both runs start in fresh interpreters before any GPU call, so the
variable is read by the runtime at initialisation.

* the native engine (MFMA convs, fused BN, steal-mode reducer over the forced 1-rank RCCL
  communicator, comm-stream AMP check, fused SGD, weight shadows): 3 steps serialized and
  overlapped must give bit-identical parameters, scale and metrics (every kernel of the path
  is deterministic: no floating-point atomics);
* the world-size-2 exact-reduction test (tests/test_multirank_gpu.py) re-runs serialized.
"""
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu

_STEPS = """
    import hashlib, torch
    from distributed_pytorch_training_amd.config import parse_args
    from distributed_pytorch_training_amd.engine.trainer import Trainer
    from distributed_pytorch_training_amd.models import build_model
    from distributed_pytorch_training_amd.parallel.comm import make_comm
    from distributed_pytorch_training_amd.utils.env import setup_miopen_env
    setup_miopen_env()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    args = parse_args(["--model", "resnet18", "--dataset", "synthetic", "--image-size", "32",
                       "--num-classes", "10", "--batch-size", "64", "--amp", "--amp-dtype", "bf16",
                       "--channels-last", "--no-cuda-graph", "--bucket-cap-mb", "4"])
    torch.manual_seed(0)
    model = build_model("resnet18", 10, dev, image_size=32, channels_last=True)
    tr = Trainer(model, args, 0, 1, dev, comm=make_comm(dev, 0, 1), log=lambda s: None)
    g = torch.Generator(device=dev).manual_seed(7)
    for _ in range(3):
        x = torch.randn(64, 3, 32, 32, device=dev, generator=g).contiguous(memory_format=torch.channels_last)
        y = torch.randint(0, 10, (64,), device=dev, generator=g)
        tr.train_step(x, y)
    torch.cuda.synchronize()
    h = hashlib.sha256(tr.ddp.arena.param_flat.cpu().numpy().tobytes()).hexdigest()
    print("RESULT", h, tr.scaler.get_scale(), tr.metrics.tolist(), flush=True)
    tr.close()
"""


def _run(serialize: bool, code: str, timeout: int = 240):
    env = dict(os.environ, DPT_FORCE_COLLECTIVES="1")
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    env.pop("AMD_SERIALIZE_KERNEL", None)
    if serialize:
        env["AMD_SERIALIZE_KERNEL"] = "3"
    return subprocess.run([sys.executable, "-c", textwrap.dedent(code)], capture_output=True, text=True,
                          env=env, timeout=timeout, cwd=ROOT)


def test_native_engine_serialized_equals_overlapped():
    res = {}
    for ser in (False, True):
        r = _run(ser, _STEPS)
        assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
        res[ser] = [l for l in r.stdout.splitlines() if l.startswith("RESULT")][-1]
    print(res[False])
    assert res[False] == res[True], res


def test_multirank_exact_reduction_serialized(tmp_path):
    """tests/test_multirank_gpu.py's exact world-size-2 reduction (fp32 wire) with every
    kernel serialized: the same exact-sum assertion must hold."""
    env = dict(os.environ, AMD_SERIALIZE_KERNEL="3")
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    node = "tests/test_multirank_gpu.py::test_world_size_2_reduces_local_gradients_exactly[native_fp32_wire]"
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-s", "-p", "no:cacheprovider", node],
                       capture_output=True, text=True, env=env, timeout=400, cwd=ROOT)
    assert r.returncode == 0 and "1 passed" in r.stdout, (r.stdout + r.stderr)[-4000:]
    print([l for l in r.stdout.splitlines() if "worst per-tensor" in l])
