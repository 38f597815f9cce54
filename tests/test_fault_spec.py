"""``--fault-inject``: one flag, one spec, one exit status (utils/fault.py)."""
import os
import subprocess
import sys

import pytest

from distributed_pytorch_training_amd.config import parse_args
from distributed_pytorch_training_amd.utils.fault import FAULT_EXIT_CODE, FaultSpec


def test_spec_forms():
    assert FaultSpec.parse("rank=1,step=3") == FaultSpec(rank=1, step=3)
    assert FaultSpec.parse("epoch=2,rank=0") == FaultSpec(rank=0, epoch=2)
    assert FaultSpec.parse(None) is None and FaultSpec.parse("") is None


@pytest.mark.parametrize("bad", ["1:3", "2:1", "rank=1", "step=3", "rank=1,step=3,epoch=2",
                                 "rank=1,rank=2,step=1", "rank=x,step=1", "node=1,step=1"])
def test_malformed_specs_are_rejected_at_parse_time(bad):
    with pytest.raises(ValueError):
        parse_args(["--fault-inject", bad])


def test_the_old_epoch_flag_is_gone():
    with pytest.raises(SystemExit):
        parse_args(["--inject-fault", "2:1"])


def test_fire_exits_once_per_output_dir(tmp_path):
    code = ("import sys; from distributed_pytorch_training_amd.utils.fault import FaultSpec; "
            f"FaultSpec.parse('rank=0,epoch=1').fire({str(tmp_path)!r}); print('survived')")
    env = dict(os.environ, PYTHONPATH=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    first = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=120)
    assert first.returncode == FAULT_EXIT_CODE and "injected fault at epoch 1" in first.stdout
    again = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=120)
    assert again.returncode == 0 and "survived" in again.stdout


def test_step_faults_fire_every_run(tmp_path):
    """a step fault leaves no marker - the same fault test run twice in one output
    directory injects the fault both times (never a silent clean pass)."""
    code = ("from distributed_pytorch_training_amd.utils.fault import FaultSpec; "
            f"FaultSpec.parse('rank=0,step=3').fire({str(tmp_path)!r}); print('survived')")
    env = dict(os.environ, PYTHONPATH=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    for _ in range(2):
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=120)
        assert r.returncode == FAULT_EXIT_CODE and "injected fault at step 3" in r.stdout
    assert not list(tmp_path.iterdir())


def test_suppressed_epoch_fault_warns_once(tmp_path):
    spec = FaultSpec.parse("rank=0,epoch=1")
    spec.marker(str(tmp_path)).touch()
    logs = []
    for _ in range(3):
        spec.fire(str(tmp_path), logs.append)
    assert len(logs) == 1 and "NOT injected" in logs[0]
