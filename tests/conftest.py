import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP kernels, RCCL)")
    config.addinivalue_line("markers", "slow: multi-process or long CPU test")
    # The session's GPU tests capture hipGraphs after other tests already ran MIOpen convolutions,
    # and MIOpen reads its solver switches once per process: exclude the graph-unsafe solvers
    # before anything runs (utils/env.py GRAPH_UNSAFE_MIOPEN_SOLVERS).
    from distributed_pytorch_training_amd.utils.env import graph_safe_miopen
    graph_safe_miopen()


# GPU suite order under ``-x``: cheap, deterministic kernel-numerics files first, then the engine
# and comm tiers, and the long stochastic graph / training-parity runs last, so a failure there
# can never hide the optimizer, scaler, reducer or kernel evidence.
_FIRST = ("test_kernels_gpu.py", "test_bn_gpu.py", "test_conv_gpu.py", "test_attention_gpu.py",
          "test_vit_gpu.py", "test_comm_gpu.py", "test_engine_gpu.py", "test_bench_contract.py",
          "test_multirank_gpu.py", "test_serialized_gpu.py")
_LAST = ("test_graph_replay_gpu.py", "test_graph_default_run_gpu.py", "test_bf16_parity_gpu.py",
         "test_training_parity_gpu.py")


def _order_key(item) -> int:
    name = os.path.basename(str(item.fspath))
    if name in _FIRST:
        return _FIRST.index(name)
    if name in _LAST:
        return 1000 + _LAST.index(name)
    return 500


def pytest_collection_modifyitems(session, config, items):
    items.sort(key=_order_key)        # stable: keeps the in-file order of each file


@pytest.fixture(autouse=True)
def _restore_cudnn_flags():
    """Tests that set ``torch.backends.cudnn.deterministic`` (parity tests) must not leak it: in
    deterministic mode MIOpen picks its CK grouped backward-data solver, which is wrong under
    hipGraph replay (utils/env.py), so a later graph test would validate-and-fall-back."""
    import torch
    old = (torch.backends.cudnn.benchmark, torch.backends.cudnn.deterministic)
    yield
    torch.backends.cudnn.benchmark, torch.backends.cudnn.deterministic = old


@pytest.fixture(autouse=True)
def _collect_before_gpu_tests(request):
    """Collect the previous tests' garbage BEFORE a GPU test starts: a reference cycle collected in
    the middle of a later hipGraph capture runs destructors whose HIP calls are illegal there (one
    such collection aborted a GPU test run; engine/graph.py also disables collection while it
    captures)."""
    if request.node.get_closest_marker("gpu") is not None:
        import gc
        gc.collect()
    yield


@pytest.fixture(scope="session")
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from distributed_pytorch_training_amd import ops

    ops.native()  # GPU tests must run the HIP path: fail loudly if it is missing
    return torch.device("cuda:0")
