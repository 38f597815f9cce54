"""CPU checks for the asynchronous host bridge's process-group seam (csrc/host_comm.cpp).

``--comm host-async`` runs its gloo collectives from C++ on HIP's host-function thread without
the GIL, on the ``c10d::ProcessGroup`` behind a ``torch.distributed`` group object.  The
binding must be able to take that object from Python (shared pybind11 type registry with
torch); the GPU side of the bridge is covered by tests/test_multirank_gpu.py.
"""

import pytest
import torch.distributed as dist

from distributed_pytorch_training_amd import ops


@pytest.fixture
def gloo_world(tmp_path):
    dist.init_process_group("gloo", init_method=f"file://{tmp_path / 'store'}", rank=0, world_size=1)
    try:
        yield
    finally:
        dist.destroy_process_group()


@pytest.mark.skipif(not ops.native_available(), reason="native extension not built")
def test_process_group_object_reaches_cpp(gloo_world):
    from distributed_pytorch_training_amd.parallel import comm

    C = ops.native()
    assert C.HostBridgeComm._process_group_size(dist.group.WORLD) == 1
    comm._ASYNC_GROUP = None
    try:
        assert C.HostBridgeComm._process_group_size(comm._async_group()) == 1
    finally:
        comm._ASYNC_GROUP = None


@pytest.mark.skipif(not ops.native_available(), reason="native extension not built")
def test_non_group_object_is_rejected():
    with pytest.raises((TypeError, RuntimeError)):
        ops.native().HostBridgeComm._process_group_size(object())
