"""engine/graph.py ``auto_enabled``: the ``--cuda-graph`` default (CPU: a policy check)."""


def test_graph_default_on_at_world_size_two():
    """The ``--cuda-graph`` default at N > 1: on for launch-bound steps with a capturable
    communicator (RCCL, host-async), off for torch's c10d communicator and the blocking bridge."""
    import torch

    from distributed_pytorch_training_amd.config import parse_args
    from distributed_pytorch_training_amd.engine.graph import auto_enabled
    a = parse_args(["--dataset", "synthetic", "--batch-size", "128", "--image-size", "32"])
    assert auto_enabled(a, torch.device("cuda:0"), 2, "rccl")
    assert auto_enabled(a, torch.device("cuda:0"), 8, "host-async")
    assert not auto_enabled(a, torch.device("cuda:0"), 2, "c10d")
    assert not auto_enabled(a, torch.device("cuda:0"), 2, "host")
    big = parse_args(["--dataset", "synthetic", "--batch-size", "256", "--image-size", "224"])
    assert not auto_enabled(big, torch.device("cuda:0"), 2, "rccl")
