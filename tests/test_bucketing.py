"""Bucket planner vs torch's own DDP bucket assignment."""
import pytest
import torch
import torch.distributed as dist

from distributed_pytorch_training_amd.models import build_model
from distributed_pytorch_training_amd.parallel.bucketing import MiB, assign_buckets, plan_for_arena
from distributed_pytorch_training_amd.parallel.flat import FlatArena


@pytest.mark.parametrize("name,classes", [("resnet18", 10), ("resnet50", 1000), ("vit_b_16", 1000)])
def test_matches_torch_bucket_assignment(name, classes):
    model = build_model(name, classes)
    params = list(reversed(list(model.parameters())))
    sizes = [p.numel() * p.element_size() for p in params]
    ours = assign_buckets(sizes, [1 * MiB, 25 * MiB])
    ref, _ = dist._compute_bucket_assignment_by_size(params, [1 * MiB, 25 * MiB], [False] * len(params))
    assert ours == [list(b) for b in ref]


def test_resnet18_bucket_sizes_match_survey():
    """ResNet-18/10 -> 3 buckets of ~9.02 / 25.27 / 8.36 MiB."""
    model = build_model("resnet18", 10)
    arena = FlatArena(list(reversed(list(model.parameters()))))
    plan = plan_for_arena(arena, 25.0, 1.0)
    mib = plan.sizes_mib()
    assert len(mib) == 3
    assert mib == pytest.approx([9.02, 25.27, 8.36], abs=0.02)


def test_plan_is_contiguous_partition():
    model = build_model("resnet50", 1000)
    arena = FlatArena(list(reversed(list(model.parameters()))))
    plan = plan_for_arena(arena, 8.0, 1.0)
    assert plan.offsets[0] == 0
    for b in range(plan.num_buckets - 1):
        assert plan.offsets[b] + plan.numels[b] == plan.offsets[b + 1]
    assert plan.offsets[-1] + plan.numels[-1] == arena.numel
    assert all(o % 16 == 0 for o in plan.offsets) and all(n % 16 == 0 for n in plan.numels)
    for i, b in enumerate(plan.param_bucket):
        s = arena.region(i)
        assert plan.offsets[b] <= s.start and s.stop <= plan.offsets[b] + plan.numels[b]
