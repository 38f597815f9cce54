"""Bucket planner vs torch's own DDP bucket assignment."""
import pytest
import torch
import torch.distributed as dist

from distributed_pytorch_training_amd.models import build_model
from distributed_pytorch_training_amd.parallel.bucketing import MiB, assign_buckets, plan_for_arena, tail_split
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


@pytest.mark.parametrize("name,classes", [("resnet50", 1000), ("vit_b_16", 1000), ("resnet18", 10)])
@pytest.mark.parametrize("cap", [0.5, 1.0, 4.0])
def test_last_bucket_cap(name, classes, cap):
    """--last-bucket-mb: the bucket that becomes ready last fits the cap (or is one tensor that
    alone exceeds it), the buckets before it are the reference's plan of the prefix, and the
    partition stays contiguous and complete."""
    model = build_model(name, classes)
    arena = FlatArena(list(reversed(list(model.parameters()))))
    plan = plan_for_arena(arena, 25.0, 1.0, last_bucket_mb=cap)
    full = plan_for_arena(arena, 25.0, 1.0)
    sizes = [p.numel() * 4 for p in arena.params]
    if tail_split(sizes, int(cap * MiB)) == len(sizes):
        # no split: the fitting suffix was under half the cap (or the plain tail already fits)
        assert plan.members == full.members
        return
    last = plan.members[-1]
    last_bytes = sum(arena.params[i].numel() * 4 for i in last)
    assert cap * MiB / 2 <= last_bytes <= cap * MiB, (last_bytes, len(last))
    # maximal: the tensor just before the tail would not have fit
    first = last[0]
    if first > 0:
        assert last_bytes + arena.params[first - 1].numel() * 4 > cap * MiB
    assert plan.offsets[-1] + plan.numels[-1] == arena.numel
    assert sorted(i for m in plan.members for i in m) == list(range(len(arena.params)))
    assert assign_buckets(sizes[:tail_split(sizes, int(cap * MiB))], [MiB, 25 * MiB]) == plan.members[:-1]
    assert plan.sizes_mib()[-1] <= full.sizes_mib()[-1]


def test_last_bucket_cap_skips_a_useless_split():
    """ViT-B/16: the suffix that fits a 1 MiB tail is the 3 KiB class token alone (the 2.25 MiB
    patch embedding before it is ready at the same moment): no split, the plan is torch's."""
    model = build_model("vit_b_16", 1000)
    arena = FlatArena(list(reversed(list(model.parameters()))))
    assert plan_for_arena(arena, 25.0, 1.0, 1.0).members == plan_for_arena(arena, 25.0, 1.0).members


def test_last_bucket_cap_resnet50_defaults():
    """The ResNet-50 plan with the default 1 MiB tail: the stem/layer1 leftover (9.27 MiB with
    torch DDP's plan) becomes a ~1 MiB tail bucket plus the rest of layer1 reduced earlier."""
    model = build_model("resnet50", 1000)
    arena = FlatArena(list(reversed(list(model.parameters()))))
    ref = plan_for_arena(arena, 25.0, 1.0).sizes_mib()
    got = plan_for_arena(arena, 25.0, 1.0, last_bucket_mb=1.0).sizes_mib()
    assert ref[-1] == pytest.approx(9.27, abs=0.02)
    assert got[-1] <= 1.0 and sum(got) == pytest.approx(sum(ref))
    assert got[:len(ref) - 1] == ref[:-1]


@pytest.mark.parametrize("name,classes", [("resnet18", 10), ("resnet50", 1000)])
def test_default_cli_plan_is_torch_ddp_plan(name, classes):
    """additive defaults reproduce the reference.  The plan NativeDDP builds from the
    default CLI (``--bucket-cap-mb 25 --first-bucket-mb 1 --last-bucket-mb 0``) is exactly
    ``dist._compute_bucket_assignment_by_size`` with 1 MiB / 25 MiB caps (reference
    train_ddp.py:305-310, DDP defaults)."""
    from distributed_pytorch_training_amd.config import parse_args
    args = parse_args([])
    assert (args.bucket_cap_mb, args.first_bucket_mb, args.last_bucket_mb) == (25.0, 1.0, 0.0)
    model = build_model(name, classes)
    params = list(reversed(list(model.parameters())))
    arena = FlatArena(params)
    plan = plan_for_arena(arena, args.bucket_cap_mb, args.first_bucket_mb, args.last_bucket_mb)
    ref, _ = dist._compute_bucket_assignment_by_size(params, [1 * MiB, 25 * MiB], [False] * len(params))
    assert plan.members == [list(b) for b in ref]
