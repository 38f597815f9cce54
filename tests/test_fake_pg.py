"""Reducer bookkeeping at larger world sizes on torch's ``fake`` process group.

The fake backend completes every collective instantly without moving data, so one process
can play rank 0 of an 8-rank job: construction-time collectives (shape verification,
parameter/buffer broadcast), per-bucket all-reduce launches in index order, BN-buffer sync,
the one-time bucket rebuild and no_sync all run through the real code paths.
"""
import pytest
import torch
import torch.distributed as dist
from torch.testing._internal.distributed.fake_pg import FakeStore

from distributed_pytorch_training_amd.models import build_model
from distributed_pytorch_training_amd.optim import FusedSGD
from distributed_pytorch_training_amd.parallel.ddp import NativeDDP


@pytest.fixture
def fake_pg():
    dist.init_process_group("fake", store=FakeStore(), rank=0, world_size=8)
    yield
    dist.destroy_process_group()


def test_reducer_launches_every_bucket_in_order(fake_pg):
    torch.manual_seed(0)
    model = build_model("resnet18", 10)
    calls = []
    ddp = NativeDDP(model, rank=0, world_size=8, bucket_cap_mb=2.0, first_bucket_mb=0.5)
    orig = ddp._cpu_allreduce

    def spy(b, off, n):
        calls.append((b, off, n))
        orig(b, off, n)

    ddp._cpu_allreduce = spy
    ddp._build_reducer()          # rebind the callback
    opt = FusedSGD(ddp.arena, lr=0.1, momentum=0.9)
    x, y = torch.randn(4, 3, 32, 32), torch.randint(0, 10, (4,))
    torch.nn.functional.cross_entropy(ddp(x), y).backward()
    nb = ddp.plan.num_buckets
    assert [c[0] for c in calls] == list(range(nb))                 # strictly in index order
    assert sum(c[2] for c in calls) == ddp.arena.numel              # the whole arena, once
    assert ddp.reducer.backward_count == 1
    assert ddp.maybe_rebuild_buckets(opt) in (True, False)
    calls.clear()
    with ddp.no_sync():
        torch.nn.functional.cross_entropy(ddp(x), y).backward()
    assert calls == []                                             # no collectives under no_sync
    torch.nn.functional.cross_entropy(ddp(x), y).backward()
    assert [c[0] for c in calls] == list(range(ddp.plan.num_buckets))
    assert ddp.grad_factor == 1 / 8


def test_bucket_plan_sizes_for_vit(fake_pg):
    model = build_model("vit_b_16", 1000)
    ddp = NativeDDP(model, rank=0, world_size=8)
    mib = ddp.bucket_sizes_mib()
    # ViT-B/16 -> 14 buckets (2.93, 12 x 27.04, 2.84 MiB) with 1/25 MiB caps
    assert len(mib) == 14
    assert mib[0] == pytest.approx(2.93, abs=0.05)
    assert all(m == pytest.approx(27.04, abs=0.1) for m in mib[1:13])
