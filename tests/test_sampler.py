"""ShardedSampler == torch DistributedSampler (reference train_ddp.py:121-127)."""
import pytest
import torch
from hypothesis import given, settings, strategies as st
from torch.utils.data import DistributedSampler

from distributed_pytorch_training_amd.data.sampler import RandomSampler, SequentialSampler, ShardedSampler


class _DS:
    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n


@settings(max_examples=60, deadline=None)
@given(n=st.integers(1, 3000), ws=st.integers(1, 9), epoch=st.integers(0, 5), shuffle=st.booleans(),
       drop_last=st.booleans())
def test_matches_torch_distributed_sampler(n, ws, epoch, shuffle, drop_last):
    if drop_last and n < ws:
        return
    for rank in range(ws):
        ref = DistributedSampler(_DS(n), num_replicas=ws, rank=rank, shuffle=shuffle, drop_last=drop_last)
        ref.set_epoch(epoch)
        ours = ShardedSampler(n, ws, rank, shuffle=shuffle, drop_last=drop_last)
        ours.set_epoch(epoch)
        assert list(ref) == list(ours)
        assert len(ref) == len(ours)


@pytest.mark.parametrize("ws,steps", [(1, 391), (2, 196), (4, 98), (8, 49)])
def test_cifar_step_counts(ws, steps):
    """SURVEY.md §2.8 derived table: steps/epoch at batch 128 on 50k images."""
    import math

    s = ShardedSampler(50000, ws, 0)
    assert math.ceil(len(s) / 128) == steps


def test_random_sampler_matches_torch_random_sampler():
    from torch.utils.data import RandomSampler as TorchRS

    torch.manual_seed(5)
    ref = list(TorchRS(range(100)))
    torch.manual_seed(5)
    ours = RandomSampler(100).indices().tolist()
    assert ref == ours


def test_sequential():
    assert SequentialSampler(5).indices().tolist() == [0, 1, 2, 3, 4]
