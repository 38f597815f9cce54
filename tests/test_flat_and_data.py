"""Flat arenas (views, channels_last, relayout) and the CIFAR readers / device loaders."""
import pickle

import numpy as np
import pytest
import torch

from distributed_pytorch_training_amd.data.cifar import MEAN, STD, load_cifar10
from distributed_pytorch_training_amd.data.loader import DeviceImageLoader, SyntheticLoader
from distributed_pytorch_training_amd.data.sampler import SequentialSampler
from distributed_pytorch_training_amd.models import build_model
from distributed_pytorch_training_amd.parallel.flat import BufferArena, FlatArena


def test_arena_views_share_storage_and_keep_strides():
    m = build_model("resnet18", 10, channels_last=True)
    params = list(m.parameters())
    strides = [p.stride() for p in params]
    values = [p.detach().clone() for p in params]
    arena = FlatArena(params)
    assert arena.numel % 64 == 0 and all(o % 16 == 0 for o in arena.offsets)
    for p, s, v, g in zip(params, strides, values, arena.grad_views):
        assert p.stride() == s and torch.equal(p, v)
        assert p.untyped_storage().data_ptr() == arena.param_flat.untyped_storage().data_ptr()
        assert p.grad is g
    with torch.no_grad():
        arena.param_flat.add_(1.0)
    assert torch.equal(params[0], values[0] + 1)
    x = torch.randn(2, 3, 32, 32).contiguous(memory_format=torch.channels_last)
    m(x).sum().backward()                           # AccumulateGrad writes into the arena
    assert arena.grad_flat.abs().sum() > 0
    assert all(p.grad.data_ptr() == g.data_ptr() for p, g in zip(params, arena.grad_views))


def test_relayout_moves_values_and_state():
    m = torch.nn.Sequential(torch.nn.Linear(5, 7), torch.nn.Linear(7, 3))
    params = list(m.parameters())
    arena = FlatArena(params)
    state = torch.arange(arena.numel, dtype=torch.float32)
    before = [p.detach().clone() for p in params]
    state_views = [v.clone() for v in arena.views(state)]
    perm = arena.relayout([3, 1, 0, 2], extra=[state])
    assert [id(p) for p in arena.params] == [id(params[i]) for i in [3, 1, 0, 2]]
    for p, b in zip(params, before):
        assert torch.equal(p, b)
    new_views = arena.views(perm.extra[0])
    for j, i in enumerate([3, 1, 0, 2]):
        assert torch.equal(new_views[j], state_views[i])


def test_buffer_arena():
    m = build_model("resnet18", 10)
    ref = {k: v.clone() for k, v in m.state_dict().items() if "running" in k or "num_batches" in k}
    ba = BufferArena(m)
    assert len(ba) == 2   # fp32 stats + int64 counters
    sd = m.state_dict()
    for k, v in ref.items():
        assert torch.equal(sd[k], v)
    m.train()
    m(torch.randn(4, 3, 32, 32))
    assert ba.flats[torch.int64].sum() == 20     # 20 BN layers, num_batches_tracked += 1 in place


def _write_fake_cifar(root, kind):
    rng = np.random.default_rng(0)
    names = [f"data_batch_{i}" for i in range(1, 6)] + ["test_batch"]
    d = root / ("cifar-10-batches-bin" if kind == "bin" else "cifar-10-batches-py")
    d.mkdir()
    truth = {}
    for n in names:
        x = rng.integers(0, 256, (10, 3072), dtype=np.uint8)
        y = rng.integers(0, 10, 10)
        truth[n] = (x, y)
        if kind == "bin":
            rec = np.concatenate([y.astype(np.uint8)[:, None], x], axis=1)
            rec.tofile(d / (n + ".bin"))
        else:
            with open(d / n, "wb") as f:
                pickle.dump({b"data": x, b"labels": y.tolist()}, f)
    return truth


@pytest.mark.parametrize("kind", ["bin", "py"])
def test_cifar_readers(tmp_path, kind):
    truth = _write_fake_cifar(tmp_path, kind)
    x, y = load_cifar10(str(tmp_path), train=True)
    assert x.shape == (50, 3, 32, 32) and x.dtype == np.uint8
    assert np.array_equal(x[:10].reshape(10, -1), truth["data_batch_1"][0])
    assert np.array_equal(y[:10], truth["data_batch_1"][1])
    xt, yt = load_cifar10(str(tmp_path), train=False)
    assert xt.shape == (10, 3, 32, 32)


def test_cifar_py_reader_refuses_code(tmp_path):
    d = tmp_path / "cifar-10-batches-py"
    d.mkdir()

    class Evil:
        def __reduce__(self):
            return (print, ("pwned",))

    for n in [f"data_batch_{i}" for i in range(1, 6)] + ["test_batch"]:
        with open(d / n, "wb") as f:
            pickle.dump({b"data": Evil(), b"labels": []}, f)
    with pytest.raises(pickle.UnpicklingError):
        load_cifar10(str(tmp_path), train=True)


def test_missing_cifar_message(tmp_path):
    with pytest.raises(FileNotFoundError, match="synthetic"):
        load_cifar10(str(tmp_path), train=True)


def test_device_loader_cpu_eval_path():
    imgs = torch.randint(0, 256, (10, 3, 32, 32), dtype=torch.uint8)
    labels = torch.arange(10)
    ld = DeviceImageLoader(imgs, labels, SequentialSampler(10), 4, "cpu", augment=False, mean=MEAN, std=STD)
    batches = list(ld)
    assert len(ld) == 3 and [b[0].shape[0] for b in batches] == [4, 4, 2]
    m = torch.tensor(MEAN).view(1, 3, 1, 1)
    s = torch.tensor(STD).view(1, 3, 1, 1)
    torch.testing.assert_close(batches[0][0], (imgs[:4].float() / 255 - m) / s)
    assert torch.equal(batches[2][1], labels[8:])


def test_synthetic_loader_lengths():
    ld = SyntheticLoader(100, 32, 16, 10, "cpu")
    sizes = [x.shape[0] for x, _ in ld]
    assert sizes == [32, 32, 32, 4]
    assert len(SyntheticLoader(100, 32, 16, 10, "cpu", max_steps=2)) == 2
