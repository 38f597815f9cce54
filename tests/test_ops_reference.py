"""The kernel semantics (ops/reference.py) vs the torch code the reference inherits."""
import pytest
import torch
from hypothesis import given, settings, strategies as st

from distributed_pytorch_training_amd.amp import DeviceGradScaler
from distributed_pytorch_training_amd.ops import reference as ref


@pytest.mark.parametrize("momentum,nesterov,wd", [(0.0, False, 0.0), (0.9, False, 5e-4), (0.9, True, 1e-4)])
def test_sgd_matches_torch_sgd(momentum, nesterov, wd):
    torch.manual_seed(0)
    p = torch.randn(1000, dtype=torch.float64)
    q = torch.nn.Parameter(p.clone())
    opt = torch.optim.SGD([q], lr=0.1, momentum=momentum, weight_decay=wd, nesterov=nesterov)
    buf = torch.zeros_like(p)
    step = torch.zeros(1)
    for i in range(5):
        g = torch.randn(1000, dtype=torch.float64)
        q.grad = g.clone()
        opt.step()
        gg = g.clone()
        ref.sgd_step(p, gg, buf, 0.1, momentum, 0.0, wd, nesterov, None, 1.0, None, step, True)
        step += 1
        assert torch.count_nonzero(gg) == 0
    torch.testing.assert_close(p, q.detach())


@pytest.mark.parametrize("adamw", [False, True])
def test_adam_matches_torch(adamw):
    torch.manual_seed(0)
    p = torch.randn(500, dtype=torch.float64)
    q = torch.nn.Parameter(p.clone())
    cls = torch.optim.AdamW if adamw else torch.optim.Adam
    opt = cls([q], lr=1e-2, betas=(0.9, 0.99), eps=1e-8, weight_decay=1e-2)
    m, v, step = torch.zeros_like(p), torch.zeros_like(p), torch.zeros(1)
    for _ in range(6):
        g = torch.randn(500, dtype=torch.float64)
        q.grad = g.clone()
        opt.step()
        ref.adam_step(p, g.clone(), m, v, 1e-2, 0.9, 0.99, 1e-8, 1e-2, adamw, None, 1.0, None, step, True)
        step += 1
    torch.testing.assert_close(p, q.detach())


@settings(max_examples=40, deadline=None)
@given(pattern=st.lists(st.booleans(), min_size=1, max_size=40), interval=st.integers(1, 5))
def test_scaler_state_machine_matches_torch(pattern, interval):
    """DeviceGradScaler + optim_tail follow torch.amp.GradScaler's update rule exactly."""
    ts = torch.amp.GradScaler("cpu", init_scale=1024.0, growth_interval=interval)
    ours = DeviceGradScaler("cpu", init_scale=1024.0, growth_interval=interval)
    ts._lazy_init_scale_growth_tracker(torch.device("cpu"))
    for inf in pattern:
        fi = torch.tensor([1.0 if inf else 0.0])
        torch._amp_update_scale_(ts._scale, ts._growth_tracker, fi, 2.0, 0.5, interval)
        ours.found_inf.fill_(1.0 if inf else 0.0)
        ref.optim_tail(ours.scale_tensor, ours.growth_tracker, ours.found_inf, None, 2.0, 0.5, interval)
        assert ours.get_scale() == ts._scale.item()
        assert ours.get_growth_tracker() == ts._growth_tracker.item()


def test_scaler_state_dict_keys_match_torch():
    ours = DeviceGradScaler("cpu")
    ts = torch.amp.GradScaler("cpu")
    ts._lazy_init_scale_growth_tracker(torch.device("cpu"))
    assert set(ours.state_dict()) == set(ts.state_dict())
    ours2 = DeviceGradScaler("cpu")
    sd = ours.state_dict()
    sd["scale"] = 8.0
    ours2.load_state_dict(sd)
    assert ours2.get_scale() == 8.0


def test_grad_check_and_unscale_semantics():
    g = torch.tensor([1.0, 2.0, 3.0, 4.0])
    fi = torch.zeros(1)
    ref.grad_check(g, torch.tensor([2.0]), 1.0, fi)
    assert fi.item() == 0.0
    g[1] = float("nan")
    ref.grad_check(g, torch.tensor([2.0]), 1.0, fi)
    assert fi.item() == 1.0


def test_metrics_reference():
    logits = torch.tensor([[0.1, 0.9], [0.8, 0.2], [0.3, 0.7]])
    t = torch.tensor([1, 1, 1])
    acc = torch.zeros(3, dtype=torch.float64)
    ref.accumulate_metrics(logits, t, torch.tensor(0.5), acc)
    assert acc.tolist() == [1.5, 2.0, 3.0]


def test_augment_reference_against_manual_torchvision_math():
    """RandomCrop(32, padding=4) + HFlip + ToTensor + Normalize, computed the slow way."""
    torch.manual_seed(0)
    data = torch.randint(0, 256, (4, 3, 32, 32), dtype=torch.uint8)
    idx = torch.tensor([2, 0, 3])
    offs = torch.tensor([[0, 8], [4, 4], [7, 1]], dtype=torch.int32)
    flips = torch.tensor([1, 0, 1], dtype=torch.uint8)
    mean, std = (0.4914, 0.4822, 0.4465), (0.2470, 0.2435, 0.2616)
    out = torch.empty(3, 3, 32, 32)
    ref.augment(data, idx, offs, flips, out, False, 4, mean, std)
    for b in range(3):
        img = torch.nn.functional.pad(data[idx[b]], (4, 4, 4, 4))            # uint8 zero pad
        dy, dx = int(offs[b, 0]), int(offs[b, 1])
        crop = img[:, dy:dy + 32, dx:dx + 32]
        if flips[b]:
            crop = crop.flip(-1)
        exp = (crop.float() / 255 - torch.tensor(mean).view(3, 1, 1)) / torch.tensor(std).view(3, 1, 1)
        torch.testing.assert_close(out[b], exp)
