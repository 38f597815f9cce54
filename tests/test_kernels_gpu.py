"""HIP kernel numerics vs the fp32 PyTorch reference (ops/reference.py). MI355X only."""
import pytest
import torch

from distributed_pytorch_training_amd import ops
from distributed_pytorch_training_amd.ops import reference as ref

pytestmark = pytest.mark.gpu

SIZES = [64, 4096, 1 << 20, 3_000_064]


def _rand(n, dev, seed=0):
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    return torch.randn(n, device=dev, generator=g)


@pytest.mark.parametrize("n", SIZES)
def test_grad_check(cuda, n):
    g = _rand(n, cuda)
    scale = torch.tensor([1024.0], device=cuda)
    fi = torch.zeros(1, device=cuda)
    ops.grad_check(g, scale, 0.5, fi)
    assert fi.item() == 0.0
    for pos, val in [(0, float("inf")), (n - 1, float("nan")), (n // 2, float("-inf"))]:
        h = g.clone()
        h[pos] = val
        fi.zero_()
        ops.grad_check(h, scale, 0.5, fi)
        assert fi.item() == 1.0, (pos, val)
    # finite g that overflows once unscaled by a tiny scale
    h = g.clone()
    h[3] = 3e38
    fi.zero_()
    ops.grad_check(h, torch.tensor([0.5], device=cuda), 1.0, fi)
    assert fi.item() == 1.0


@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("momentum,nesterov", [(0.0, False), (0.9, False), (0.9, True)])
def test_sgd_matches_reference(cuda, n, momentum, nesterov):
    p0, g0 = _rand(n, cuda, 1), _rand(n, cuda, 2)
    scale = torch.tensor([256.0], device=cuda)
    step = torch.zeros(1, device=cuda)
    fi = torch.zeros(1, device=cuda)
    pa, ga, ba = p0.clone(), g0.clone() * 256, torch.zeros(n, device=cuda)
    pb, gb, bb = p0.clone(), g0.clone() * 256, torch.zeros(n, device=cuda)
    for it in range(3):
        kw = dict(lr=0.1, momentum=momentum, dampening=0.0, weight_decay=5e-4, nesterov=nesterov,
                  scale=scale, host_factor=0.25, found_inf=fi, step=step, zero_grad=True)
        ops.sgd_step(pa, ga, ba, **kw)
        ref.sgd_step(pb, gb, bb, 0.1, momentum, 0.0, 5e-4, nesterov, scale, 0.25, fi, step, True)
        assert torch.count_nonzero(ga) == 0
        step += 1
        ga.copy_(g0 * 256 * (it + 2))
        gb.copy_(g0 * 256 * (it + 2))
    torch.testing.assert_close(pa, pb, rtol=1e-5, atol=1e-6)
    if momentum:
        torch.testing.assert_close(ba, bb, rtol=1e-5, atol=1e-6)


def test_sgd_skips_on_inf(cuda):
    n = 8192
    p, g, b = _rand(n, cuda, 1), _rand(n, cuda, 2), _rand(n, cuda, 3)
    p0, b0 = p.clone(), b.clone()
    fi = torch.ones(1, device=cuda)
    ops.sgd_step(p, g, b, lr=0.1, momentum=0.9, dampening=0.0, weight_decay=5e-4, nesterov=False,
                 scale=None, host_factor=1.0, found_inf=fi, step=torch.ones(1, device=cuda), zero_grad=True)
    assert torch.equal(p, p0) and torch.equal(b, b0)
    assert torch.count_nonzero(g) == 0


@pytest.mark.parametrize("adamw", [False, True])
def test_adam_matches_reference(cuda, adamw):
    n = 1 << 18
    p0, g0 = _rand(n, cuda, 4), _rand(n, cuda, 5)
    step = torch.zeros(1, device=cuda)
    fi = torch.zeros(1, device=cuda)
    pa, ma, va = p0.clone(), torch.zeros(n, device=cuda), torch.zeros(n, device=cuda)
    pb, mb, vb = p0.clone(), torch.zeros(n, device=cuda), torch.zeros(n, device=cuda)
    for it in range(4):
        ga, gb = g0 * (it + 1), g0 * (it + 1)
        ops.adam_step(pa, ga, ma, va, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=1e-2,
                      adamw=adamw, scale=None, host_factor=1.0, found_inf=fi, step=step, zero_grad=True)
        ref.adam_step(pb, gb, mb, vb, 1e-3, 0.9, 0.999, 1e-8, 1e-2, adamw, None, 1.0, fi, step, True)
        step += 1
    torch.testing.assert_close(pa, pb, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(ma, mb, rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(va, vb, rtol=1e-5, atol=1e-9)


def test_optim_tail_matches_torch_scaler_semantics(cuda):
    dev_s, dev_t = torch.tensor([65536.0], device=cuda), torch.zeros(1, dtype=torch.int32, device=cuda)
    cpu_s, cpu_t = torch.tensor([65536.0]), torch.zeros(1, dtype=torch.int32)
    step_d, step_c = torch.zeros(1, device=cuda), torch.zeros(1)
    pattern = [0, 0, 1, 0, 0, 0, 1, 1, 0, 0, 0]
    for inf in pattern:
        fd, fc = torch.tensor([float(inf)], device=cuda), torch.tensor([float(inf)])
        ops.optim_tail(dev_s, dev_t, fd, step_d, 2.0, 0.5, 3)
        ref.optim_tail(cpu_s, cpu_t, fc, step_c, 2.0, 0.5, 3)
        assert fd.item() == 0.0
        assert dev_s.item() == cpu_s.item() and dev_t.item() == cpu_t.item()
    assert step_d.item() == step_c.item() == pattern.count(0)


def test_bf16_pack_unpack(cuda):
    n = 1 << 16
    x = _rand(n, cuda, 7) * 100
    w = torch.empty(n, dtype=torch.bfloat16, device=cuda)
    ops.pack_bf16(x, w)
    assert torch.equal(w, x.to(torch.bfloat16))
    y = torch.empty(n, device=cuda)
    fi = torch.zeros(1, device=cuda)
    ops.unpack_bf16(w, y, None, 1.0, fi)
    assert torch.equal(y, w.float()) and fi.item() == 0.0
    w[5] = float("nan")
    ops.unpack_bf16(w, y, None, 1.0, fi)
    assert fi.item() == 1.0


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("rows,cols", [(1, 10), (128, 10), (257, 1000)])
def test_metrics(cuda, dtype, rows, cols):
    logits = torch.randn(rows, cols, device=cuda).to(dtype)
    targets = torch.randint(0, cols, (rows,), device=cuda)
    targets[: rows // 2] = logits[: rows // 2].float().argmax(1)
    loss = torch.tensor(1.5, device=cuda)
    a = torch.zeros(3, dtype=torch.float64, device=cuda)
    b = torch.zeros(3, dtype=torch.float64, device=cuda)
    ops.accumulate_metrics(logits, targets, loss, a)
    ref.accumulate_metrics(logits, targets, loss, b)
    assert a.tolist() == pytest.approx(b.tolist())


@pytest.mark.parametrize("nhwc", [False, True])
def test_augment_matches_reference(cuda, nhwc):
    from distributed_pytorch_training_amd.data.cifar import MEAN, STD

    data = torch.randint(0, 256, (50, 3, 32, 32), dtype=torch.uint8, device=cuda)
    idx = torch.randint(0, 50, (33,), device=cuda)
    offs = torch.randint(0, 9, (33, 2), dtype=torch.int32, device=cuda)
    flips = torch.randint(0, 2, (33,), dtype=torch.uint8, device=cuda)
    mf = torch.channels_last if nhwc else torch.contiguous_format
    a = torch.empty(33, 3, 32, 32, device=cuda, memory_format=mf)
    b = torch.empty(33, 3, 32, 32, device=cuda, memory_format=mf)
    ops.augment(data, idx, offs, flips, a, nhwc=nhwc, pad=4, mean=MEAN, std=STD)
    ref.augment(data, idx, offs, flips, b, nhwc, 4, MEAN, STD)
    torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-5)
    # eval path: no crop/flip == plain normalisation
    ops.augment(data, idx, None, None, a, nhwc=nhwc, pad=4, mean=MEAN, std=STD)
    m = torch.tensor(MEAN, device=cuda).view(1, 3, 1, 1)
    s = torch.tensor(STD, device=cuda).view(1, 3, 1, 1)
    torch.testing.assert_close(a, (data[idx].float() / 255 - m) / s, rtol=1e-5, atol=1e-5)
