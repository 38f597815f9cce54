"""Fused channels_last BN(+add)(+ReLU) HIP kernels vs the unfused PyTorch fp32 composition."""
import pytest
import torch

from distributed_pytorch_training_amd.models.layers import FusedBatchNorm2d, bn_act
from distributed_pytorch_training_amd.ops.bn import reference_bn_act

pytestmark = pytest.mark.gpu

TOL = {torch.float32: (1e-4, 1e-4), torch.bfloat16: (2e-2, 2e-2), torch.float16: (3e-3, 3e-3)}


def _mk(shape, dtype, dev, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    t = torch.randn(shape, device=dev, generator=g) * 1.7 + 0.3
    return t.to(dtype).contiguous(memory_format=torch.channels_last)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("shape", [(4, 64, 7, 9), (32, 256, 14, 14), (8, 2048, 7, 7), (2, 8, 3, 3)])
@pytest.mark.parametrize("relu,res", [(True, False), (True, True), (False, False), (False, True)])
def test_fused_bn_train_matches_reference(cuda, dtype, shape, relu, res):
    C = shape[1]
    x = _mk(shape, dtype, cuda, 1).requires_grad_()
    r = _mk(shape, dtype, cuda, 2).requires_grad_() if res else None
    bn = FusedBatchNorm2d(C).to(cuda)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
        bn.running_mean.uniform_(-0.1, 0.1)
    ref_rm, ref_rv = bn.running_mean.clone(), bn.running_var.clone()
    w = bn.weight.detach().clone().requires_grad_()
    b = bn.bias.detach().clone().requires_grad_()
    xr = x.detach().float().requires_grad_()
    rr = r.detach().float().requires_grad_() if res else None
    y = bn_act(bn, x, relu=relu, residual=r)
    zr = reference_bn_act(xr, rr, w, b, ref_rm, ref_rv, True, bn.momentum, bn.eps, False)
    rt, at = TOL[dtype]
    assert y.dtype == dtype and y.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(y.float(), torch.relu(zr) if relu else zr, rtol=rt, atol=at)
    # Backward oracle through OUR ReLU mask: at z ~ 0 the two roundings of z may disagree on
    # the sign, which flips one gradient element between pass-through and zero (a tie, not
    # an error).
    yr = zr * (y.detach() > 0).float() if relu else zr
    torch.testing.assert_close(bn.running_mean, ref_rm, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(bn.running_var, ref_rv, rtol=1e-4, atol=1e-5)
    assert bn.num_batches_tracked.item() == 1
    gy = _mk(shape, dtype, cuda, 3)
    y.backward(gy)
    # reference backward through the same (rounded) output mask
    yr.backward(gy.float())
    # ...and the backward recomputes the mask as fma(x, a, b) > 0 in fp32 (ops/bn.py), which can
    # still disagree with the rounded y at |z| ~ 0 (e.g. a positive z that rounds to +0): those
    # elements' own gradients are a tie, not compared (their effect on the sums is negligible)
    keep = zr.detach().abs() > 1e-2 if relu else torch.ones_like(zr, dtype=torch.bool)
    torch.testing.assert_close(x.grad.float()[keep], xr.grad[keep], rtol=rt * 4, atol=at * 4)
    torch.testing.assert_close(bn.weight.grad, w.grad, rtol=rt * 4, atol=at * 20 * (shape[0] * shape[2] * shape[3]) ** 0.5)
    torch.testing.assert_close(bn.bias.grad, b.grad, rtol=rt * 4, atol=at * 20 * (shape[0] * shape[2] * shape[3]) ** 0.5)
    if res:
        torch.testing.assert_close(r.grad.float(), rr.grad, rtol=rt, atol=at)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_fused_bn_eval(cuda, dtype):
    bn = FusedBatchNorm2d(128).to(cuda).eval()
    with torch.no_grad():
        bn.running_mean.uniform_(-1, 1)
        bn.running_var.uniform_(0.5, 2)
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    x = _mk((4, 128, 5, 5), dtype, cuda, 4)
    r = _mk((4, 128, 5, 5), dtype, cuda, 5)
    with torch.no_grad():
        y = bn_act(bn, x, relu=True, residual=r)
        yr = reference_bn_act(x.float(), r.float(), bn.weight, bn.bias, bn.running_mean, bn.running_var,
                              False, 0.1, bn.eps, True)
    rt, at = TOL[dtype]
    torch.testing.assert_close(y.float(), yr, rtol=rt, atol=at)


def test_fused_bn_large_batch_statistics(cuda):
    """ResNet-50 stem-sized reduction (M = 64*112*112): fp64 finalize keeps the variance exact."""
    x = (torch.randn(64, 64, 112, 112, device=cuda) * 0.05 + 3.0).to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    bn = FusedBatchNorm2d(64).to(cuda)
    y = bn_act(bn, x, relu=False)
    xf = x.float()
    mean = xf.mean(dim=(0, 2, 3))
    var = xf.var(dim=(0, 2, 3), unbiased=True)
    torch.testing.assert_close(bn.running_mean, 0.1 * mean, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(bn.running_var, 0.9 + 0.1 * var, rtol=1e-4, atol=1e-6)
    yf = y.float()
    assert abs(yf.mean().item()) < 2e-2 and abs(yf.std().item() - 1) < 2e-2


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("batch,size", [(32, 64), (8, 64)])
def test_resnet_fused_matches_unfused(cuda, batch, size):
    """Whole network against an fp64 reference: the fused network's error (forward output and
    every parameter gradient) must be of the same order as the stock MIOpen network's error.
    (Small-batch BN backward is ill-conditioned, so fp32-vs-fp32 differences alone say little.)"""
    import copy

    from distributed_pytorch_training_amd.models import build_model
    from distributed_pytorch_training_amd.models.layers import fuse_native_layers

    torch.manual_seed(0)
    ref = build_model("resnet50", 100, cuda, image_size=size, channels_last=True)
    fused = copy.deepcopy(ref)
    f64 = copy.deepcopy(ref).double()
    assert fuse_native_layers(fused) == 55  # 53 BN + stem max-pool + global avg-pool
    x = torch.randn(batch, 3, size, size, device=cuda).contiguous(memory_format=torch.channels_last)
    torch.backends.cudnn.deterministic = True
    outs = []
    for m, xx in ((f64, x.double()), (ref, x), (fused, x)):
        y = m(xx)
        y = y[0] if isinstance(y, tuple) else y
        y.sum().backward()
        outs.append(y)
    e_ref, e_fused = _rel(outs[1], outs[0]), _rel(outs[2], outs[0])
    assert e_fused < max(3 * e_ref, 1e-5), (e_fused, e_ref)
    gr = [_rel(p.grad, q.grad) for p, q in zip(ref.parameters(), f64.parameters())]
    gf = [_rel(p.grad, q.grad) for p, q in zip(fused.parameters(), f64.parameters())]
    med = lambda v: sorted(v)[len(v) // 2]
    assert med(gf) < max(3 * med(gr), 1e-4), (med(gf), med(gr))
    assert max(gf) < max(3 * max(gr), 1e-3), (max(gf), max(gr))
    with torch.autocast("cuda", dtype=torch.bfloat16):
        a16 = ref(x)
        b16 = fused(x)
    b16 = b16[0] if isinstance(b16, tuple) else b16
    err_unfused, err_fused = _rel(a16, outs[0]), _rel(b16, outs[0])
    assert err_fused < max(3 * err_unfused, 0.05), (err_fused, err_unfused)


@pytest.mark.parametrize("use", ["both", "first", "second"])
def test_pair_outputs_sum_gradients(cuda, use):
    """Block-tail op with two aliased outputs: gradients of both consumers are summed in-kernel."""
    from distributed_pytorch_training_amd.models.layers import bn_act_block_out

    shape = (8, 256, 7, 7)
    x = _mk(shape, torch.bfloat16, cuda, 11).requires_grad_()
    r = _mk(shape, torch.bfloat16, cuda, 12).requires_grad_()
    bn = FusedBatchNorm2d(256).to(cuda)
    xr, rr = x.detach().float().requires_grad_(), r.detach().float().requires_grad_()
    w = bn.weight.detach().clone().requires_grad_()
    b = bn.bias.detach().clone().requires_grad_()
    y1, y2 = bn_act_block_out(bn, x, r)
    assert y1.data_ptr() == y2.data_ptr()
    g1, g2 = _mk(shape, torch.bfloat16, cuda, 13), _mk(shape, torch.bfloat16, cuda, 14)
    loss = 0
    if use in ("both", "first"):
        loss = loss + (y1.float() * g1.float()).sum()
    if use in ("both", "second"):
        loss = loss + (y2.float() * g2.float()).sum()
    loss.backward()
    zr = reference_bn_act(xr, rr, w, b, bn.running_mean.clone(), bn.running_var.clone(), True, 0.1, bn.eps, False)
    yr = zr * (y1.detach() > 0).float()
    gsum = (g1.float() if use != "second" else 0) + (g2.float() if use != "first" else 0)
    (yr * gsum).sum().backward()
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=8e-2, atol=8e-2)
    torch.testing.assert_close(r.grad.float(), rr.grad, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(bn.bias.grad, b.grad, rtol=2e-2, atol=0.5)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("shape,k,s,p", [((8, 64, 112, 112), 3, 2, 1), ((2, 16, 9, 7), 3, 2, 1),
                                         ((2, 16, 10, 11), 3, 2, 1), ((3, 8, 5, 6), 3, 2, 1), ((1, 8, 1, 2), 3, 2, 1),
                                         ((2, 8, 8, 8), 2, 2, 0), ((3, 24, 10, 10), 3, 1, 1)])
def test_maxpool_matches_torch(cuda, dtype, shape, k, s, p):
    from distributed_pytorch_training_amd.ops.pool import max_pool2d_nhwc

    x = _mk(shape, dtype, cuda, 21)
    x[0, :, 0, 0] = x[0, :, 0, 1]          # ties: first max wins in both
    xa = x.detach().clone().requires_grad_()
    xb = x.detach().clone().requires_grad_()
    ya = max_pool2d_nhwc(xa, k, s, p)
    yb = torch.nn.functional.max_pool2d(xb, k, s, p)
    assert torch.equal(ya, yb)
    g = _mk(tuple(ya.shape), dtype, cuda, 22)
    ya.backward(g)
    yb.backward(g)
    rt, at = TOL[dtype]
    torch.testing.assert_close(xa.grad.float(), xb.grad.float(), rtol=rt, atol=at)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("k,s,p", [(3, 2, 1), (3, 1, 1)])
def test_maxpool_nan_and_neg_inf(cuda, dtype, k, s, p):
    """NaN propagates (torch's max_pool2d returns NaN for a window holding one, and routes the
    gradient to it); -inf only wins an all--inf window.  Planted at the first tap of padded
    windows (row/col 0), mid-image, and in a window whose other taps are -inf.  Reference: torch's
    NCHW kernel (the reference's layout): an all--inf window routes its gradient to the first
    in-image tap there (torch's NHWC kernel sends it to flat index 0 of the image instead)."""
    from distributed_pytorch_training_amd.ops.pool import max_pool2d_nhwc

    x = _mk((2, 16, 11, 10), dtype, cuda, 51)
    x[0, 0, 0, 0] = float("nan")            # first tap of the top-left (padded) window
    x[0, 3, 5, 4] = float("nan")            # interior
    x[1, 2, 0, 3] = float("nan")            # top border
    x[1, 5, 4:7, 4:7] = float("-inf")       # a whole 3x3 block of -inf ...
    x[1, 6, 4:7, 4:7] = float("-inf")
    x[1, 6, 5, 5] = float("nan")            # ... with a NaN in the middle
    x[0, 7, :, :] = float("-inf")           # an all--inf channel
    x = x.contiguous(memory_format=torch.channels_last)
    xa = x.detach().clone().requires_grad_()
    xb = x.detach().contiguous().requires_grad_()          # NCHW
    ya = max_pool2d_nhwc(xa, k, s, p)
    yb = torch.nn.functional.max_pool2d(xb, k, s, p)
    assert torch.equal(torch.isnan(ya), torch.isnan(yb))
    m = ~torch.isnan(yb)
    assert torch.equal(ya[m], yb[m])
    g = _mk(tuple(ya.shape), dtype, cuda, 52)
    ya.backward(g)
    yb.backward(g)
    rt, at = TOL[dtype]
    torch.testing.assert_close(xa.grad.float(), xb.grad.float(), rtol=rt, atol=at, equal_nan=True)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_maxpool_pair_sums_both_gradients(cuda, dtype):
    """Stem-pool pair outputs: the backward gather sums the conv-path and identity-path
    gradients (ops/pool.py _MaxPoolNHWCPair) - equal to torch's pool with the summed grad."""
    from distributed_pytorch_training_amd.ops.pool import max_pool2d_nhwc

    x = _mk((4, 64, 56, 56), dtype, cuda, 31)
    xa = x.detach().clone().requires_grad_()
    xb = x.detach().clone().requires_grad_()
    y1, y2 = max_pool2d_nhwc(xa, 3, 2, 1, pair=True)
    yb = torch.nn.functional.max_pool2d(xb, 3, 2, 1)
    assert torch.equal(y1, yb) and torch.equal(y2, yb)
    g1 = _mk(tuple(yb.shape), dtype, cuda, 32)
    g2 = _mk(tuple(yb.shape), dtype, cuda, 33)
    torch.autograd.backward([y1, y2], [g1, g2])
    yb.backward(g1.float().add(g2.float()).to(dtype))
    rt, at = TOL[dtype]
    torch.testing.assert_close(xa.grad.float(), xb.grad.float(), rtol=rt, atol=2 * at)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_global_avg_pool_backward(cuda, dtype):
    from distributed_pytorch_training_amd.ops.pool import global_avg_pool_nhwc

    x = _mk((5, 2048, 7, 7), dtype, cuda, 41)
    xa = x.detach().clone().requires_grad_()
    xb = x.detach().clone().requires_grad_()
    ya = global_avg_pool_nhwc(xa)
    yb = torch.nn.functional.adaptive_avg_pool2d(xb, 1)
    assert torch.equal(ya, yb)
    g = _mk(tuple(yb.shape), dtype, cuda, 42)
    ya.backward(g)
    yb.backward(g)
    assert xa.grad.is_contiguous(memory_format=torch.channels_last)
    rt, at = TOL[dtype]
    torch.testing.assert_close(xa.grad.float(), xb.grad.float(), rtol=rt, atol=at)


def test_stem_bn_statistics_from_pool_backward(cuda):
    """ResNet stem: BN+ReLU -> 3x3/2 max-pool (pair outputs).  The pool's backward gather also
    sums the BN's backward statistics (pool_kernels.hip BNS); gradients must equal the BN's own
    statistics pass."""
    from distributed_pytorch_training_amd.ops import bn as fbn
    from distributed_pytorch_training_amd.ops import conv as nc
    from distributed_pytorch_training_amd.ops.pool import max_pool2d_nhwc

    x0 = _mk((4, 64, 30, 30), torch.bfloat16, cuda, 51)
    g1 = _mk((4, 64, 15, 15), torch.bfloat16, cuda, 52)
    g2 = _mk((4, 64, 15, 15), torch.bfloat16, cuda, 53)
    w0 = torch.rand(64, device=cuda) + 0.5
    b0 = torch.randn(64, device=cuda) * 0.2
    grads = []
    for fuse in (True, False):
        nc.BN_BWD_FUSE = fuse
        x = x0.detach().clone().requires_grad_(True)
        w, b = w0.clone().requires_grad_(True), b0.clone().requires_grad_(True)
        rm, rv = torch.zeros(64, device=cuda), torch.ones(64, device=cuda)
        nb = torch.zeros((), dtype=torch.long, device=cuda)
        y = fbn.bn_act_train(x, None, w, b, rm, rv, nb, 0.1, 1e-5, True)
        p1, p2 = max_pool2d_nhwc(y, 3, 2, 1, pair=True)
        torch.autograd.backward([p1, p2], [g1, g2])
        grads.append([x.grad.float(), w.grad, b.grad])
    nc.BN_BWD_FUSE = True
    assert not nc._BNB_PARTIALS
    for a, b in zip(*grads):
        torch.testing.assert_close(a, b, rtol=2e-2, atol=2e-2 * b.abs().max().item() + 1e-6)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_stem_bn_relu_maxpool_fused(cuda, dtype, monkeypatch):
    """ResNet stem pool(relu(bn(x))) as one op (BN apply folded into the pool's loads): the
    pooled output is bitwise the unfused chain's, running statistics equal, and gradients match
    (the backward is the same pool-gather statistics + BN apply either way)."""
    import copy

    from distributed_pytorch_training_amd.models import layers

    x0 = _mk((4, 64, 30, 29), dtype, cuda, 61)  # odd pooled extents: partial 2x2 output blocks
    g1 = _mk((4, 64, 15, 15), dtype, cuda, 62)
    g2 = _mk((4, 64, 15, 15), dtype, cuda, 63)
    bn0 = layers.FusedBatchNorm2d(64).to(cuda)
    with torch.no_grad():
        bn0.weight.uniform_(-1.0, 1.5)  # negative scales too: the pool must not assume monotone
        bn0.bias.uniform_(-0.3, 0.3)
    pool = layers.FusedMaxPool2d(3, 2, 1)
    pool.dpt_pair = True
    res = []
    for fuse in (True, False):
        monkeypatch.setattr(layers, "STEM_FUSE", fuse)
        bn = copy.deepcopy(bn0)
        x = x0.detach().clone().requires_grad_(True)
        y1, y2 = layers.bn_relu_maxpool(bn, pool, x)
        torch.autograd.backward([y1, y2], [g1, g2])
        res.append((y1.detach(), x.grad.float(), bn.weight.grad, bn.bias.grad, bn.running_mean, bn.running_var))
    (a, *ra), (b, *rb) = res
    assert torch.equal(a, b)
    for u, v in zip(ra, rb):
        torch.testing.assert_close(u, v, rtol=2e-2, atol=2e-2 * v.abs().max().item() + 1e-6)


def test_finalize_of_tens_of_thousands_of_partials(cuda):
    """The stem's conv epilogue leaves 25,088 partials per channel at batch 256: that finalize runs
    1024-thread blocks (bn_kernels.hip, > 8192 partials); same statistics as the fp32 reference."""
    from distributed_pytorch_training_amd import ops
    C_ = ops.native()
    c, chunks = 64, 10000
    x = (torch.randn(chunks * 8, c, device=cuda) * 0.5 + 2.0).to(torch.bfloat16)
    rows = x.float().view(chunks, 8, c)
    ps = rows.sum(1).t().contiguous()
    pq = (rows ** 2).sum(1).t().contiguous()
    x4 = x.view(chunks * 8, 1, 1, c).permute(0, 3, 1, 2)      # channels_last [M, C, 1, 1]
    w = torch.rand(c, device=cuda) + 0.5
    b = torch.rand(c, device=cuda) - 0.5
    rm, rv = torch.zeros(c, device=cuda), torch.ones(c, device=cuda)
    nb = torch.zeros((), dtype=torch.long, device=cuda)
    y, mean, invstd, _ = C_.bn_fwd_train(x4, None, w, b, rm, rv, nb, 0.1, 1e-5, False, ps, pq)
    xf = x.float()
    torch.testing.assert_close(mean, xf.mean(0), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(invstd, torch.rsqrt(xf.var(0, unbiased=False) + 1e-5), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(rv, 0.9 + 0.1 * xf.var(0, unbiased=True), rtol=1e-4, atol=1e-5)
    zr = (xf - xf.mean(0)) * torch.rsqrt(xf.var(0, unbiased=False) + 1e-5) * w + b
    torch.testing.assert_close(y.permute(0, 2, 3, 1).reshape(-1, c).float(), zr, rtol=2e-2, atol=2e-2)
    assert int(nb) == 1
