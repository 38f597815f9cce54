"""BatchNorm finalize run inside the apply launch (csrc/kernels/handoff.h) vs its own launch.

The fused launch runs the very same finalize and apply code, only the hand-off differs
(write-through granules carrying tag and value), so every output must be BITWISE equal to
the two-launch path - and both must match the fp32 PyTorch reference of the op.  Covered: every
entry point that runs a finalize (forward with and without conv-epilogue partials, half-wave and
wide finalize, the two-BatchNorm block tail, the three backward forms), many launches in one step
(granule arena exhausted: the rest run unfused), hipGraph capture + replay of the per-step
zeroing, and a concurrent load on a second stream (uneven scheduling).
A bounded spin that ever timed out would show in ``bn_handoff_errors()``.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _C():
    from distributed_pytorch_training_amd import ops
    return ops.native()


@pytest.fixture(autouse=True)
def _fusion_on(cuda):
    was = _C().bn_fuse_finalize_enabled()
    _C().bn_set_fuse_finalize(1)
    yield
    _C().bn_set_fuse_finalize(was)


def _act(n, c, h, w, dtype, dev, seed, scale=1.0, shift=0.0):
    g = torch.Generator(device=dev).manual_seed(seed)
    t = torch.randn((n, c, h, w), device=dev, generator=g) * scale + shift
    return t.to(dtype).contiguous(memory_format=torch.channels_last)


def _partials(x, chunks):
    """[C][chunks] fp32 (sum, sum of squares) over row chunks of the [M, C] view (any split works)."""
    c = x.shape[1]
    rows = x.permute(0, 2, 3, 1).reshape(-1, c).float()
    m = rows.shape[0]
    bounds = torch.linspace(0, m, chunks + 1).round().long().tolist()
    ps = torch.stack([rows[a:b].sum(0) for a, b in zip(bounds, bounds[1:])], 1).contiguous()
    pq = torch.stack([(rows[a:b] ** 2).sum(0) for a, b in zip(bounds, bounds[1:])], 1).contiguous()
    return ps, pq


def _bn_params(c, dev, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    w = torch.rand(c, device=dev, generator=g) + 0.5
    b = torch.rand(c, device=dev, generator=g) - 0.5
    rm = torch.rand(c, device=dev, generator=g) * 0.2 - 0.1
    rv = torch.rand(c, device=dev, generator=g) + 0.5
    nb = torch.zeros((), dtype=torch.long, device=dev)
    return w, b, rm, rv, nb


def _both(fn, min_fused=1):
    """fn() with the finalize in its own launch, then fused (inside a step: bn_handoff_begin);
    returns (unfused, fused) outputs."""
    C = _C()
    try:
        C.bn_set_fuse_finalize(0)
        a = fn()
        C.bn_set_fuse_finalize(1)
        C.bn_handoff_begin()
        n0 = C.bn_handoff_fused_launches()
        b = fn()
        assert C.bn_handoff_fused_launches() - n0 >= min_fused, "the fused path did not run"
    finally:
        C.bn_set_fuse_finalize(1)   # the fixture restores the process default afterwards
    torch.cuda.synchronize()
    return a, b


def _same(a, b):
    for u, v in zip(a, b):
        if isinstance(u, torch.Tensor) and u.numel():
            assert torch.equal(u, v), (u.flatten()[:8], v.flatten()[:8])


SHAPES = [(4, 64, 14, 14, 16), (4, 64, 14, 14, 300), (8, 256, 7, 7, 24), (2, 2048, 7, 7, 4), (16, 512, 7, 7, 400),
          (2, 8, 3, 3, 1)]


@pytest.mark.parametrize("n,c,h,w,chunks", SHAPES)
@pytest.mark.parametrize("relu,res", [(True, False), (True, True), (False, False)])
def test_forward_from_partials_fused_equals_two_launches(cuda, n, c, h, w, chunks, relu, res):
    C = _C()
    dt = torch.bfloat16
    x = _act(n, c, h, w, dt, cuda, 1, 1.7, 0.3)
    r = _act(n, c, h, w, dt, cuda, 2) if res else None
    ps, pq = _partials(x, chunks)
    wt, b, rm0, rv0, _ = _bn_params(c, cuda, 3)

    def run():
        rm, rv = rm0.clone(), rv0.clone()
        nb = torch.zeros((), dtype=torch.long, device=cuda)
        y, mean, invstd, coef = C.bn_fwd_train(x, r, wt, b, rm, rv, nb, 0.1, 1e-5, relu, ps, pq)
        return y, mean, invstd, coef, rm, rv, nb

    u, f = _both(run)
    _same(u, f)
    assert int(f[6]) == 1
    # and against the fp32 reference of the op
    xf = x.float()
    mean = xf.mean((0, 2, 3))
    var = xf.var((0, 2, 3), unbiased=False)
    z = (xf - mean[None, :, None, None]) * torch.rsqrt(var + 1e-5)[None, :, None, None] * wt[None, :, None, None] \
        + b[None, :, None, None]
    if res:
        z = z + r.float()
    if relu:
        z = torch.relu(z)
    torch.testing.assert_close(f[0].float(), z, rtol=2e-2, atol=3e-2)
    torch.testing.assert_close(f[4], 0.9 * rm0 + 0.1 * mean, rtol=1e-4, atol=1e-5)
    assert C.bn_handoff_errors() == 0


@pytest.mark.parametrize("n,c,h,w", [(4, 64, 14, 14), (2, 2048, 7, 7), (16, 256, 8, 8)])
def test_forward_own_statistics_fused_equals_two_launches(cuda, n, c, h, w):
    C = _C()
    x = _act(n, c, h, w, torch.bfloat16, cuda, 4, 2.0, -0.5)
    wt, b, rm0, rv0, _ = _bn_params(c, cuda, 5)

    def run():
        rm, rv = rm0.clone(), rv0.clone()
        nb = torch.zeros((), dtype=torch.long, device=cuda)
        return (*C.bn_fwd_train(x, None, wt, b, rm, rv, nb, 0.1, 1e-5, True), rm, rv, nb)

    u, f = _both(run)
    _same(u, f)
    assert C.bn_handoff_errors() == 0


@pytest.mark.parametrize("n,c,h,w,chunks", [(4, 256, 14, 14, 40), (4, 256, 28, 28, 392), (2, 2048, 7, 7, 2)])
def test_block_tail_two_batchnorms_one_launch(cuda, n, c, h, w, chunks):
    """bn2_fwd_train (both finalizes + apply in one launch) == two finalizes + bn_apply_aff == fp32."""
    C = _C()
    x = _act(n, c, h, w, torch.bfloat16, cuda, 6, 1.3, 0.2)
    x2 = _act(n, c, h, w, torch.bfloat16, cuda, 7, 0.8, -0.1)
    ps, pq = _partials(x, chunks)
    ps2, pq2 = _partials(x2, max(1, chunks // 2))
    p1 = _bn_params(c, cuda, 8)
    p2 = _bn_params(c, cuda, 9)

    def fresh(p):
        return p[0], p[1], p[2].clone(), p[3].clone(), p[4].clone()

    def fused():
        a, b_ = fresh(p1), fresh(p2)
        out = C.bn2_fwd_train(x, x2, *a, 0.1, 1e-5, *b_, 0.05, 2e-5, ps, pq, ps2, pq2)
        return (*out, a[2], a[3], b_[2], b_[3], a[4], b_[4])

    def two_ops():
        a, b_ = fresh(p1), fresh(p2)
        _, m, i, cf = C.bn_fwd_train(x, None, *a, 0.1, 1e-5, True, ps, pq, False)
        _, m2, i2, cf2 = C.bn_fwd_train(x2, None, *b_, 0.05, 2e-5, False, ps2, pq2, False)
        y = C.bn_apply_aff(x, x2, cf, cf2)
        return (y, m, i, cf, m2, i2, cf2, a[2], a[3], b_[2], b_[3], a[4], b_[4])

    C.bn_set_fuse_finalize(0)
    try:
        ref2 = fused()        # bn2_fwd_train with the finalizes as their own launches
    finally:
        C.bn_set_fuse_finalize(1)
    C.bn_handoff_begin()
    n0 = C.bn_handoff_fused_launches()
    f = fused()
    assert C.bn_handoff_fused_launches() == n0 + 1
    o = two_ops()
    torch.cuda.synchronize()
    _same(ref2, f)
    _same(o, f)
    assert int(f[11]) == 1 and int(f[12]) == 1

    def bn_ref(t, p, eps):
        tf = t.float()
        mu = tf.mean((0, 2, 3))
        var = tf.var((0, 2, 3), unbiased=False)
        return (tf - mu[None, :, None, None]) * torch.rsqrt(var + eps)[None, :, None, None] * p[0][None, :, None, None] \
            + p[1][None, :, None, None]

    z = torch.relu(bn_ref(x, p1, 1e-5) + bn_ref(x2, p2, 2e-5))
    torch.testing.assert_close(f[0].float(), z, rtol=2e-2, atol=4e-2)
    assert C.bn_handoff_errors() == 0


@pytest.mark.parametrize("n,c,h,w,chunks", [(4, 64, 14, 14, 20), (4, 64, 28, 28, 400), (2, 2048, 7, 7, 3)])
@pytest.mark.parametrize("from_dz", [False, True])
def test_backward_from_partials_fused_equals_two_launches(cuda, n, c, h, w, chunks, from_dz):
    C = _C()
    dt = torch.bfloat16
    x = _act(n, c, h, w, dt, cuda, 10, 1.5, 0.2)
    dy = _act(n, c, h, w, dt, cuda, 11)
    wt, b, rm, rv, nb = _bn_params(c, cuda, 12)
    _, mean, invstd, coef = C.bn_fwd_train(x, None, wt, b, rm, rv, nb, 0.1, 1e-5, True)
    # the statistics partials a dgrad epilogue would write: s1 = sum dz, s2 = sum dz*(x - mean)
    xf, g = x.float(), dy.float()
    if not from_dz:
        mask = (xf * coef[:c][None, :, None, None] + coef[c:][None, :, None, None]) > 0
        g = g * mask
    rows = lambda t: t.permute(0, 2, 3, 1).reshape(-1, c)
    p1, _ = _partials(g, chunks)
    p2, _ = _partials(g * (xf - mean[None, :, None, None]), chunks)

    def run():
        return C.bn_bwd_partials(dy, x, wt, mean, invstd, coef, p1, p2, True, from_dz)

    u, f = _both(run)
    _same(u, f)
    # fp32 reference: dx = k1*dz + k2*(x - mean) + k3
    m = rows(xf).shape[0]
    s1, s2 = rows(g).sum(0), rows(g * (xf - mean[None, :, None, None])).sum(0)
    k1 = wt * invstd
    ref = k1[None, :, None, None] * g - (k1 * invstd ** 2 * s2 / m)[None, :, None, None] * \
        (xf - mean[None, :, None, None]) - (k1 * s1 / m)[None, :, None, None]
    torch.testing.assert_close(f[0].float(), ref, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(f[1], s2 * invstd, rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(f[2], s1, rtol=1e-3, atol=1e-3)
    assert C.bn_handoff_errors() == 0


@pytest.mark.parametrize("n,c,h,w", [(4, 64, 14, 14), (2, 1024, 7, 7)])
@pytest.mark.parametrize("relu,two", [(True, False), (True, True), (False, False)])
def test_backward_own_statistics_fused_equals_two_launches(cuda, n, c, h, w, relu, two):
    C = _C()
    dt = torch.bfloat16
    x = _act(n, c, h, w, dt, cuda, 13, 1.2)
    dy = _act(n, c, h, w, dt, cuda, 14)
    dy2 = _act(n, c, h, w, dt, cuda, 15) if two else None
    wt, b, rm, rv, nb = _bn_params(c, cuda, 16)
    y, mean, invstd, coef = C.bn_fwd_train(x, None, wt, b, rm, rv, nb, 0.1, 1e-5, relu)

    def run():
        return C.bn_bwd(dy, dy2, y, x, wt, mean, invstd, relu, two, True, None if two else coef)

    u, f = _both(run)
    _same(u, f)
    assert C.bn_handoff_errors() == 0


@pytest.mark.parametrize("n,c,h,w,chunks", [(4, 256, 14, 14, 30), (4, 256, 28, 28, 300)])
def test_backward_block_tail_two_batchnorms_fused_equals_two_launches(cuda, n, c, h, w, chunks):
    C = _C()
    dt = torch.bfloat16
    dz = _act(n, c, h, w, dt, cuda, 17)
    x = _act(n, c, h, w, dt, cuda, 18, 1.1)
    x2 = _act(n, c, h, w, dt, cuda, 19, 0.9)
    w1, b1, rm, rv, nb = _bn_params(c, cuda, 20)
    w2, b2, rm2, rv2, nb2 = _bn_params(c, cuda, 21)
    _, mean, invstd, _ = C.bn_fwd_train(x, None, w1, b1, rm, rv, nb, 0.1, 1e-5, False)
    _, mean2, invstd2, _ = C.bn_fwd_train(x2, None, w2, b2, rm2, rv2, nb2, 0.1, 1e-5, False)
    g = dz.float()
    p1, _ = _partials(g, chunks)
    p2, _ = _partials(g * (x.float() - mean[None, :, None, None]), chunks)
    p3, _ = _partials(g * (x2.float() - mean2[None, :, None, None]), chunks)

    def run():
        return C.bn2_bwd_partials(dz, x, x2, w1, w2, mean, invstd, mean2, invstd2, p1, p2, p3, True)

    u, f = _both(run)
    _same(u, f)
    assert C.bn_handoff_errors() == 0


def test_many_launches_in_one_step_and_across_steps(cuda):
    """One step draws granule ranges until the arena is exhausted (the rest run unfused); the next
    steps zero what the previous one drew and fuse again - every output identical throughout."""
    C = _C()
    x = _act(4, 2048, 7, 7, torch.bfloat16, cuda, 22)
    ps, pq = _partials(x, 4)
    wt, b, rm, rv, nb = _bn_params(2048, cuda, 23)
    y0 = C.bn_fwd_train(x, None, wt, b, None, None, None, 0.1, 1e-5, True, ps, pq)[0]
    for step in range(3):
        C.bn_handoff_begin()
        n0 = C.bn_handoff_fused_launches()
        for _ in range(300):   # 300 x 4096 granules > the 1M-granule arena
            y = C.bn_fwd_train(x, None, wt, b, None, None, None, 0.1, 1e-5, True, ps, pq)[0]
            assert torch.equal(y, y0)
        fused = C.bn_handoff_fused_launches() - n0
        assert 0 < fused < 300, fused
    torch.cuda.synchronize()
    assert C.bn_handoff_errors() == 0


def test_fused_finalize_under_graph_replay_and_concurrent_load(cuda):
    """Captured fused launches replay correctly (the slot they captured is reset by each launch)
    while a second stream streams a large copy (uneven block scheduling)."""
    C = _C()
    dt = torch.bfloat16
    x = _act(8, 256, 14, 14, dt, cuda, 24, 1.4, 0.1)
    r = _act(8, 256, 14, 14, dt, cuda, 25)
    ps, pq = _partials(x, 100)
    wt, b, rm, rv, nb = _bn_params(256, cuda, 26)
    # eager once (allocates the slot pool outside capture), then the reference values
    y_ref = C.bn_fwd_train(x, r, wt, b, None, None, None, 0.1, 1e-5, True, ps, pq)[0]
    dy = _act(8, 256, 14, 14, dt, cuda, 27)
    _, mean, invstd, coef = C.bn_fwd_train(x, None, wt, b, None, None, None, 0.1, 1e-5, True, ps, pq)
    dx_ref = C.bn_bwd(dy, None, None, x, wt, mean, invstd, True, False, True, coef)[0]
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()

    def step():
        C.bn_handoff_begin()
        y = C.bn_fwd_train(x, r, wt, b, None, None, None, 0.1, 1e-5, True, ps, pq)[0]
        dx = C.bn_bwd(dy, None, None, x, wt, mean, invstd, True, False, True, coef)[0]
        return y, dx

    with torch.cuda.stream(s):
        for _ in range(2):  # warm up on the capture stream (the arena follows it there)
            step()
        n0 = C.bn_handoff_fused_launches()
        with torch.cuda.graph(g, stream=s):
            y, dx = step()
        assert C.bn_handoff_fused_launches() == n0 + 2, "the captured step is not fused"
    torch.cuda.current_stream().wait_stream(s)
    big = torch.empty(64 << 20, dtype=torch.float32, device=cuda)
    other = torch.cuda.Stream()
    for k in range(20):
        if k % 2:
            with torch.cuda.stream(other):
                big.mul_(1.0001)
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(y, y_ref), k
        assert torch.equal(dx, dx_ref), k
    assert C.bn_handoff_errors() == 0


@pytest.mark.parametrize("n,c,h,w,chunks", [(4, 64, 7, 7, 8), (2, 128, 7, 7, 300), (2, 1024, 3, 3, 2)])
def test_waiting_blocks_finish_the_finalize_themselves(cuda, n, c, h, w, chunks):
    """Correctness may not rest on dispatch order: with the finalize blocks forced idle
    (bn_set_handoff_idle_finalizers), every apply block times out, runs the finalize items itself
    and the outputs are still bitwise those of the two-launch path - with the running statistics
    and num_batches_tracked updated exactly once (the claim words)."""
    C = _C()
    dt = torch.bfloat16
    x = _act(n, c, h, w, dt, cuda, 30, 1.3, 0.4)
    x2 = _act(n, c, h, w, dt, cuda, 31, 0.7)
    dy = _act(n, c, h, w, dt, cuda, 32)
    ps, pq = _partials(x, chunks)
    ps2, pq2 = _partials(x2, chunks)
    wt, b, rm0, rv0, _ = _bn_params(c, cuda, 33)

    def fwd():
        rm, rv = rm0.clone(), rv0.clone()
        nb = torch.zeros((), dtype=torch.long, device=cuda)
        rm2, rv2 = rm0.clone(), rv0.clone()
        nb2 = torch.zeros((), dtype=torch.long, device=cuda)
        o1 = C.bn_fwd_train(x, x2, wt, b, rm, rv, nb, 0.1, 1e-5, True, ps, pq)
        o2 = C.bn2_fwd_train(x, x2, wt, b, rm2, rv2, nb2, 0.1, 1e-5, wt, b, None, None, None, 0.1, 1e-5,
                             ps, pq, ps2, pq2)
        return (*o1, rm, rv, nb, *o2, rm2, rv2, nb2)

    _, mean, invstd, coef = C.bn_fwd_train(x, None, wt, b, None, None, None, 0.1, 1e-5, True)
    xf, g = x.float(), dy.float()
    mask = (xf * coef[:c][None, :, None, None] + coef[c:][None, :, None, None]) > 0
    p1, _ = _partials(g * mask, chunks)
    p2, _ = _partials(g * mask * (xf - mean[None, :, None, None]), chunks)
    p3, _ = _partials(g * (x2.float() - mean[None, :, None, None]), chunks)

    def bwd():
        return (*C.bn_bwd_partials(dy, x, wt, mean, invstd, coef, p1, p2, True, False),
                *C.bn2_bwd_partials(dy, x, x2, wt, wt, mean, invstd, mean, invstd, p1, p2, p3, True))

    C.bn_set_handoff_idle_finalizers(1)
    try:
        uf, ff = _both(fwd, min_fused=2)
        ub, fb = _both(bwd, min_fused=2)
    finally:
        C.bn_set_handoff_idle_finalizers(0)
    _same(uf, ff)
    _same(ub, fb)
    assert int(ff[6]) == 1 and int(ff[16]) == 1   # num_batches_tracked: exactly once
    assert C.bn_handoff_errors() == 0
