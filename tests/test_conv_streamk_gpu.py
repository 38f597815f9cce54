"""Stream-K conv_fwd_kernel grids (csrc/kernels/conv_kernels.hip, ``conv_set_streamk``): the
(tile, K-step) iterations of a conv spread evenly over 256 x k blocks, a tile cut between blocks
finished by the block holding its last K-step from the others' fp32 partials.

Checked against the data-parallel grid (same kernel, one block per tile) and an fp32 reference:
forward with BN statistics, backward-data with the BN statistics epilogue, ragged grids (tile
counts not a multiple of 8, partial last M-tile, 64-wide N tiles), bitwise run-to-run
determinism, hipGraph replay (the publish flags are reset by their consumers, so every replay
starts from zeros), and a zero give-up count of the bounded spin."""
import pytest
import torch
import torch.nn.functional as F

from distributed_pytorch_training_amd import ops

pytestmark = pytest.mark.gpu
CL = torch.channels_last

# (N, C, H, W, Cout, k, stride, pad): tiles = ceil(N*Ho*Wo / 128) * Cout / BN
SHAPES = [
    (256, 1024, 14, 14, 256, 1, 1, 0),   # ResNet-50 layer3 1x1 reduce: 784 tiles, 16 K-steps
    (128, 512, 28, 28, 128, 1, 1, 0),    # layer2 1x1 reduce at batch 128: 784 tiles, 8 K-steps
    (64, 256, 28, 28, 192, 1, 1, 0),     # 64-wide N tiles: 392 x 3 tiles
    (48, 64, 40, 20, 128, 3, 1, 0),      # 3x3 without padding (per-tap loop): 257 tiles, ragged M
    (128, 512, 28, 28, 512, 1, 2, 0),    # stride-2 1x1 downsample: 196 x 4 tiles, 8 K-steps
]


def _operands(cuda, N, C, H, W, Cout, k, seed=0):
    g = torch.Generator(device=cuda).manual_seed(seed)
    x = torch.randn(N, C, H, W, device=cuda, generator=g).to(torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(Cout, C, k, k, device=cuda, generator=g) / (C * k * k) ** 0.5).to(torch.bfloat16)
    return x, w.contiguous(memory_format=CL)


def _run(C_, mode, fn):
    C_.conv_set_streamk(mode)
    try:
        out = fn()
        torch.cuda.synchronize()
        return out
    finally:
        C_.conv_set_streamk(0)


def _bf16_close(a, b, frac=1e-3):
    """Same products summed in another order: within one bf16 rounding step, almost everywhere."""
    a, b = a.float(), b.float()
    tol = 2 ** -7 * b.abs() + 1e-3
    bad = ((a - b).abs() > tol).float().mean().item()
    assert bad <= frac, bad


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_streamk_forward_matches_data_parallel_grid(cuda, shape):
    N, C, H, W, Cout, k, st, pad = shape
    C_ = ops.native()
    x, w = _operands(cuda, N, C, H, W, Cout, k, seed=sum(shape))
    Ho, Wo = (H + 2 * pad - k) // st + 1, (W + 2 * pad - k) // st + 1
    M = N * Ho * Wo
    bn = 128 if Cout % 128 == 0 else 64
    tiles = -(-M // 128) * (Cout // bn)
    G = C_.conv_sk_blocks(tiles, k * k * C // 64, bn, 2)
    assert G > 0, (tiles, G)   # every shape here is eligible when forced
    e0 = C_.conv_sk_errors()
    dp = _run(C_, 0, lambda: C_.conv_fwd(x, w, st, pad, True))
    sk = _run(C_, 2, lambda: C_.conv_fwd(x, w, st, pad, True))
    sk2 = _run(C_, 2, lambda: C_.conv_fwd(x, w, st, pad, True))
    assert C_.conv_sk_errors() == e0
    y0, s0, q0 = dp[0], dp[1], dp[2]
    y1, s1, q1 = sk[0], sk[1], sk[2]
    assert y1.shape == y0.shape and y1.is_contiguous(memory_format=CL)
    for a, b in zip(sk, sk2):       # deterministic for a given grid
        assert torch.equal(a, b)
    _bf16_close(y1, y0)
    ref = F.conv2d(x.float(), w.float(), stride=st, padding=pad)
    torch.testing.assert_close(y1.float(), ref, rtol=1e-2, atol=2e-2)
    # BN sums over M outputs that differ by single bf16 roundings: ~sqrt(M) x 2^-8 apart
    tol = 2 ** -8 * M ** 0.5
    torch.testing.assert_close(s1.sum(-1), s0.sum(-1), rtol=1e-3, atol=tol)
    torch.testing.assert_close(q1.sum(-1), q0.sum(-1), rtol=1e-3, atol=tol)


def test_streamk_dgrad_bnstats_matches_data_parallel_grid(cuda):
    """1x1 backward-data (the forward kernel on dy and the transposed weight) with the BN
    statistics epilogue, at ResNet-50 layer3 shape (784 tiles)."""
    N, C, H, W, Cout = 256, 256, 14, 14, 1024
    C_ = ops.native()
    g = torch.Generator(device=cuda).manual_seed(5)
    w = (torch.randn(Cout, C, 1, 1, device=cuda, generator=g) / C ** 0.5).to(torch.bfloat16)
    w = w.contiguous(memory_format=CL)
    gy = torch.randn(N, Cout, H, W, device=cuda, generator=g).to(torch.bfloat16).contiguous(memory_format=CL)
    bn_x = torch.randn(N, C, H, W, device=cuda, generator=g).to(torch.bfloat16).contiguous(memory_format=CL)
    bn_mean = torch.randn(C, device=cuda, generator=g)
    bn_coef = torch.randn(2 * C, device=cuda, generator=g)
    dp = _run(C_, 0, lambda: C_.conv_dgrad_bnstats(gy, w, 0, bn_x, bn_mean, bn_coef))
    sk = _run(C_, 2, lambda: C_.conv_dgrad_bnstats(gy, w, 0, bn_x, bn_mean, bn_coef))
    _bf16_close(sk[0], dp[0])
    dref = torch.nn.grad.conv2d_input(bn_x.shape, w.float(), gy.float())
    torch.testing.assert_close(sk[0].float(), dref, rtol=1e-2, atol=2e-2)
    tol = 2 ** -8 * (N * H * W) ** 0.5
    for a, b in zip(sk[1:3], dp[1:3]):
        torch.testing.assert_close(a.sum(-1), b.sum(-1), rtol=1e-3, atol=tol)


def test_streamk_replays_in_a_graph(cuda):
    """Captured once, replayed three times: every replay equals the eager stream-K result bitwise
    (a publish flag left set would let a consumer read a stale partial)."""
    C_ = ops.native()
    x, w = _operands(cuda, 256, 1024, 14, 14, 256, 1, seed=9)
    C_.conv_set_streamk(2)
    try:
        C_.conv_sk_prepare()
        eager = C_.conv_fwd(x, w, 1, 0, True)
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            C_.conv_fwd(x, w, 1, 0, True)    # warm-up on the capture stream
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = C_.conv_fwd(x, w, 1, 0, True)
        for _ in range(3):
            for o in out:
                o.zero_()
            g.replay()
            torch.cuda.synchronize()
            for a, b in zip(out, eager):
                assert torch.equal(a, b)
        assert C_.conv_sk_errors() == 0
    finally:
        C_.conv_set_streamk(0)


def test_streamk_policy(cuda):
    C_ = ops.native()
    # auto: only grids whose tiles spread unevenly over the 256 CUs
    assert C_.conv_sk_blocks(784, 16, 128, 1) == 1024       # 3.06 tiles per CU
    assert C_.conv_sk_blocks(392, 16, 128, 1) == 512        # 1.53 per CU
    assert C_.conv_sk_blocks(3136, 16, 128, 1) == 0         # 12.25 per CU: balanced enough
    assert C_.conv_sk_blocks(1024, 16, 128, 1) == 0         # exactly 4 per CU
    assert C_.conv_sk_blocks(100, 16, 128, 2) == 0          # below one tile per CU
    assert C_.conv_sk_blocks(784, 1, 128, 2) == 0           # one K-step: nothing to split
    assert C_.conv_sk_blocks(784, 16, 128, 0) == 0
