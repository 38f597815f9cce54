"""CPU checks of the index algebra behind the native convolution paths (no GPU needed):

* stride-2 backward-data as four parity-class stride-1 convs (conv_kernels.hip
  launch_conv_dgrad_s2) - the same formulas, executed with torch ops;
* the downsample-branch deferral in the model blocks (models/layers.py DeferredBN) falls back
  to the plain composition when the BatchNorms cannot run fused.
"""
import pytest
import torch
import torch.nn.functional as F


def s2_classes(R, S, pad):
    """Per parity class (ph, pw): (taps_r, taps_s, pad_k, weight taps r(j), s(j)) exactly as
    launch_conv_dgrad_s2 derives them."""
    out = {}
    for ph in range(2):
        for pw in range(2):
            cls = []
            for p, K in ((ph, R), (pw, S)):
                r0 = (p + pad) % 2
                J = (K - 1 - r0) // 2 + 1 if r0 < K else 0
                D = (p + pad - r0) // 2
                cls.append((J, J - 1 - D, [r0 + 2 * (J - 1) - 2 * j for j in range(J)]))
            out[(ph, pw)] = cls
    return out


def dgrad_s2_by_classes(dy, w, pad, H, W):
    N, Cout, Ho, Wo = dy.shape
    _, C, R, S = w.shape
    dx = torch.zeros(N, C, H, W, dtype=dy.dtype)
    for (ph, pw), ((Jr, pr, rt), (Js, ps, st)) in s2_classes(R, S, pad).items():
        Ha, Wa = (H - ph + 1) // 2, (W - pw + 1) // 2
        if Jr == 0 or Js == 0 or Ha <= 0 or Wa <= 0:
            continue  # zero class (written as zeros by the class-(0,0) launch on the GPU)
        assert pr == ps  # the kernel takes one pad for both axes
        # GEMM tap (jr, js) reads weight tap (rt[jr], st[js]) transposed: [C, Cout, Jr, Js]
        wc = w[:, :, rt][:, :, :, st].transpose(0, 1)
        # stride-1 conv of dy, top/left pad pr, explicit output Ha x Wa (bottom/right: bounds)
        dyp = F.pad(dy, (pr, max(0, Wa + Js - 1 - Wo - pr), pr, max(0, Ha + Jr - 1 - Ho - pr)))
        y = F.conv2d(dyp, wc)[:, :, :Ha, :Wa]
        dx[:, :, ph::2, pw::2] = y
    return dx


@pytest.mark.parametrize("N,C,H,W,Cout,k,p", [(2, 3, 14, 14, 5, 1, 0), (2, 4, 15, 15, 3, 3, 1),
                                              (1, 2, 11, 12, 3, 3, 1), (2, 3, 12, 12, 2, 7, 3),
                                              (1, 2, 9, 9, 2, 1, 0), (1, 2, 10, 10, 3, 2, 0)])
def test_stride2_dgrad_parity_classes(N, C, H, W, Cout, k, p):
    g = torch.Generator().manual_seed(0)
    x = torch.randn(N, C, H, W, generator=g, dtype=torch.float64)
    w = torch.randn(Cout, C, k, k, generator=g, dtype=torch.float64)
    Ho, Wo = (H + 2 * p - k) // 2 + 1, (W + 2 * p - k) // 2 + 1
    dy = torch.randn(N, Cout, Ho, Wo, generator=g, dtype=torch.float64)
    ref = torch.nn.grad.conv2d_input(x.shape, w, dy, stride=2, padding=p)
    torch.testing.assert_close(dgrad_s2_by_classes(dy, w, p, H, W), ref)


def test_deferred_downsample_bn_falls_back():
    from distributed_pytorch_training_amd.models.layers import DeferredBN, bn_act_block_out, downsample_branch

    torch.manual_seed(0)
    ds = torch.nn.Sequential(torch.nn.Conv2d(8, 16, 1, stride=2, bias=False), torch.nn.BatchNorm2d(16))
    tail = torch.nn.BatchNorm2d(16)
    x = torch.randn(2, 8, 8, 8)
    h = torch.randn(2, 16, 4, 4)
    ident = downsample_branch(ds, x, tail)     # stock BNs: computed right away
    assert torch.is_tensor(ident)
    ref = torch.relu(tail(h) + ds(x))
    torch.testing.assert_close(bn_act_block_out(tail, h, ident), ref)
    # a deferral reaching a tail that cannot fuse materialises the downsample BN first
    d = DeferredBN(ds[1], ds[0](x))
    torch.testing.assert_close(bn_act_block_out(tail, h, d), ref)


def halo_flat_fwd(x, w):
    """The forward HALO K loop's index algebra (conv_fwd_kernel, HALO): output row m of tap (r, s)
    reads flattened input pixel m + (r-1)*W + (s-1) - a strip shifted by s rows - and the rows
    whose (ho + r - 1, wo + s - 1) falls in the padding (where the flat index wraps) are zeroed."""
    N, C, H, W = x.shape
    Cout = w.shape[0]
    xf = x.permute(0, 2, 3, 1).reshape(-1, C)
    M = xf.shape[0]
    m = torch.arange(M)
    ho, wo = (m // W) % H, m % W
    y = torch.zeros(M, Cout, dtype=x.dtype)
    for r in range(3):
        for s in range(3):
            q = m + (r - 1) * W + (s - 1)
            ok = (ho + r - 1 >= 0) & (ho + r - 1 < H) & (wo + s - 1 >= 0) & (wo + s - 1 < W)
            a = torch.where(ok[:, None], xf[q.clamp(0, M - 1)], torch.zeros(()))
            y += a @ w[:, :, r, s].T
    return y.reshape(N, H, W, Cout).permute(0, 3, 1, 2)


def halo_padded_wgrad(x, dy):
    """conv_wgrad_halo_kernel's index algebra: K runs over padded output pixels p = (n*H + ho)*(W+2)
    + wo (dy = 0 for wo >= W); tap (r, s) pairs dy row p with padded input index p + (r-1)*(W+2) +
    s (padded columns 0 and W+1 are zero), and dy rows whose tap row leaves the image are zeroed -
    no per-element masks, one strip per tap row."""
    N, C, H, W = x.shape
    Cout = dy.shape[1]
    Wp = W + 2
    xp = F.pad(x, (1, 1)).permute(0, 2, 3, 1).reshape(-1, C)                 # [N*H*Wp, C]
    dyp = F.pad(dy, (0, 2)).permute(0, 2, 3, 1).reshape(-1, Cout)          # [N*H*Wp, Cout]
    Mp = dyp.shape[0]
    p = torch.arange(Mp)
    ho = (p // Wp) % H
    dw = torch.zeros(Cout, C, 3, 3, dtype=x.dtype)
    for r in range(3):
        rows_ok = (ho + r - 1 >= 0) & (ho + r - 1 < H)
        dr = torch.where(rows_ok[:, None], dyp, torch.zeros(()))
        for s in range(3):
            q = p + (r - 1) * Wp + s
            inb = (q >= 0) & (q < Mp)
            xs = torch.where(inb[:, None], xp[q.clamp(0, Mp - 1)], torch.zeros(()))
            dw[:, :, r, s] = dr.T @ xs
    return dw


@pytest.mark.parametrize("N,C,H,W,Cout", [(2, 3, 5, 7, 4), (1, 2, 4, 4, 3), (3, 4, 6, 2, 2)])
def test_halo_index_algebra(N, C, H, W, Cout):
    g = torch.Generator().manual_seed(3)
    x = torch.randn(N, C, H, W, generator=g, dtype=torch.float64)
    w = torch.randn(Cout, C, 3, 3, generator=g, dtype=torch.float64)
    dy = torch.randn(N, Cout, H, W, generator=g, dtype=torch.float64)
    torch.testing.assert_close(halo_flat_fwd(x, w), F.conv2d(x, w, padding=1))
    torch.testing.assert_close(halo_padded_wgrad(x, dy),
                               torch.nn.grad.conv2d_weight(x, w.shape, dy, padding=1))
