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
