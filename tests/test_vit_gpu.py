"""Fused ViT block kernels (vit_kernels.hip) vs fp32 PyTorch references, and the fused ViT
encoder vs the module-by-module path under bf16 autocast."""
import copy

import pytest
import torch
import torch.nn.functional as F

from distributed_pytorch_training_amd import ops
from distributed_pytorch_training_amd.ops.vit import add_bias_layer_norm16, bias_gelu16, layer_norm16

pytestmark = pytest.mark.gpu


def _ln(D, dev):
    ln = torch.nn.LayerNorm(D, eps=1e-6).to(dev)
    with torch.no_grad():
        ln.weight.uniform_(0.5, 1.5)
        ln.bias.uniform_(-0.2, 0.2)
    return ln


def _close(a, b, rtol, atol, what):
    torch.testing.assert_close(a.float(), b.float(), rtol=rtol, atol=atol, msg=what)


@pytest.mark.parametrize("D", [256, 768, 1024])
def test_layer_norm16_matches_fp32(cuda, D):
    torch.manual_seed(0)
    ln = _ln(D, cuda)
    x = (torch.randn(3, 197, D, device=cuda) * 2 + 0.5).requires_grad_(True)
    h = layer_norm16(x, ln, torch.bfloat16)
    assert h.dtype == torch.bfloat16
    gh = torch.randn_like(h)
    h.backward(gh)
    xr = x.detach().clone().requires_grad_(True)
    lr = copy.deepcopy(ln)
    hr = F.layer_norm(xr, (D,), lr.weight, lr.bias, lr.eps)
    hr.backward(gh.float())
    _close(h, hr, 1e-2, 2e-2, "h")
    _close(x.grad, xr.grad, 1e-3, 1e-3, "dx")
    _close(ln.weight.grad, lr.weight.grad, 1e-3, 1e-2, "dgamma")
    _close(ln.bias.grad, lr.bias.grad, 1e-3, 1e-2, "dbeta")


@pytest.mark.parametrize("bias_dtype", [torch.float32, torch.bfloat16, None])
def test_add_bias_layer_norm16_matches_fp32(cuda, bias_dtype):
    torch.manual_seed(1)
    D = 768
    ln = _ln(D, cuda)
    x = torch.randn(2, 197, D, device=cuda).requires_grad_(True)
    a = torch.randn(2, 197, D, device=cuda).to(torch.bfloat16).requires_grad_(True)
    b = None if bias_dtype is None else (torch.randn(D, device=cuda) * 0.1).to(bias_dtype).requires_grad_(True)
    s, h = add_bias_layer_norm16(x, a, b, ln)
    gs, gh = torch.randn_like(s), torch.randn_like(h)
    torch.autograd.backward([s, h], [gs, gh])
    # fp32 reference on the same (rounded) inputs
    xr, ar = x.detach().clone().requires_grad_(True), a.detach().float().requires_grad_(True)
    br = None if b is None else b.detach().float().requires_grad_(True)
    lr = copy.deepcopy(ln)
    for p in lr.parameters():
        p.grad = None
    sr = xr + ar + (br if br is not None else 0.0)
    hr = F.layer_norm(sr, (D,), lr.weight, lr.bias, lr.eps)
    torch.autograd.backward([sr, hr], [gs, gh.float()])
    _close(s, sr, 1e-6, 1e-6, "s")
    _close(h, hr, 1e-2, 2e-2, "h")
    _close(x.grad, xr.grad, 1e-4, 1e-4, "dx")
    assert a.grad.dtype == torch.bfloat16
    _close(a.grad, ar.grad, 1e-2, 1e-2, "da")
    if b is not None:
        assert b.grad.dtype == bias_dtype
        tol = 1e-4 if bias_dtype == torch.float32 else 1e-2
        _close(b.grad, br.grad, tol, tol * 10, "dbias")
    _close(ln.weight.grad, lr.weight.grad, 1e-3, 1e-2, "dgamma")
    _close(ln.bias.grad, lr.bias.grad, 1e-3, 1e-2, "dbeta")


@pytest.mark.parametrize("with_bias", [True, False])
def test_bias_gelu16_matches_fp32(cuda, with_bias):
    torch.manual_seed(2)
    u = (torch.randn(2 * 197, 3072, device=cuda) * 2).to(torch.bfloat16).requires_grad_(True)
    b = (torch.randn(3072, device=cuda) * 0.5).requires_grad_(True) if with_bias else None
    h = bias_gelu16(u, b)
    gh = torch.randn_like(h)
    h.backward(gh)
    ur = u.detach().float().requires_grad_(True)
    br = b.detach().clone().requires_grad_(True) if with_bias else None
    hr = F.gelu(ur + (br if with_bias else 0.0))
    hr.backward(gh.float())
    _close(h, hr, 1e-2, 1e-2, "h")
    _close(u.grad, ur.grad, 1e-2, 1e-2, "du")
    if with_bias:
        _close(b.grad, br.grad, 1e-3, 5e-2, "dbias")


def test_vit_fused_encoder_matches_unfused(cuda):
    """Fused encoder path vs the module-by-module path under bf16 autocast: both are compared
    to an fp32 run and the fused error must be of the same order."""
    from distributed_pytorch_training_amd.models import build_model
    from distributed_pytorch_training_amd.models.vit import Encoder

    torch.manual_seed(0)
    base = build_model("vit_b_16", 10, cuda, image_size=64)
    with torch.no_grad():      # torchvision zero-inits the head: give it values so grads flow
        base.heads.head.weight.normal_(std=0.02)
    x = torch.randn(4, 3, 64, 64, device=cuda)
    y = torch.randint(0, 10, (4,), device=cuda)

    def run(model, autocast, fused):
        orig = Encoder._fused_ok
        if not fused:
            Encoder._fused_ok = lambda self, t: False
        try:
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
                loss = F.cross_entropy(model(x), y)
            loss.backward()
        finally:
            Encoder._fused_ok = orig
        return loss.detach(), {n: p.grad.detach().float().clone() for n, p in model.named_parameters()}

    from distributed_pytorch_training_amd.models.vit import set_native

    fused_m, unf_m, ref_m = (copy.deepcopy(base) for _ in range(3))
    set_native(fused_m)
    set_native(unf_m)      # native module-by-module (the fused encoder switched off below)
    lf, gf = run(fused_m, True, True)
    lu, gu = run(unf_m, True, False)
    lr, gr = run(ref_m, False, False)
    assert abs(lf - lr) < 2e-2 and abs(lu - lr) < 2e-2
    for n in gr:
        scale = gr[n].abs().max().item() + 1e-6
        ef = (gf[n] - gr[n]).abs().max().item() / scale
        eu = (gu[n] - gr[n]).abs().max().item() / scale
        assert ef < max(3 * eu, 0.05), (n, ef, eu)


def test_vit_trainer_fused_step(cuda):
    """One native AdamW step of ViT through the fused path with weight shadows."""
    from distributed_pytorch_training_amd.config import parse_args
    from distributed_pytorch_training_amd.engine.trainer import Trainer
    from distributed_pytorch_training_amd.models import build_model

    torch.manual_seed(0)
    m = build_model("vit_b_16", 10, cuda, image_size=32)
    args = parse_args(["--model", "vit_b_16", "--dataset", "synthetic", "--no-cuda-graph", "--amp", "--amp-dtype", "bf16",
                       "--optimizer", "adamw", "--lr", "1e-3"])
    tr = Trainer(m, args, 0, 1, cuda, log=lambda s: None)
    before = tr.ddp.arena.param_flat.clone()
    x = torch.randn(8, 3, 32, 32, device=cuda)
    y = torch.randint(0, 10, (8,), device=cuda)
    for _ in range(2):
        tr.train_step(x, y)
    torch.cuda.synchronize()
    assert torch.isfinite(tr.ddp.arena.param_flat).all()
    assert not torch.equal(before, tr.ddp.arena.param_flat)
    assert ops.native_available()


def test_split_merge_heads_match_torch(cuda):
    from distributed_pytorch_training_amd.ops.vit import merge_heads, split_heads

    torch.manual_seed(3)
    b, s, h, dh = 3, 197, 12, 64
    qkv = torch.randn(b, s, 3 * h * dh, device=cuda).to(torch.bfloat16).requires_grad_(True)
    q, k, v = split_heads(qkv, h)
    ref = qkv.detach().view(b, s, 3, h, dh).permute(2, 0, 3, 1, 4)
    assert torch.equal(q, ref[0]) and torch.equal(k, ref[1]) and torch.equal(v, ref[2])
    y = F.scaled_dot_product_attention(q, k, v)
    m = merge_heads(y)
    assert m.is_contiguous() and torch.equal(m, y.detach().transpose(1, 2).reshape(b, s, h * dh))
    g = torch.randn_like(m)
    m.backward(g)
    qkv2 = qkv.detach().clone().requires_grad_(True)
    r = qkv2.view(b, s, 3, h, dh).permute(2, 0, 3, 1, 4)
    y2 = F.scaled_dot_product_attention(r[0], r[1], r[2])
    y2.transpose(1, 2).reshape(b, s, h * dh).backward(g)
    torch.testing.assert_close(qkv.grad.float(), qkv2.grad.float(), rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("n_out,n_in,bias", [(3072, 768, False), (768, 768, False), (2304, 768, True)])
def test_linear16_splitk_wgrad(cuda, n_out, n_in, bias):
    from distributed_pytorch_training_amd.ops.vit import _wgrad_splits, linear16

    torch.manual_seed(4)
    T = 8 * 197 * 4
    assert _wgrad_splits(n_out, n_in, T) > 1
    x = torch.randn(T, n_in, device=cuda).to(torch.bfloat16).requires_grad_(True)
    w = (torch.randn(n_out, n_in, device=cuda) * 0.02).to(torch.bfloat16).requires_grad_(True)
    b = torch.randn(n_out, device=cuda).requires_grad_(True) if bias else None
    y = linear16(x, w, b)
    g = torch.randn_like(y)
    y.backward(g)
    xr, wr = x.detach().float().requires_grad_(True), w.detach().float().requires_grad_(True)
    br = b.detach().clone().requires_grad_(True) if bias else None
    F.linear(xr, wr, br).backward(g.float())
    assert w.grad.dtype == torch.bfloat16
    _close(w.grad, wr.grad, 1e-2, 1e-1, "dW")
    _close(x.grad, xr.grad, 1e-2, 1e-2, "dx")
    if bias:   # autocast semantics: the bf16 copy's gradient, rounded once (<= 1 ulp = 2^-8 relative)
        assert b.grad.dtype == torch.float32
        _close(b.grad, br.grad, 1e-2, 1e-1, "db")


@pytest.mark.parametrize("T,dt", [(2 * 197, torch.bfloat16), (1000, torch.bfloat16), (2 * 197, torch.float16)])
def test_linear_dgrad_dgelu_matches_fp32(cuda, T, dt):
    """fc2's backward-data with GELU's backward fused (conv_fwd_kernel DGELU epilogue) against fp32:
    gu = (dz W2) * gelu'(u + b1), and the per-tile column sums that make fc1's bias gradient.
    T = 1000 leaves a partial last 128-row tile."""
    from distributed_pytorch_training_amd.ops import native
    torch.manual_seed(4)
    n_in, n_out = 3072, 768
    u = (torch.randn(T, n_in, device=cuda) * 2).to(dt)
    b = torch.randn(n_in, device=cuda) * 0.5
    w = (torch.randn(n_out, n_in, device=cuda) / n_in ** 0.5).to(dt)
    dz = torch.randn(T, n_out, device=cuda).to(dt)
    gu, part = native().linear_dgrad_dgelu(dz, w.t().contiguous(), u, b)
    assert part.shape == ((T + 127) // 128, n_in)
    # the kernel rounds g = dz W2 to bf16 before the GELU derivative, as the unfused path's GEMM
    # output does: the reference does too (otherwise the column sums of T values carry
    # sqrt(T) bf16 roundings of difference)
    gh = (dz.float() @ w.float()).to(dt).float()
    ur = (u.float() + b).requires_grad_(True)
    F.gelu(ur).backward(gh)
    _close(gu, ur.grad, 2e-2, 2e-2, "gu")
    _close(part.sum(0), ur.grad.sum(0), 1e-2, 5e-2, "dbias")


def test_gelu_linear16_fused_matches_unfused(cuda):
    """The fused MLP tail (gelu_linear16) against the two-launch composition it replaces: same
    forward bits, gradients within the bf16 rounding of gh."""
    from distributed_pytorch_training_amd.ops import vit as vops
    torch.manual_seed(5)
    T, n_in, n_out = 4 * 197, 3072, 768
    u0 = (torch.randn(T, n_in, device=cuda) * 2).to(torch.bfloat16)
    b0 = (torch.randn(n_in, device=cuda) * 0.5).to(torch.bfloat16)
    w0 = (torch.randn(n_out, n_in, device=cuda) / n_in ** 0.5)
    gz = torch.randn(T, n_out, device=cuda).to(torch.bfloat16)
    outs = {}
    for fused in (True, False):
        u, b, w = (t.clone().requires_grad_(True) for t in (u0, b0, w0))
        old = vops.FUSED_DGELU
        vops.FUSED_DGELU = fused
        try:
            z = vops.gelu_linear16(u, b, w)
            z.backward(gz)
        finally:
            vops.FUSED_DGELU = old
        outs[fused] = (z.detach(), u.grad, b.grad, w.grad)
    assert torch.equal(outs[True][0], outs[False][0])
    for name, a, r in zip(("du", "db", "dw"), outs[True][1:], outs[False][1:]):
        _close(a, r, 2e-2, 5e-2, name)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_transpose16_is_exact(cuda, dt):
    """fc2's weight transpose for the DGELU backward-data (tiled weight-flip kernel) == .t()."""
    from distributed_pytorch_training_amd.ops.vit import _transpose16
    w = torch.randn(768, 3072, device=cuda).to(dt)
    assert torch.equal(_transpose16(w), w.t().contiguous())


@pytest.mark.parametrize("n,D,dt", [(197, 3072, torch.bfloat16), (5, 64, torch.float32), (1000, 768, torch.float16)])
def test_colsum_rows_matches_fp64(cuda, n, D, dt):
    from distributed_pytorch_training_amd.ops import native
    part = torch.randn(n, D, device=cuda)
    kind = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}[dt]
    out = native().colsum_rows(part, kind)
    assert out.dtype == dt and out.shape == (D,)
    torch.testing.assert_close(out, part.double().sum(0).float().to(dt), rtol=0, atol=0)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_linear_dgrad_dgelu_16bit_bias_same_bits(cuda, dt):
    """A bias in the operands' 16-bit type (read in the epilogue) == the same values as fp32."""
    from distributed_pytorch_training_amd.ops import native
    torch.manual_seed(5)
    T, n_in, n_out = 300, 3072, 768
    u = torch.randn(T, n_in, device=cuda).to(dt)
    b16 = (torch.randn(n_in, device=cuda) * 0.5).to(dt)
    wt = (torch.randn(n_in, n_out, device=cuda) / n_out ** 0.5).to(dt)
    dz = torch.randn(T, n_out, device=cuda).to(dt)
    gu16, p16 = native().linear_dgrad_dgelu(dz, wt, u, b16)
    gu32, p32 = native().linear_dgrad_dgelu(dz, wt, u, b16.float())
    assert torch.equal(gu16, gu32) and torch.equal(p16, p32)
