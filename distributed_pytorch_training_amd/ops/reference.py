"""Pure-PyTorch reference implementations of every native kernel.

They define the semantics the gfx950 kernels must reproduce (tests compare the HIP path
against these in fp32) and they are the execution path for CPU tensors (gloo runs in the
build sandbox).  Each mirrors the torch code path the reference inherits:

* ``grad_check`` - torch._amp_foreach_non_finite_check_and_unscale_ (torch/amp/grad_scaler.py:280)
* ``sgd_step``   - torch.optim.SGD single-tensor math (torch/optim/sgd.py:343-380)
* ``adam_step``  - torch.optim.Adam / AdamW single-tensor math
* ``optim_tail`` - torch._amp_update_scale_ (torch/amp/grad_scaler.py:529-536) + step count
* ``accumulate_metrics`` - loss.item()*bs and preds.eq(targets).sum() (reference train_ddp.py:217-220)
* ``augment``    - RandomCrop(32, padding=4) + RandomHorizontalFlip + ToTensor + Normalize
                   (reference train_ddp.py:91-101)
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch


def _factor(scale: Optional[torch.Tensor], host_factor: float) -> torch.Tensor | float:
    if scale is None:
        return host_factor
    return host_factor / scale.reshape(-1)[0].to(torch.float32)


@torch.no_grad()
def grad_check(grad: torch.Tensor, scale: Optional[torch.Tensor], host_factor: float,
               found_inf: torch.Tensor) -> None:
    f = _factor(scale, host_factor)
    if not bool(torch.isfinite(grad * f).all()):
        found_inf.fill_(1.0)


@torch.no_grad()
def sgd_step(param, grad, momentum_buffer, lr, momentum, dampening, weight_decay, nesterov,
             scale, host_factor, found_inf, step, zero_grad) -> None:
    skip = found_inf is not None and float(found_inf.reshape(-1)[0]) != 0.0
    if not skip:
        d = grad * _factor(scale, host_factor)
        if weight_decay != 0:
            d = d.add(param, alpha=weight_decay)
        if momentum != 0:
            first = step is None or float(step.reshape(-1)[0]) == 0.0
            if first:
                momentum_buffer.copy_(d)
            else:
                momentum_buffer.mul_(momentum).add_(d, alpha=1 - dampening)
            d = d.add(momentum_buffer, alpha=momentum) if nesterov else momentum_buffer
        param.add_(d, alpha=-lr)
    if zero_grad:
        grad.zero_()


@torch.no_grad()
def adam_step(param, grad, exp_avg, exp_avg_sq, lr, beta1, beta2, eps, weight_decay, adamw,
              scale, host_factor, found_inf, step, zero_grad) -> None:
    skip = found_inf is not None and float(found_inf.reshape(-1)[0]) != 0.0
    if not skip:
        g = grad * _factor(scale, host_factor)
        if adamw:
            param.mul_(1 - lr * weight_decay)
        elif weight_decay != 0:
            g = g.add(param, alpha=weight_decay)
        t = (float(step.reshape(-1)[0]) if step is not None else 0.0) + 1.0
        exp_avg.lerp_(g, 1 - beta1)
        exp_avg_sq.mul_(beta2).addcmul_(g, g, value=1 - beta2)
        bc1 = 1 - beta1 ** t
        bc2_sqrt = (1 - beta2 ** t) ** 0.5
        denom = (exp_avg_sq.sqrt() / bc2_sqrt).add_(eps)
        param.addcdiv_(exp_avg, denom, value=-lr / bc1)
    if zero_grad:
        grad.zero_()


@torch.no_grad()
def optim_tail(scale, growth_tracker, found_inf, step, growth_factor, backoff_factor,
               growth_interval) -> None:
    inf = float(found_inf.reshape(-1)[0]) != 0.0
    if scale is not None:
        if inf:
            scale.mul_(backoff_factor)
            growth_tracker.zero_()
        else:
            successful = int(growth_tracker.reshape(-1)[0]) + 1
            if successful == growth_interval:
                ns = scale * growth_factor
                if bool(torch.isfinite(ns).all()):
                    scale.copy_(ns)
                growth_tracker.zero_()
            else:
                growth_tracker.fill_(successful)
    if step is not None and not inf:
        step.add_(1.0)
    found_inf.zero_()


@torch.no_grad()
def accumulate_metrics(logits: torch.Tensor, targets: torch.Tensor, loss: Optional[torch.Tensor],
                       acc: torch.Tensor) -> None:
    preds = logits.float().argmax(dim=1)
    acc[1] += preds.eq(targets).sum().to(acc.dtype)
    if loss is not None:
        acc[0] += loss.detach().to(acc.dtype) * logits.shape[0]
    acc[2] += logits.shape[0]


@torch.no_grad()
def augment(data: torch.Tensor, idx: torch.Tensor, offs: Optional[torch.Tensor],
            flips: Optional[torch.Tensor], out: torch.Tensor, nhwc: bool, pad: int,
            mean: Sequence[float], std: Sequence[float]) -> None:
    imgs = data.index_select(0, idx).float()                      # [B,C,H,W] 0..255
    b, c, h, w = imgs.shape
    padded = torch.nn.functional.pad(imgs, (pad, pad, pad, pad))  # zero pad in pixel space
    if offs is None:
        dy = torch.full((b,), pad, dtype=torch.long, device=imgs.device)
        dx = dy.clone()
    else:
        dy, dx = offs[:, 0].long(), offs[:, 1].long()
    ys = (torch.arange(h, device=imgs.device)[None, :] + dy[:, None])          # [B,H]
    xs = (torch.arange(w, device=imgs.device)[None, :] + dx[:, None])          # [B,W]
    if flips is not None:
        fl = flips.bool()[:, None]
        xs_f = (torch.arange(w - 1, -1, -1, device=imgs.device)[None, :] + dx[:, None])
        xs = torch.where(fl, xs_f, xs)
    bi = torch.arange(b, device=imgs.device)[:, None, None, None]
    ci = torch.arange(c, device=imgs.device)[None, :, None, None]
    crop = padded[bi, ci, ys[:, None, :, None], xs[:, None, None, :]]
    m = torch.tensor(mean, dtype=torch.float32, device=imgs.device).view(1, c, 1, 1)
    s = torch.tensor(std, dtype=torch.float32, device=imgs.device).view(1, c, 1, 1)
    res = (crop / 255.0 - m) / s
    out.copy_(res.to(memory_format=torch.channels_last) if nhwc else res)


@torch.no_grad()
def pack_bf16(src: torch.Tensor, dst: torch.Tensor) -> None:
    dst.copy_(src.to(torch.bfloat16))


@torch.no_grad()
def unpack_bf16(src, dst, scale, host_factor, found_inf) -> None:
    dst.copy_(src.float())
    if found_inf is not None:
        grad_check(dst, scale, host_factor, found_inf)
