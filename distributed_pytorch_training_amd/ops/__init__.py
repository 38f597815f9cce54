"""Op dispatch: GPU tensors run the gfx950 HIP kernels from the in-tree ``_C`` extension,
CPU tensors run the PyTorch reference (``ops/reference.py``).

There is no silent fallback for GPU tensors: if a GPU tensor reaches an op and the native
extension is not importable, the op raises.  Build it with ``python csrc/build.py`` (or
``__graft_entry__.build()``).
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch

from . import reference

def _load():
    """The in-tree extension built by csrc/build.py, or the file named by ``DPT_NATIVE_LIB``
    (the AddressSanitizer build under build/asan/, CPU debug runs only)."""
    import os
    path = os.environ.get("DPT_NATIVE_LIB")
    if not path:
        from .. import _C as mod  # type: ignore[attr-defined]
        return mod
    import importlib.util
    import sys
    spec = importlib.util.spec_from_file_location("distributed_pytorch_training_amd._C", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    sys.modules["distributed_pytorch_training_amd._C"] = mod
    return mod


try:
    _C = _load()
    _IMPORT_ERROR: Optional[BaseException] = None
except Exception as e:  # pragma: no cover - depends on the build
    _C = None
    _IMPORT_ERROR = e


def native_available() -> bool:
    return _C is not None


def native():
    """Return the extension module or raise with the import error."""
    if _C is None:
        raise RuntimeError(
            "distributed_pytorch_training_amd._C (gfx950 HIP kernels) is not built or failed to "
            f"import: {_IMPORT_ERROR!r}. Run `python csrc/build.py`.")
    return _C


def _gpu(t: Optional[torch.Tensor]) -> bool:
    return t is not None and t.is_cuda


def grad_check(grad, scale, host_factor: float, found_inf) -> None:
    if _gpu(grad):
        native().grad_check(grad, scale, float(host_factor), found_inf)
    else:
        reference.grad_check(grad, scale, host_factor, found_inf)


def sgd_step(param, grad, momentum_buffer, *, lr, momentum, dampening, weight_decay, nesterov,
             scale=None, host_factor=1.0, found_inf=None, step=None, zero_grad=True, shadow=None) -> None:
    if _gpu(param):
        native().sgd_step(param, grad, momentum_buffer if momentum_buffer is not None else param,
                          float(lr), float(momentum), float(dampening), float(weight_decay),
                          bool(nesterov), scale, float(host_factor), found_inf, step, bool(zero_grad),
                          shadow)
    else:
        reference.sgd_step(param, grad, momentum_buffer, lr, momentum, dampening, weight_decay,
                           nesterov, scale, host_factor, found_inf, step, zero_grad)
        if shadow is not None:
            shadow.copy_(param)


def adam_step(param, grad, exp_avg, exp_avg_sq, *, lr, beta1, beta2, eps, weight_decay, adamw,
              scale=None, host_factor=1.0, found_inf=None, step=None, zero_grad=True, shadow=None) -> None:
    if _gpu(param):
        native().adam_step(param, grad, exp_avg, exp_avg_sq, float(lr), float(beta1), float(beta2),
                           float(eps), float(weight_decay), bool(adamw), scale, float(host_factor),
                           found_inf, step, bool(zero_grad), shadow)
    else:
        reference.adam_step(param, grad, exp_avg, exp_avg_sq, lr, beta1, beta2, eps, weight_decay,
                            adamw, scale, host_factor, found_inf, step, zero_grad)
        if shadow is not None:
            shadow.copy_(param)


def optim_tail(scale, growth_tracker, found_inf, step, growth_factor=2.0, backoff_factor=0.5,
               growth_interval=2000) -> None:
    if _gpu(found_inf):
        native().optim_tail(scale, growth_tracker, found_inf, step, float(growth_factor),
                            float(backoff_factor), int(growth_interval))
    else:
        reference.optim_tail(scale, growth_tracker, found_inf, step, growth_factor,
                             backoff_factor, growth_interval)


def accumulate_metrics(logits, targets, loss, acc) -> None:
    if _gpu(logits):
        native().accumulate_metrics(logits.detach(), targets, loss, acc)
    else:
        reference.accumulate_metrics(logits.detach(), targets, loss, acc)


def augment(data, idx, offs, flips, out, *, nhwc: bool, pad: int, mean: Sequence[float],
            std: Sequence[float]) -> None:
    if _gpu(data):
        native().augment(data, idx, offs, flips, out, bool(nhwc), int(pad), list(map(float, mean)),
                         list(map(float, std)))
    else:
        reference.augment(data, idx, offs, flips, out, nhwc, pad, mean, std)


def pack_bf16(src, dst) -> None:
    if _gpu(src):
        native().pack_bf16(src, dst)
    else:
        reference.pack_bf16(src, dst)


def unpack_bf16(src, dst, scale=None, host_factor=1.0, found_inf=None) -> None:
    if _gpu(dst):
        native().unpack_bf16(src, dst, scale, float(host_factor), found_inf)
    else:
        reference.unpack_bf16(src, dst, scale, host_factor, found_inf)


__all__ = ["native_available", "native", "grad_check", "sgd_step", "adam_step", "optim_tail",
           "accumulate_metrics", "augment", "pack_bf16", "unpack_bf16", "reference"]
