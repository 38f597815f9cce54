"""Fused, loss-scale-aware optimizers over a flat parameter arena.

``FusedSGD`` reproduces ``torch.optim.SGD(params, lr, momentum, weight_decay)`` as the
reference constructs it (reference train_ddp.py:339-344; math torch/optim/sgd.py:343-380,
dampening 0, nesterov False by default) and ``FusedAdam`` reproduces torch.optim.Adam /
AdamW.  One ``step()`` is at most three launches on the current stream, none of which
synchronises with the host:

1. ``grad_check`` (only if the reducer has not already checked every bucket and a scaler
   is enabled): found_inf |= !isfinite(g / (world_size * scale));
2. the fused update kernel: reads found_inf and the device scale, skips itself on inf,
   applies g * host_factor / scale, weight decay, momentum / Adam moments, writes the
   parameter and zeroes the gradient for the next step (the reference's
   ``zero_grad(set_to_none=True)``, reference train_ddp.py:201) - skipped
   (``zero_grad=False``) when the reducer overwrites the whole arena in the next backward
   (GPU steal mode without accumulation: 4 B/param of HBM writes saved);
3. the one-thread tail: GradScaler growth/backoff, step counter, clear found_inf.

State dicts use torch's layout (``state[i]['momentum_buffer']`` / ``exp_avg`` /
``exp_avg_sq`` / ``step`` keyed by the module's parameter order, ``param_groups``) so
checkpoints load into stock torch optimizers and back.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Sequence

import torch

from .. import ops
from ..amp.grad_scaler import DeviceGradScaler


class _FlatOptimizer:
    def __init__(self, arena, params_in_order: Optional[Sequence[torch.Tensor]] = None,
                 defaults: Optional[Dict[str, Any]] = None) -> None:
        self.arena = arena
        self.defaults = dict(defaults or {})
        ordered = list(params_in_order) if params_in_order is not None else list(arena.params)
        index = {id(p): i for i, p in enumerate(arena.params)}
        missing = [p for p in ordered if id(p) not in index]
        if missing:
            raise ValueError("optimizer parameters must all live in the arena")
        self._order = ordered          # module parameter order (state_dict ids)
        self._step = torch.zeros(1, dtype=torch.float32, device=arena.device)
        self.param_groups = [dict(self.defaults, params=ordered)]
        self._fallback_found_inf = torch.zeros(1, dtype=torch.float32, device=arena.device)

    # lr etc. are read from param_groups[0] each step so schedulers can edit them.
    @property
    def group(self) -> Dict[str, Any]:
        return self.param_groups[0]

    @property
    def steps_taken(self) -> torch.Tensor:
        return self._step

    def zero_grad(self, set_to_none: bool = True) -> None:
        """Gradients are zeroed by the fused kernel; this is for out-of-band use."""
        if self.arena.grad_flat is not None:
            self.arena.grad_flat.zero_()
        self.arena.reattach_grads()

    def _prologue(self, scaler: Optional[DeviceGradScaler], host_factor: float,
                  grads_checked: bool):
        scale = scaler.scale_tensor if scaler is not None else None
        found_inf = scaler.found_inf if scaler is not None else self._fallback_found_inf
        if scale is not None and not grads_checked:
            ops.grad_check(self.arena.grad_flat, scale, host_factor, found_inf)
        return scale, found_inf

    def _epilogue(self, scaler: Optional[DeviceGradScaler], found_inf: torch.Tensor) -> None:
        if scaler is not None and scaler.is_enabled():
            ops.optim_tail(scaler.scale_tensor, scaler.growth_tracker, found_inf, self._step,
                           scaler.growth_factor, scaler.backoff_factor, scaler.growth_interval)
        else:
            ops.optim_tail(None, None, found_inf, self._step)

    def _index(self, p: torch.Tensor) -> int:
        for i, q in enumerate(self.arena.params):
            if q is p:
                return i
        raise KeyError("parameter not in arena")

    def _export(self, flat: torch.Tensor) -> List[torch.Tensor]:
        views = self.arena.views(flat)
        pos = {id(p): i for i, p in enumerate(self.arena.params)}
        return [views[pos[id(p)]].clone() for p in self._order]

    def _import(self, flat: torch.Tensor, tensors: Sequence[torch.Tensor]) -> None:
        views = self.arena.views(flat)
        pos = {id(p): i for i, p in enumerate(self.arena.params)}
        with torch.no_grad():
            for p, t in zip(self._order, tensors):
                views[pos[id(p)]].copy_(t.to(flat.device, flat.dtype).reshape(p.shape))

    def _groups_state(self) -> List[Dict[str, Any]]:
        g = {k: v for k, v in self.group.items() if k != "params"}
        g["params"] = list(range(len(self._order)))
        return [g]


class FusedSGD(_FlatOptimizer):
    def __init__(self, arena, lr: float = 0.1, momentum: float = 0.0, dampening: float = 0.0,
                 weight_decay: float = 0.0, nesterov: bool = False,
                 params_in_order: Optional[Sequence[torch.Tensor]] = None) -> None:
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        super().__init__(arena, params_in_order, dict(lr=lr, momentum=momentum, dampening=dampening,
                                                      weight_decay=weight_decay, nesterov=nesterov,
                                                      maximize=False, foreach=None,
                                                      differentiable=False, fused=True))
        self.momentum_buffer: Optional[torch.Tensor] = None

    def arena_state(self) -> List[torch.Tensor]:
        return [self.momentum_buffer] if self.momentum_buffer is not None else []

    def set_arena_state(self, tensors: Sequence[torch.Tensor]) -> None:
        if tensors:
            self.momentum_buffer = tensors[0]

    def step(self, scaler: Optional[DeviceGradScaler] = None, host_factor: float = 1.0,
             grads_checked: bool = False, shadow: Optional[torch.Tensor] = None,
             zero_grad: bool = True) -> None:
        g = self.group
        if g["momentum"] != 0 and self.momentum_buffer is None:
            self.momentum_buffer = self.arena.zeros_like_arena()
        scale, found_inf = self._prologue(scaler, host_factor, grads_checked)
        ops.sgd_step(self.arena.param_flat, self.arena.grad_flat, self.momentum_buffer,
                     lr=g["lr"], momentum=g["momentum"], dampening=g["dampening"],
                     weight_decay=g["weight_decay"], nesterov=g["nesterov"], scale=scale,
                     host_factor=host_factor, found_inf=found_inf, step=self._step, zero_grad=zero_grad,
                     shadow=shadow)
        self._epilogue(scaler, found_inf)

    def state_dict(self) -> Dict[str, Any]:
        state: Dict[int, Dict[str, Any]] = {}
        if self.momentum_buffer is not None and float(self._step.item()) > 0:
            for i, t in enumerate(self._export(self.momentum_buffer)):
                state[i] = {"momentum_buffer": t}
        return {"state": state, "param_groups": self._groups_state()}

    def load_state_dict(self, sd: Dict[str, Any]) -> None:
        for k, v in sd["param_groups"][0].items():
            if k != "params":
                self.group[k] = v
        st = sd.get("state", {})
        if st:
            if self.momentum_buffer is None:
                self.momentum_buffer = self.arena.zeros_like_arena()
            bufs = [st[i]["momentum_buffer"] if i in st else st[str(i)]["momentum_buffer"]
                    for i in range(len(self._order))]
            self._import(self.momentum_buffer, bufs)
            self._step.fill_(max(1.0, float(self._step.item())))


class FusedAdam(_FlatOptimizer):
    def __init__(self, arena, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, adamw: bool = False,
                 params_in_order: Optional[Sequence[torch.Tensor]] = None) -> None:
        super().__init__(arena, params_in_order, dict(lr=lr, betas=tuple(betas), eps=eps,
                                                      weight_decay=weight_decay, amsgrad=False,
                                                      maximize=False, foreach=None,
                                                      capturable=True, differentiable=False,
                                                      fused=True))
        self.adamw = adamw
        self.exp_avg: Optional[torch.Tensor] = None
        self.exp_avg_sq: Optional[torch.Tensor] = None

    def arena_state(self) -> List[torch.Tensor]:
        return [self.exp_avg, self.exp_avg_sq] if self.exp_avg is not None else []

    def set_arena_state(self, tensors: Sequence[torch.Tensor]) -> None:
        if tensors:
            self.exp_avg, self.exp_avg_sq = tensors

    def step(self, scaler: Optional[DeviceGradScaler] = None, host_factor: float = 1.0,
             grads_checked: bool = False, shadow: Optional[torch.Tensor] = None,
             zero_grad: bool = True) -> None:
        g = self.group
        if self.exp_avg is None:
            self.exp_avg = self.arena.zeros_like_arena()
            self.exp_avg_sq = self.arena.zeros_like_arena()
        scale, found_inf = self._prologue(scaler, host_factor, grads_checked)
        b1, b2 = g["betas"]
        ops.adam_step(self.arena.param_flat, self.arena.grad_flat, self.exp_avg, self.exp_avg_sq,
                      lr=g["lr"], beta1=b1, beta2=b2, eps=g["eps"], weight_decay=g["weight_decay"],
                      adamw=self.adamw, scale=scale, host_factor=host_factor, found_inf=found_inf,
                      step=self._step, zero_grad=zero_grad, shadow=shadow)
        self._epilogue(scaler, found_inf)

    def state_dict(self) -> Dict[str, Any]:
        state: Dict[int, Dict[str, Any]] = {}
        if self.exp_avg is not None:
            step = self._step.detach().reshape(()).clone()
            for i, (m, v) in enumerate(zip(self._export(self.exp_avg), self._export(self.exp_avg_sq))):
                state[i] = {"step": step.clone(), "exp_avg": m, "exp_avg_sq": v}
        return {"state": state, "param_groups": self._groups_state()}

    def load_state_dict(self, sd: Dict[str, Any]) -> None:
        for k, v in sd["param_groups"][0].items():
            if k != "params":
                self.group[k] = tuple(v) if k == "betas" else v
        st = sd.get("state", {})
        if st:
            if self.exp_avg is None:
                self.exp_avg = self.arena.zeros_like_arena()
                self.exp_avg_sq = self.arena.zeros_like_arena()
            get = lambda i: st[i] if i in st else st[str(i)]
            self._import(self.exp_avg, [get(i)["exp_avg"] for i in range(len(self._order))])
            self._import(self.exp_avg_sq, [get(i)["exp_avg_sq"] for i in range(len(self._order))])
            self._step.fill_(float(torch.as_tensor(get(0)["step"]).item()))


def build_optimizer(name: str, arena, args, params_in_order=None) -> _FlatOptimizer:
    if name == "sgd":
        return FusedSGD(arena, lr=args.lr, momentum=args.momentum, weight_decay=args.weight_decay,
                        nesterov=getattr(args, "nesterov", False), params_in_order=params_in_order)
    if name in ("adam", "adamw"):
        return FusedAdam(arena, lr=args.lr, betas=getattr(args, "betas", (0.9, 0.999)),
                         eps=getattr(args, "eps", 1e-8), weight_decay=args.weight_decay,
                         adamw=(name == "adamw"), params_in_order=params_in_order)
    raise ValueError(f"unknown optimizer {name!r}")
