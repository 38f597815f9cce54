"""Flat parameter / gradient arenas.

MI355X-first layout for the data-parallel hot path: every trainable parameter of one
dtype becomes a view into ONE contiguous ``param_flat`` buffer and its ``.grad`` a view
into ONE contiguous ``grad_flat`` buffer, in the same order.  Consequences:

* autograd's AccumulateGrad writes each gradient directly into its all-reduce bucket
  (buckets are contiguous slices of ``grad_flat``), so the DDP copy-in/copy-out passes of
  the reference's inherited reducer disappear;
* the fused optimizer is ONE kernel launch over the whole arena instead of 4 foreach
  passes over 62-161 tensors (K15);
* checkpoint/broadcast/consistency checks are single contiguous operations.

Each parameter starts on a 16-element (64-byte) boundary so per-parameter views are
16-byte aligned for the vendor kernels that read them, and the arena length is a multiple
of 64 so the float4 / bf16x8 kernels never need a tail.  Padding elements stay zero in
params, grads and optimizer state (the update of a zero with a zero gradient is zero for
SGD and Adam), so kernels can sweep the whole arena blindly.

Parameters keep their memory format: a channels_last conv weight becomes a
channels_last-strided view (``as_strided``) over its arena region.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import torch

ALIGN = 16        # elements; 64 B for fp32
TOTAL_ALIGN = 64  # elements


def _round_up(x: int, a: int) -> int:
    return (x + a - 1) // a * a


def _is_dense(t: torch.Tensor) -> bool:
    return t.is_contiguous() or t.is_contiguous(memory_format=torch.channels_last)


class FlatArena:
    """Parameters (``params``, in arena order) re-homed into flat param/grad buffers."""

    def __init__(self, params: Sequence[torch.nn.Parameter], with_grads: bool = True,
                 names: Optional[Sequence[str]] = None) -> None:
        params = list(params)
        if not params:
            raise ValueError("FlatArena needs at least one parameter")
        dtype, device = params[0].dtype, params[0].device
        for p in params:
            if p.dtype != dtype or p.device != device:
                raise ValueError("FlatArena parameters must share dtype and device")
            if not _is_dense(p):
                raise ValueError("FlatArena parameters must be dense (contiguous or channels_last)")
        self.params: List[torch.nn.Parameter] = params
        self.names = list(names) if names is not None else [f"p{i}" for i in range(len(params))]
        self.dtype, self.device = dtype, device
        self.offsets: List[int] = []
        cur = 0
        for p in params:
            off = _round_up(cur, ALIGN)
            self.offsets.append(off)
            cur = off + p.numel()
        self.numel = _round_up(max(cur, 1), TOTAL_ALIGN)
        self.param_flat = torch.zeros(self.numel, dtype=dtype, device=device)
        self.grad_flat = torch.zeros(self.numel, dtype=dtype, device=device) if with_grads else None
        self.grad_views: List[torch.Tensor] = []
        with torch.no_grad():
            for p, off in zip(params, self.offsets):
                view = self.view_of(self.param_flat, p, off)
                view.copy_(p.data)
                p.data = view
                if with_grads:
                    g = self.view_of(self.grad_flat, p, off)
                    if p.grad is not None:
                        g.copy_(p.grad)
                    p.grad = g
                    self.grad_views.append(g)

    @staticmethod
    def view_of(flat: torch.Tensor, p: torch.Tensor, off: int) -> torch.Tensor:
        return torch.as_strided(flat, p.shape, p.stride(), off)

    def region(self, i: int) -> slice:
        return slice(self.offsets[i], self.offsets[i] + self.params[i].numel())

    def views(self, flat: torch.Tensor) -> List[torch.Tensor]:
        """Per-parameter views (param shapes/strides) of any arena-shaped tensor."""
        return [self.view_of(flat, p, off) for p, off in zip(self.params, self.offsets)]

    def zeros_like_arena(self, dtype: Optional[torch.dtype] = None) -> torch.Tensor:
        return torch.zeros(self.numel, dtype=dtype or self.dtype, device=self.device)

    def reattach_grads(self) -> None:
        """Point every ``p.grad`` back at its arena view (after ``zero_grad(set_to_none)``)."""
        for p, g in zip(self.params, self.grad_views):
            if p.grad is None or p.grad.data_ptr() != g.data_ptr():
                with torch.no_grad():
                    if p.grad is not None:
                        g.copy_(p.grad)
                    else:
                        g.zero_()
                p.grad = g

    def relayout(self, order: Sequence[int], extra: Sequence[torch.Tensor] = ()) -> "ArenaPermutation":
        """Re-home the parameters in ``order`` (indices into ``self.params``).

        Parameter values and gradients move with their parameters; ``extra`` arena-shaped
        tensors (optimizer state) are permuted and returned through the permutation object.
        """
        order = list(order)
        if sorted(order) != list(range(len(self.params))):
            raise ValueError("relayout order must be a permutation of the parameter indices")
        old_offsets, old_params = list(self.offsets), list(self.params)
        old_param_flat, old_grad_flat = self.param_flat, self.grad_flat
        new = FlatArena.__new__(FlatArena)
        new.params = [old_params[i] for i in order]
        new.names = [self.names[i] for i in order]
        new.dtype, new.device = self.dtype, self.device
        new.offsets, cur = [], 0
        for p in new.params:
            off = _round_up(cur, ALIGN)
            new.offsets.append(off)
            cur = off + p.numel()
        new.numel = _round_up(max(cur, 1), TOTAL_ALIGN)
        perm = ArenaPermutation(old_offsets, new.offsets, order, [p.numel() for p in old_params], new.numel)
        new.param_flat = perm.apply(old_param_flat)
        new.grad_flat = perm.apply(old_grad_flat) if old_grad_flat is not None else None
        new.grad_views = []
        for p, off in zip(new.params, new.offsets):
            p.data = FlatArena.view_of(new.param_flat, p, off)
            if new.grad_flat is not None:
                g = FlatArena.view_of(new.grad_flat, p, off)
                p.grad = g
                new.grad_views.append(g)
        self.__dict__.update(new.__dict__)
        perm.extra = [perm.apply(t) for t in extra]
        return perm


class ArenaPermutation:
    def __init__(self, old_offsets, new_offsets, order, numels, new_numel) -> None:
        self.old_offsets, self.new_offsets, self.order = old_offsets, new_offsets, order
        self.numels, self.new_numel = numels, new_numel
        self.extra: List[torch.Tensor] = []

    @torch.no_grad()
    def apply(self, old: torch.Tensor) -> torch.Tensor:
        new = torch.zeros(self.new_numel, dtype=old.dtype, device=old.device)
        for j, i in enumerate(self.order):
            n = self.numels[i]
            new[self.new_offsets[j]:self.new_offsets[j] + n].copy_(
                old[self.old_offsets[i]:self.old_offsets[i] + n])
        return new


class BufferArena:
    """Module buffers (BN running stats, counters) re-homed into one flat buffer per dtype,
    so the per-step rank-0 buffer broadcast is one collective per
    dtype instead of one per tensor."""

    def __init__(self, module: torch.nn.Module) -> None:
        groups: Dict[torch.dtype, List] = {}
        for mod_name, mod in module.named_modules():
            for name, buf in list(mod._buffers.items()):
                if buf is None:
                    continue
                groups.setdefault(buf.dtype, []).append((mod, name, buf))
        self.flats: Dict[torch.dtype, torch.Tensor] = {}
        for dtype, items in groups.items():
            total = sum(_round_up(b.numel(), 4) for _, _, b in items)
            device = items[0][2].device
            flat = torch.zeros(max(total, 1), dtype=dtype, device=device)
            off = 0
            with torch.no_grad():
                for mod, name, buf in items:
                    view = torch.as_strided(flat, buf.shape, buf.stride() if _is_dense(buf) else
                                            torch.empty(buf.shape).stride(), off)
                    view.copy_(buf)
                    mod._buffers[name] = view
                    off += _round_up(buf.numel(), 4)
            self.flats[dtype] = flat

    def __len__(self) -> int:
        return len(self.flats)

    def tensors(self) -> List[torch.Tensor]:
        return list(self.flats.values())
