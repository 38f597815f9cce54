"""Gradient bucket planning.

Same policy as the reference's inherited DDP reducer:
walk the parameters in gradient-ready order (reverse definition order before the first
backward, the observed order after it), close a bucket once its byte size reaches the
current cap, and use a small first cap (1 MiB) so the first all-reduce starts early in
backward, then the regular cap (25 MiB).  ``assign_buckets`` reproduces
``torch.distributed._compute_bucket_assignment_by_size`` for one dtype (tested).

Bucket caps are a first-class tuning knob on MI355X: an all-reduce over 8 GPUs on 7
point-to-point xGMI links wants per-channel chunks past the latency knee, so the bench
sweeps caps rather than assuming NVSwitch-era defaults.

Tail cap (``last_bucket_mb``, not in torch DDP): the bucket that becomes ready LAST can not
overlap any backward compute - its all-reduce is exposed by construction.  With the plain
policy it is whatever is left over (ResNet-50: the stem + layer1, 9.3 MiB; ViT-B/16: the
patch embedding, class token and position embedding), so the plan closes the longest
suffix of the ready order that fits the tail cap (at least one tensor) as its own bucket:
the tensors before it are reduced while the last layers' backward still runs, and only a
small, latency-bound collective is left after backward (docs/DESIGN.md §3.3).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Sequence

MiB = 1024 * 1024


def assign_buckets(sizes_bytes: Sequence[int], caps_bytes: Sequence[int]) -> List[List[int]]:
    """Indices of ``sizes_bytes`` grouped into buckets (input order preserved)."""
    buckets: List[List[int]] = []
    cur: List[int] = []
    cur_size = 0
    cap_i = 0
    for i, s in enumerate(sizes_bytes):
        cur.append(i)
        cur_size += s
        if cur_size >= caps_bytes[cap_i]:
            buckets.append(cur)
            cur, cur_size = [], 0
            cap_i = min(cap_i + 1, len(caps_bytes) - 1)
    if cur:
        buckets.append(cur)
    return buckets


@dataclass
class BucketPlan:
    offsets: List[int]        # element offset of each bucket in the arena
    numels: List[int]         # elements per bucket (contiguous, includes alignment padding)
    param_bucket: List[int]   # bucket index of each arena parameter
    members: List[List[int]]  # arena parameter indices per bucket

    @property
    def num_buckets(self) -> int:
        return len(self.offsets)

    def sizes_mib(self, elem_bytes: int = 4) -> List[float]:
        return [n * elem_bytes / MiB for n in self.numels]


def tail_split(sizes_bytes: Sequence[int], last_cap_bytes: int) -> int:
    """Index where the tail bucket starts: the longest suffix whose bytes fit ``last_cap_bytes``
    (at least the last tensor).  ``len(sizes)`` (no split) when there is no tail cap, or when
    that suffix holds less than half the cap: then the tensors just before it are big ones
    whose gradients arrive at the very end too (ViT-B/16: the 2.25 MiB patch embedding ahead
    of the 3 KiB class token), splitting would only add a collective (measured:
    profiles/comm_model_r3.md)."""
    n = len(sizes_bytes)
    if last_cap_bytes <= 0 or n < 2:
        return n
    start, total = n - 1, sizes_bytes[-1]
    while start > 0 and total + sizes_bytes[start - 1] <= last_cap_bytes:
        start -= 1
        total += sizes_bytes[start]
    if total > last_cap_bytes or 2 * total < last_cap_bytes:
        return n
    return start


def assign_buckets_with_tail(sizes_bytes: Sequence[int], caps_bytes: Sequence[int],
                             last_cap_bytes: int = 0) -> List[List[int]]:
    """``assign_buckets`` over the prefix, then the tail (``tail_split``) as the last bucket."""
    cut = tail_split(sizes_bytes, last_cap_bytes)
    if cut <= 0 or cut >= len(sizes_bytes):
        return assign_buckets(sizes_bytes, caps_bytes)
    head = assign_buckets(sizes_bytes[:cut], caps_bytes)
    return head + [list(range(cut, len(sizes_bytes)))]


def plan_for_arena(arena, bucket_cap_mb: float = 25.0, first_bucket_mb: float = 1.0,
                   last_bucket_mb: float = 0.0) -> BucketPlan:
    """Partition ``arena`` (already laid out in ready order) into contiguous buckets."""
    elem = arena.param_flat.element_size()
    sizes = [p.numel() * elem for p in arena.params]
    caps = [max(1, int(first_bucket_mb * MiB)), max(1, int(bucket_cap_mb * MiB))]
    groups = assign_buckets_with_tail(sizes, caps, int(max(0.0, last_bucket_mb) * MiB))
    offsets, numels, param_bucket = [], [], [0] * len(arena.params)
    for b, members in enumerate(groups):
        start = arena.offsets[members[0]]
        for i in members:
            param_bucket[i] = b
        offsets.append(start)
    for b in range(len(groups)):
        end = offsets[b + 1] if b + 1 < len(groups) else arena.numel
        numels.append(end - offsets[b])
    return BucketPlan(offsets, numels, param_bucket, groups)
