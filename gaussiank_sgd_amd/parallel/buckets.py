"""Flat parameter / gradient arenas and gradient buckets.

Reference behaviour (distributed_optimizer.py:112-134, 312-401): parameters
are grouped in REVERSE registration order until the cumulative element count
reaches ``threshold``; each group owns a freshly allocated flat buffer; every
hook COPIES the gradient into it and, after the exchange, ``p.grad`` is
re-pointed into the buffer.

MI355X design: one flat fp32 arena per role (weights, gradients, residuals,
momentum), laid out bucket by bucket in backward order.  ``p.data`` and
``p.grad`` are views into the arenas from the start, so autograd accumulates
straight into the bucket (no pack copy, K10 eliminated), a bucket is a
contiguous slice the HIP kernels stream with 16-byte loads, and the fused
optimizer updates the whole model in one launch.  Every tensor is padded to
64 elements (256 B) so each view is 256-byte aligned (MIOpen / hipBLASLt keep
their aligned fast paths); padding stays zero and is excluded from the
statistics (``n_stats``) and from ``k``.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import torch

ALIGN = 64


def _pad(n: int, a: int = ALIGN) -> int:
    return (n + a - 1) // a * a


def group_with_threshold(keys: Sequence[str], sizes: Dict[str, int], threshold: int) -> List[List[str]]:
    """Reference grouping rule (distributed_optimizer.py:112-134), reverse order."""
    groups: List[List[str]] = []
    group: List[str] = []
    sub = 0
    for k in list(keys)[::-1]:
        sub += sizes[k]
        group.append(k)
        if sub >= threshold:
            groups.append(group)
            group = []
            sub = 0
    if group:
        groups.append(group)
    return groups


@dataclass
class Bucket:
    index: int
    name: str
    keys: List[str]
    start: int                  # element offset in the arenas
    span: int                   # padded length (multiple of ALIGN)
    numel: int                  # real elements (reference's merged-buffer numel)
    offsets: List[int] = field(default_factory=list)   # per-key offset inside the bucket
    params: List[torch.nn.Parameter] = field(default_factory=list)
    ready: int = 0
    launched: bool = False
    # filled by the exchange engine
    k: int = 1
    k_cap: int = 1
    density: float = 1.0
    bufs: object = None
    gathered: Optional[torch.Tensor] = None
    done_event: object = None
    extra: dict = field(default_factory=dict)

    def slice(self, arena: torch.Tensor) -> torch.Tensor:
        return arena[self.start:self.start + self.span]


def _dense_strides_ok(p: torch.Tensor) -> bool:
    return p.is_contiguous() or (p.dim() == 4 and p.is_contiguous(memory_format=torch.channels_last))


class GradArena:
    """Owns the arenas and the bucket table of one model."""

    def __init__(self, named_parameters: Sequence[Tuple[str, torch.nn.Parameter]], groups: List[List[str]],
                 with_residuals: bool = True):
        self.named = {k: v for k, v in named_parameters}
        params = [p for _, p in named_parameters]
        if not params:
            raise ValueError("no parameters")
        dev = params[0].device
        for k, p in self.named.items():
            if p.device != dev:
                raise ValueError("all parameters must live on one device (%s is on %s)" % (k, p.device))
            if p.dtype != torch.float32:
                raise ValueError("fp32 master parameters required (%s is %s); use bf16 autocast for compute"
                                 % (k, p.dtype))
        self.device = dev
        self.buckets: List[Bucket] = []
        self.key_to_bucket: Dict[str, int] = {}
        self.key_offset: Dict[str, int] = {}
        off = 0
        for bi, g in enumerate(groups):
            b = Bucket(index=bi, name=":".join(g), keys=list(g), start=off, span=0, numel=0)
            inner = 0
            for k in g:
                p = self.named[k]
                b.offsets.append(inner)
                b.params.append(p)
                self.key_to_bucket[k] = bi
                self.key_offset[k] = off + inner
                inner += _pad(p.numel())
                b.numel += p.numel()
            b.span = inner
            off += inner
            self.buckets.append(b)
        self.total = off
        self.weights = torch.zeros(self.total, dtype=torch.float32, device=dev)
        self.grads = torch.zeros(self.total, dtype=torch.float32, device=dev)
        self.residuals = torch.zeros(self.total, dtype=torch.float32, device=dev) if with_residuals else None
        self.momentum: Optional[torch.Tensor] = None
        self.grad_views: Dict[str, torch.Tensor] = {}
        self.weight_views: Dict[str, torch.Tensor] = {}
        with torch.no_grad():
            for k, p in self.named.items():
                if k not in self.key_offset:
                    continue
                o = self.key_offset[k]
                src = p.data if _dense_strides_ok(p.data) else p.data.contiguous()
                wv = self.weights.as_strided(src.shape, src.stride(), o)
                wv.copy_(src)
                gv = self.grads.as_strided(src.shape, src.stride(), o)
                if p.grad is not None:
                    gv.copy_(p.grad)
                p.data = wv
                p.grad = gv
                p._gk_arena = self.weights
                self.grad_views[k] = gv
                self.weight_views[k] = wv

    # ------------------------------------------------------------------
    def view_of(self, arena: torch.Tensor, key: str) -> torch.Tensor:
        p = self.named[key]
        return arena.as_strided(p.shape, p.data.stride(), self.key_offset[key])

    def ensure_momentum(self, fill: float = 0.0) -> torch.Tensor:
        if self.momentum is None:
            self.momentum = torch.full((self.total,), fill, dtype=torch.float32, device=self.device)
        return self.momentum

    def check_grad(self, key: str, p: torch.nn.Parameter) -> None:
        """Re-attach p.grad to the arena if someone replaced it (e.g. zero_grad(set_to_none))."""
        gv = self.grad_views[key]
        g = p.grad
        if g is None:
            p.grad = gv
        elif g.data_ptr() != gv.data_ptr():
            with torch.no_grad():
                gv.copy_(g)
            p.grad = gv

    def reattach(self) -> None:
        for k, p in self.named.items():
            if k in self.grad_views:
                if p.grad is None or p.grad.data_ptr() != self.grad_views[k].data_ptr():
                    self.check_grad(k, p)
                if p.data.data_ptr() != self.weight_views[k].data_ptr():
                    with torch.no_grad():
                        self.weight_views[k].copy_(p.data)
                    p.data = self.weight_views[k]

    def segments(self, group_of_key: Dict[str, int]) -> List[Tuple[int, int, int, int]]:
        """(start, padded numel, group id, segment id) per tensor, for chunk tables."""
        segs = []
        sid = 0
        for b in self.buckets:
            for k, o in zip(b.keys, b.offsets):
                segs.append((b.start + o, _pad(self.named[k].numel()), group_of_key.get(k, 0), sid))
                sid += 1
        return segs
