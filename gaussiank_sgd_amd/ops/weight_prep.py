"""Per-step batched weight re-layouts (csrc/kernels/prep.hip).

The convolution kernels read their weights in kernel-specific layouts that
must be rebuilt whenever the weights change, i.e. every step: the Winograd
filter tiles of the forward and of the flipped grad-input filter, the
transposed [C][K] weight of a 1x1 grad-input GEMM and the per-tap transposed
weight of a non-Winograd 3x3 grad-input.  Built at each call site that is one
small launch per layer and direction -- 63 launches, ~0.4 ms of a 13 ms
ResNet-50 step at the reference's batch of 32.

``WeightPrep`` (one per trainer) remembers every re-layout the model's
convolutions asked for, and ``with prep.step():`` (``DLTrainer.train`` /
``test`` wrap their forward + backward in it) rebuilds ALL of them in one
launch at the start of the step; inside the scope the call sites receive the
prepared buffers (a backward function re-enters the scope its forward
recorded, ``use()``: autograd runs a GPU backward on its own thread).  A re-layout asked for the first time (or while a HIP graph
is being captured, when the descriptor table cannot be re-uploaded) is built
by the call site itself and registered for the next step.  Outside a scope
nothing is cached, so a weight update between scopes can never be missed.

Only weights that live in persistent storage (the parameter itself or its
bf16-shadow view) are registered; the registry holds references to them.
"""
from __future__ import annotations

import contextlib
import os
import struct
import threading
from typing import Callable, Dict, List, Optional, Tuple

import torch

KIND_WINO, KIND_WINO_FLIP, KIND_T32, KIND_T16, KIND_WINO_X6, KIND_WINO_X6_FLIP = 0, 1, 2, 3, 4, 5
_DESC = struct.Struct("<QQqqqiiii")      # gk::PrepDesc (gk_kernels.h): 56 bytes
_MAX_DESCS = 512                          # prep.hip kMaxDescs (descriptor table in LDS)
_tls = threading.local()
# GKSGD_WEIGHT_PREP=0: every call site builds its re-layout itself (A/B, tests)
ENABLED = os.environ.get("GKSGD_WEIGHT_PREP", "1") != "0"


def _ops():
    return torch.ops.gksgd


class _Entry:
    __slots__ = ("src", "dst", "descs", "ready")

    def __init__(self, src: torch.Tensor, dst: torch.Tensor, descs: List[tuple]):
        self.src, self.dst, self.descs, self.ready = src, dst, descs, False


class WeightPrep:
    """Registry of one model's per-step weight re-layouts."""

    def __init__(self):
        self.entries: Dict[tuple, _Entry] = {}
        self._tables: List[Tuple[torch.Tensor, int, int]] = []   # (device table, ndesc, blocks) per launch
        self._built_for = 0        # number of entries the current tables cover
        self._keep: List[torch.Tensor] = []   # earlier tables: a captured graph may still replay them
        self.active = False
        self.launches = 0          # batched launches issued (tests / diagnostics)

    # -- table --------------------------------------------------------------
    def _build(self, device: torch.device) -> None:
        descs = [d for e in self.entries.values() for d in e.descs]
        self._keep += [t for t, _, _ in self._tables]
        self._tables = []
        for i in range(0, len(descs), _MAX_DESCS):
            part = descs[i:i + _MAX_DESCS]
            packed = bytearray()
            begin = 0
            for kind, src, dst, ld_in, ld_out, R, S in part:
                packed += _DESC.pack(src, dst, ld_in, ld_out, begin, kind, R, S, (S + 63) // 64)
                begin += int(_ops().weight_prep_blocks(kind, R, S))
            host = torch.frombuffer(packed, dtype=torch.uint8)
            self._tables.append((host.to(device), len(part), begin))
        self._built_for = len(self.entries)

    def _launch(self, device: torch.device) -> None:
        capturing = torch.cuda.is_current_stream_capturing()
        if self._built_for != len(self.entries) and not capturing:
            self._build(device)
        if not self._tables:
            return
        for t, n, blocks in self._tables:
            _ops().weight_prep(t, n, blocks)
        self.launches += 1
        covered = list(self.entries.values())[: self._built_for]
        for e in covered:
            e.ready = True

    @contextlib.contextmanager
    def step(self, device: Optional[torch.device] = None):
        """Scope of one training (or evaluation) step: every registered
        re-layout is rebuilt from the current weights in one launch here, and
        the call sites inside reuse the buffers."""
        prev = getattr(_tls, "cur", None)
        if not ENABLED:
            yield self
            return
        if self.entries and device is not None and device.type == "cuda":
            self._launch(device)
        self.active = True
        _tls.cur = self
        try:
            yield self
        finally:
            _tls.cur = prev
            self.active = False
            for e in self.entries.values():
                e.ready = False

    # -- call sites ---------------------------------------------------------
    def acquire(self, key: tuple, src: torch.Tensor, make_dst: Callable[[], torch.Tensor],
                descs_of: Callable[[torch.Tensor], List[tuple]], fill: Callable[[torch.Tensor], None]) -> torch.Tensor:
        e = self.entries.get(key)
        if e is None:
            dst = make_dst()
            if torch.cuda.is_current_stream_capturing():
                fill(dst)              # not registered: the table cannot be re-uploaded inside a capture
                return dst
            e = self.entries[key] = _Entry(src, dst, descs_of(dst))
        if not e.ready:
            fill(e.dst)
            e.ready = True
        return e.dst


def current() -> Optional[WeightPrep]:
    """The WeightPrep of the step scope running on this thread, if any."""
    return getattr(_tls, "cur", None)


@contextlib.contextmanager
def use(prep: Optional[WeightPrep]):
    """Make ``prep`` current on this thread while its step scope is open: the
    autograd engine runs a GPU backward on its own device thread, so a
    backward function re-enters the scope its forward recorded."""
    prev = getattr(_tls, "cur", None)
    _tls.cur = prep if (prep is not None and prep.active) else None
    try:
        yield
    finally:
        _tls.cur = prev


def _key(kind: str, w: torch.Tensor) -> tuple:
    return (kind, w.data_ptr(), tuple(w.shape), w.dtype)


def wino_filter(w: torch.Tensor, flip: bool, persistent: bool) -> torch.Tensor:
    """Winograd filter tiles of the fp32 3x3 weight ``w`` ([K, C, 3, 3]
    channels-last; ``flip``: of the grad-input filter) -- gksgd.wino_weights."""
    K, C = w.shape[0], w.shape[1]

    def make():
        return torch.empty(16 * K * C, dtype=torch.float32, device=w.device)

    def fill(u):
        _ops().wino_weights(w, u, flip)
    p = current()
    if p is None or not persistent:
        u = make()
        fill(u)
        return u
    Co, Ci = (C, K) if flip else (K, C)
    kind = KIND_WINO_FLIP if flip else KIND_WINO
    return p.acquire(_key("wino%d" % int(flip), w), w, make,
                     lambda u: [(kind, w.data_ptr(), u.data_ptr(), 0, 0, Co, Ci)], fill)


def wino_x6_filter(w: torch.Tensor, flip: bool, persistent: bool) -> torch.Tensor:
    """bf16x6 Winograd filter planes of the fp32 3x3 weight ``w`` ([K, C, 3, 3]
    channels-last; ``flip``: of the grad-input filter) -- gksgd.wino_x6_weights."""
    K, C = w.shape[0], w.shape[1]

    def make():
        return torch.empty(48 * K * C, dtype=torch.bfloat16, device=w.device)

    def fill(u3):
        _ops().wino_x6_weights(w, u3, flip)
    p = current()
    if p is None or not persistent:
        u3 = make()
        fill(u3)
        return u3
    Co, Ci = (C, K) if flip else (K, C)
    kind = KIND_WINO_X6_FLIP if flip else KIND_WINO_X6
    return p.acquire(_key("wx6%d" % int(flip), w), w, make,
                     lambda u3: [(kind, w.data_ptr(), u3.data_ptr(), 0, 0, Co, Ci)], fill)


def transposed_1x1(w: torch.Tensor, persistent: bool) -> torch.Tensor:
    """[C, K] contiguous transpose of the 1x1 weight ``w`` ([K, C, 1, 1])."""
    K, C = w.shape[0], w.shape[1]

    def make():
        return torch.empty(C, K, dtype=w.dtype, device=w.device)

    def fill(out):
        out.copy_(w.reshape(K, C).t())
    p = current()
    if p is None or not persistent or w.dtype not in (torch.float32, torch.bfloat16) or not w.is_contiguous():
        out = make()
        fill(out)
        return out
    kind = KIND_T32 if w.dtype == torch.float32 else KIND_T16
    return p.acquire(_key("t1", w), w, make,
                     lambda out: [(kind, w.data_ptr(), out.data_ptr(), C, K, K, C)], fill)


def flipped_3x3(w: torch.Tensor, persistent: bool) -> torch.Tensor:
    """Grad-input filter W'[c][kh][kw][k] = W[k][2-kh][2-kw][c] of a 3x3
    weight ``w`` ([K, C, 3, 3] channels-last), channels-last [C, K, 3, 3]."""
    K, C = w.shape[0], w.shape[1]

    def make():
        return torch.empty((C, K, 3, 3), dtype=w.dtype, device=w.device, memory_format=torch.channels_last)

    def fill(out):
        out.copy_(w.flip(2, 3).transpose(0, 1))
    p = current()
    if p is None or not persistent or w.dtype not in (torch.float32, torch.bfloat16) or \
            not w.is_contiguous(memory_format=torch.channels_last):
        out = make()
        fill(out)
        return out
    kind = KIND_T32 if w.dtype == torch.float32 else KIND_T16
    es = w.element_size()

    def descs(out):
        # tap t of the output takes tap 8 - t of the input, transposed (k, c) -> (c, k)
        return [(kind, w.data_ptr() + (8 - t) * C * es, out.data_ptr() + t * K * es, 9 * C, 9 * K, K, C)
                for t in range(9)]
    return p.acquire(_key("f3", w), w, make, descs, fill)
