"""roctx ranges on the hot path (rocprofv3 --marker-trace / omnitrace).

Parity: the reference's per-group compress / all-reduce / update timers
(distributed_optimizer.py:522-540) only print averages; here every phase of
every bucket is also a named roctx range, so a rocprofv3 trace shows *when*
the host issued it next to the kernels it enqueued (compress / exchange /
decompress on the high-priority comm stream, overlapping backward on the
compute stream).

Off by default (zero cost: ``range`` returns a shared null context).  Enable
with ``GKSGD_ROCTX=1``.  The markers go through rocprofiler-sdk's roctx
(``librocprofiler-sdk-roctx.so``, what rocprofv3 intercepts), called with
ctypes (~1 us per call, no torch dispatcher in between); torch's bundled
roctx (``torch.cuda.nvtx``) is the fallback.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
from typing import Callable, Optional

_push: Optional[Callable[[bytes], int]] = None
_pop: Optional[Callable[[], int]] = None
_mark: Optional[Callable[[bytes], None]] = None
_enabled = False


def _load() -> bool:
    global _push, _pop, _mark
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    for name in (os.path.join(rocm, "lib", "librocprofiler-sdk-roctx.so.1"),
                 os.path.join(rocm, "lib", "librocprofiler-sdk-roctx.so"), "librocprofiler-sdk-roctx.so.1"):
        try:
            lib = ctypes.CDLL(name)
        except OSError:
            continue
        lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
        lib.roctxRangePushA.restype = ctypes.c_int
        lib.roctxRangePop.argtypes = []
        lib.roctxRangePop.restype = ctypes.c_int
        lib.roctxMarkA.argtypes = [ctypes.c_char_p]
        lib.roctxMarkA.restype = None
        _push, _pop, _mark = lib.roctxRangePushA, lib.roctxRangePop, lib.roctxMarkA
        return True
    try:
        import torch
        nv = torch.cuda.nvtx
        _push = lambda b: nv.range_push(b.decode())  # noqa: E731
        _pop = nv.range_pop
        _mark = lambda b: nv.mark(b.decode())  # noqa: E731
        return True
    except Exception:  # pragma: no cover
        return False


def enable(on: bool = True) -> bool:
    """Turn the ranges on / off at run time; returns whether they are on."""
    global _enabled
    _enabled = bool(on) and (_push is not None or _load())
    return _enabled


def enabled() -> bool:
    return _enabled


class _Range:
    __slots__ = ("name",)

    def __init__(self, name: str):
        self.name = name.encode()

    def __enter__(self):
        _push(self.name)
        return self

    def __exit__(self, *exc):
        _pop()
        return False


_NULL = contextlib.nullcontext()


def range(name: str):  # noqa: A001 - mirrors roctx naming
    """``with trace.range("gk/b0/compress"): ...`` -- a roctx range when enabled."""
    return _Range(name) if _enabled else _NULL


def push(name: str) -> None:
    if _enabled:
        _push(name.encode())


def pop() -> None:
    if _enabled:
        _pop()


def mark(name: str) -> None:
    if _enabled:
        _mark(name.encode())


if os.environ.get("GKSGD_ROCTX", "0") == "1":
    enable(True)
