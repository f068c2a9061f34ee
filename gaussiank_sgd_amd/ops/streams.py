"""Side HIP stream for off-critical-path backward work.

The backward of a convolution network is a chain  dgrad(L) -> BN bwd(L-1) ->
dgrad(L-1) -> ...  in which every grad-weight GEMM hangs off to the side: its
result is read only by the optimizer.  On MI355X the chain alternates
compute-bound MFMA GEMMs with memory-bound BatchNorm passes (a quarter of an
fp32 ResNet-50 step, a third of a bf16 one, at HBM speed); issuing the
grad-weight GEMMs on a second HIP stream lets the hardware co-schedule their
workgroups with the BN passes and the grad-input GEMMs instead of running
everything back to back.

Contract (ops/conv1x1.py, parallel/distributed_optimizer.py):

* ``fork(device)``: the side stream waits for everything issued so far on the
  current stream and is returned (the caller issues work under
  ``torch.cuda.stream(side)`` and then ``hold``s the tensors it reads);
  the first fork of a backward pass queues an autograd callback that makes the
  calling stream wait on the side stream when the backward pass ends, so
  ``loss.backward()`` returns with all side work ordered before anything the
  caller issues next;
* ``hold(device, *tensors)``: keeps the tensors the side work reads alive
  until that work has completed (its event queried done) or the allocating
  stream has been joined to the side stream -- whichever the host sees first;
* ``join(device, stream)``: ``stream`` (default: current) waits on the side
  stream -- consumers that read gradients mid-backward (a bucket launch on the
  communication stream) call it first.

Tensor lifetime: NOT ``record_stream``.  With ``record_stream`` the caching
allocator keeps a block freed on the main stream out of reuse until an event
it records at free time completes; the host runs a whole step ahead of the
GPU, so at each free that event is still pending and the block is dropped
from reuse, and the allocator grows by every forked tensor of a step until
the device is full and every allocation retries (a full synchronise + cache
flush): fp32 ResNet-50 bs512 ran 475-492 ms/step instead of ~102 after ~10
steps (r6c28 / r6c30; ``bench/stream_probe.py``, which synchronises every step,
never saw it).  Holding Python references instead frees each block into the
main stream's pool only after the main stream has waited on the side stream
(or the side work is known complete), so reuse is stream-ordered and the
pool stays at the inline footprint plus the held tensors of one backward.

``GKSGD_WGRAD_STREAM``: ``1`` forks, ``0`` never forks (default: ``1``);
never during HIP-graph capture.  Measured on MI355X, same box interleaved
(r6c31, ``profiles/r06_wgrad_stream_ab.txt``): ResNet-50 bs512 fp32 5,243 /
5,231 img/s vs 5,073 / 5,054 inline (+3.4%; all of it from the Winograd
grad-weight, ``GKSGD_WGRAD_STREAM_WINO=0`` gives 5,073 / 5,061), bf16 13,372 /
13,363 vs 12,905 / 12,847 (+3.8%); LSTM bs128 +0.8%, BERT +0.2% (linear and
LSTM weight gradients, ops/linear.py / ops/lstm.py).  Inside a
captured HIP graph (``GKSGD_WGRAD_STREAM_GRAPH=1`` lifts the capture
exclusion) the forked grad-weights become parallel graph branches and the
bs32 step DOUBLES: 23.2 / 23.8 ms against 12.59 / 12.59 inline, interleaved
A/B/A/B (r5c8) -- the graph executor's cross-branch synchronisation costs more
than the overlap gains, so the graph path stays single-stream.  MIOpen
grad-weights on the side stream were worse still (532 ms/step: its handle and
workspace follow the stream), so a fork only ever carries a HIP-kernel choice.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Tuple

import torch

_side: Dict[int, "torch.cuda.Stream"] = {}
_pending: Dict[int, bool] = {}
_callback_queued: Dict[int, bool] = {}
# per device: (event recorded on the side stream after the work, tensors it reads)
_held: Dict[int, List[Tuple["torch.cuda.Event", tuple]]] = {}


def enabled(device: torch.device) -> bool:
    """Fork this convolution's grad-weight onto the side stream?"""
    if device.type != "cuda":
        return False
    if torch.cuda.is_current_stream_capturing() and os.environ.get("GKSGD_WGRAD_STREAM_GRAPH", "0") != "1":
        return False
    return os.environ.get("GKSGD_WGRAD_STREAM", "1") == "1"


# Forks of smaller grad-weights are not worth their host cost (an event query,
# a stream wait and an event record per fork): a step whose grad-weights are
# this small is launch-bound, and the fork made it slower and erratic -- ResNet-50
# at the reference's batch of 32, eager: 15.2 / 20.7 ms per step forked vs 14.5 /
# 15.9 inline (r6c32).  Every ResNet-50 bs512 grad-weight is >= 13 GFLOP, at bs32
# <= 7.4 GFLOP (BERT seq512 bs32 linears >= 19, LSTM bs20 12.6, VGG-16 bs128 >= 9.6).
# ``GKSGD_WGRAD_STREAM_MIN_GFLOP`` (default 8) sets the bound.


def worth(device: torch.device, flops: float) -> bool:
    """Fork a grad-weight of ``flops`` onto the side stream?  ``enabled`` and
    large enough to pay for the fork."""
    return flops >= float(os.environ.get("GKSGD_WGRAD_STREAM_MIN_GFLOP", "8")) * 1e9 and enabled(device)


def _index(device) -> int:
    d = torch.device(device)
    return d.index if d.index is not None else torch.cuda.current_device()


def side_stream(device) -> "torch.cuda.Stream":
    i = _index(device)
    s = _side.get(i)
    if s is None:
        s = torch.cuda.Stream(device=i)
        _side[i] = s
    return s


def _reap(i: int) -> None:
    """Release held tensors whose side work has completed (in issue order)."""
    h = _held.get(i)
    if h and torch.cuda.is_current_stream_capturing():
        return      # events recorded in a capture cannot be queried (GKSGD_WGRAD_STREAM_GRAPH=1)
    while h and h[0][0].query():
        h.pop(0)


def fork(device) -> "torch.cuda.Stream":
    i = _index(device)
    _reap(i)
    side = side_stream(i)
    side.wait_stream(torch.cuda.current_stream(i))
    _pending[i] = True
    if not _callback_queued.get(i):
        _callback_queued[i] = True
        main = torch.cuda.current_stream(i)

        def _end_of_backward():
            _callback_queued[i] = False
            join(i, main, release=True)
        torch.autograd.Variable._execution_engine.queue_callback(_end_of_backward)
    return side


def hold(device, *tensors: torch.Tensor) -> None:
    """Keep ``tensors`` (read by work just issued on the side stream) alive
    until that work is done or the allocating stream is joined."""
    i = _index(device)
    ev = torch.cuda.Event()
    ev.record(side_stream(i))
    _held.setdefault(i, []).append((ev, tensors))


def held(device=None) -> int:
    """Number of forked operations whose tensors are still held."""
    if not _held:
        return 0
    return len(_held.get(_index(device if device is not None else torch.device("cuda")), ()))


def join(device=None, stream: Optional["torch.cuda.Stream"] = None, release: bool = False) -> None:
    """``stream`` (default: the current stream) waits on the side stream's work.
    ``release``: ``stream`` is the one the held tensors were allocated on (the
    end-of-backward join), so they are dropped after its wait."""
    if not _pending:
        return
    i = _index(device if device is not None else torch.device("cuda"))
    if not _pending.get(i):
        return
    cur = torch.cuda.current_stream(i)
    target = stream if stream is not None else cur
    target.wait_stream(_side[i])
    if target == cur or release:
        _pending[i] = False
        # the held tensors were allocated on this stream: after its wait on the
        # side stream, reusing their blocks here is ordered after the side work
        _held.pop(i, None)


def pending(device=None) -> bool:
    if not _pending:
        return False
    return bool(_pending.get(_index(device if device is not None else torch.device("cuda"))))
