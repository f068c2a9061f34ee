"""Side HIP stream for off-critical-path backward work.

The backward of a convolution network is a chain  dgrad(L) -> BN bwd(L-1) ->
dgrad(L-1) -> ...  in which every grad-weight GEMM hangs off to the side: its
result is read only by the optimizer.  On MI355X the chain alternates
compute-bound MFMA GEMMs with memory-bound BatchNorm passes (~20% of an fp32
ResNet-50 step at HBM speed); issuing the grad-weight GEMMs on a second HIP
stream lets the hardware co-schedule their workgroups with the BN passes and
the grad-input GEMMs instead of running everything back to back.

Contract (ops/conv1x1.py, parallel/distributed_optimizer.py):

* ``fork(device)``: the side stream waits for everything issued so far on the
  current stream and is returned (the caller issues work under
  ``torch.cuda.stream(side)`` and ``record_stream``s the tensors it reads);
  the first fork of a backward pass queues an autograd callback that makes the
  calling stream wait on the side stream when the backward pass ends, so
  ``loss.backward()`` returns with all side work ordered before anything the
  caller issues next;
* ``join(device, stream)``: ``stream`` (default: current) waits on the side
  stream -- consumers that read gradients mid-backward (a bucket launch on the
  communication stream) call it first.

``GKSGD_WGRAD_STREAM``: ``0`` (default) never forks, ``1`` always; never
during HIP-graph capture.  Measured on MI355X, fp32 ResNet-50 bs512
(bench/stream_probe.py): 146.0 ms/step inline vs 147.8 ms with the side
stream, and 2x the reserved memory; bf16 41.0 vs 41.8 ms.  Most likely cause
(not traced): the persistent GEMM grids keep the CUs' register files and LDS
occupied, so a BN pass issued on the other stream finds few free wave slots
until the GEMM drains and little actually runs concurrently.  At bs32 the
grids are small and the fork usually pays (13.38 -> 13.21 ms/step, r4c6;
12.85 vs 13.15 / 13.06 off in an interleaved A/B, r4c34) but one of the two
forked runs of that A/B took 17.1 ms/step -- not root-caused, so the small-batch
``auto`` mode of round 4 was removed (round 5) and the fork is opt-in only.
The reference batch now replays as one HIP graph on one GPU anyway
(bench.py ``--ref-graph``), where the fork does not apply (below).  Inside a captured HIP graph
(``GKSGD_WGRAD_STREAM_GRAPH=1`` lifts the capture exclusion) the forked
grad-weights become parallel graph branches and the bs32 step DOUBLES: 23.2 /
23.8 ms against 12.59 / 12.59 inline, interleaved A/B/A/B (r5c8) -- the graph
executor's cross-branch synchronisation costs more than the overlap gains, so
the graph path stays single-stream.  MIOpen grad-weights on the side stream were
worse still (532 ms/step: its handle and workspace follow the stream), so a
fork only ever carries a HIP-kernel choice.
"""
from __future__ import annotations

import os
from typing import Dict, Optional

import torch

_side: Dict[int, "torch.cuda.Stream"] = {}
_pending: Dict[int, bool] = {}
_callback_queued: Dict[int, bool] = {}


def enabled(device: torch.device) -> bool:
    """Fork this convolution's grad-weight onto the side stream?"""
    if device.type != "cuda":
        return False
    if torch.cuda.is_current_stream_capturing() and os.environ.get("GKSGD_WGRAD_STREAM_GRAPH", "0") != "1":
        return False
    return os.environ.get("GKSGD_WGRAD_STREAM", "0") == "1"


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


def fork(device) -> "torch.cuda.Stream":
    i = _index(device)
    side = side_stream(i)
    side.wait_stream(torch.cuda.current_stream(i))
    _pending[i] = True
    if not _callback_queued.get(i):
        _callback_queued[i] = True
        main = torch.cuda.current_stream(i)

        def _end_of_backward():
            _callback_queued[i] = False
            join(i, main)
        torch.autograd.Variable._execution_engine.queue_callback(_end_of_backward)
    return side


def join(device=None, stream: Optional["torch.cuda.Stream"] = None) -> None:
    """``stream`` (default: the current stream) waits on the side stream's work."""
    if not _pending:
        return
    i = _index(device if device is not None else torch.device("cuda"))
    if not _pending.get(i):
        return
    target = stream if stream is not None else torch.cuda.current_stream(i)
    target.wait_stream(_side[i])
    if stream is None or stream == torch.cuda.current_stream(i):
        _pending[i] = False


def pending(device=None) -> bool:
    if not _pending:
        return False
    return bool(_pending.get(_index(device if device is not None else torch.device("cuda"))))
