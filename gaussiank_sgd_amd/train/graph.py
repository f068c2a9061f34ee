"""Whole-step HIP-graph capture of a training iteration.

Small per-GPU batches (the reference's ResNet-20 bs32 runs,
logs/results/SGD_32_0.0001_topk) are launch-bound on MI355X: a step is a few
hundred short kernels.  ``GraphedStep`` captures ONE complete iteration --
forward, backward, bucket hooks -> fused Gaussian-k compression + exchange +
decompression on the high-priority side stream, fused SGD update -- into a
HIP graph (``torch.cuda.CUDAGraph`` is hipGraph on ROCm) and replays it; each
call first copies the next batch into the graph's static input buffers, so
every replay trains on fresh data.

What the graph freezes: host-side scalars read at capture time -- the
compression density / k, momentum flags.  NOT frozen: the learning rate (the
fused SGD kernel multiplies the captured lr by a device scalar,
``opt._lr_mult``, refreshed from the host schedule before every replay), the
compressor seeds (random-k / DGC sampling read one int32 device word per
bucket, ``opt.refresh_device_seeds``, so every replay draws new indices) and
the dropout masks (the attention / add+LayerNorm kernels mix a per-device
replay word, ``ops.graph_seed_word``, into their seed).  ``recapture()`` rebuilds the graph when the density schedule moves
(epoch boundary with the reference's density warm-up).
Single stream: the optimizer's side (compression / exchange) stream is
dropped for the captured step -- a hipGraph with cross-stream branches
replays on ROCm 7 at ~10 ms per ResNet-20 bs32 step (the runtime resolves
the branch edges from the host), the same step captured on one stream at
1.43 ms (eager: 4.9 ms; scripts/gpurun/graph_probe.sh, profiles/r02_graph_probe.txt).
Overlap buys nothing in a replay whose launches are already on the device.
``GKSGD_GRAPH_COMM_STREAM=1`` keeps the side stream.
Recurrent models (the PTB LSTM) carry their hidden state across steps in
static buffers: the captured step reads them as the initial state and
copies the final state back into them (``reset_hidden()`` zeroes them, e.g.
at an epoch start as the reference re-initialises its hidden state,
dist_trainer.py:64-67).
Requirements: every op of the step is stream-ordered without host syncs
(true for the DistributedOptimizer / fused kernels of this package) and the
autotuned convolution choices are cached by the eager warm-up steps.
"""
from __future__ import annotations

import os
from typing import Callable, Optional

import torch


def _clone(v):
    if torch.is_tensor(v):
        return v.clone()
    if isinstance(v, (tuple, list)):
        return type(v)(_clone(e) for e in v)
    return v


def _copy(dst, src) -> None:
    if torch.is_tensor(dst):
        dst.copy_(src, non_blocking=True)
    elif isinstance(dst, (tuple, list)):
        for a, b in zip(dst, src):
            _copy(a, b)


class GraphedStep:
    def __init__(self, trainer, opt, clip: Optional[float] = None, warmup: int = 3):
        self.trainer = trainer
        self.opt = opt
        self.clip = clip
        self.warmup = warmup
        d = trainer.data_iter()
        self.x = d[0].clone()
        self.y = _clone(d[1])
        # recurrent state (LSTM): static (h, c) the captured step reads and rewrites
        self.hidden = None
        if getattr(trainer, "dnn", None) == "lstm":
            self.hidden = tuple(v.detach().clone() for v in trainer.net.init_hidden(self.x.shape[1]))
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.lr0 = None            # lr baked into the captured update
        self.density = None
        self.captures = 0
        self.replays = 0
        dev = self.x.device
        self.mult = torch.ones(1, dtype=torch.float32, device=dev)
        cs = getattr(opt, "_comm_stream", None)
        if cs is not None and os.environ.get("GKSGD_GRAPH_COMM_STREAM", "0") != "1":
            torch.cuda.current_stream(dev).wait_stream(cs)   # drain the side stream, then go single-stream
            opt._comm_stream = None

    def _body(self) -> None:
        t, opt = self.trainer, self.opt
        t._graph_body = True    # epoch boundaries / log lines are this class's job (no host syncs in a capture)
        try:
            self._step(t, opt)
        finally:
            t._graph_body = False

    def _step(self, t, opt) -> None:
        opt.zero_grad()
        if self.hidden is not None:
            _, new = t.train(1, data=(self.x, self.y), hidden=self.hidden)
            with torch.no_grad():        # after the backward: the saved initial state is consumed
                for dst, src in zip(self.hidden, new):
                    dst.copy_(src.detach())
        else:
            t.train(1, data=(self.x, self.y))
        if self.clip is not None:
            opt.synchronize()
            opt.clip_grad_norm_(self.clip)
        t.update_model()

    def reset_hidden(self) -> None:
        """Zero the carried recurrent state (stream-ordered; no recapture)."""
        if self.hidden is not None:
            for v in self.hidden:
                v.zero_()

    def _density(self):
        f = getattr(self.opt, "get_current_density", None)
        return f() if f is not None else None

    def recapture(self) -> None:
        self.opt._lr_mult = None             # eager warm-up steps use the plain lr
        # warm-up on the current stream by default: MIOpen picked naive fallback
        # solvers on a fresh side stream (ResNet-20 bs1024: 16.8 ms/step replayed
        # vs 5.9 ms with this warm-up; eager 4.8-5.1 ms, profiles/r02_graph_probe.txt)
        if os.environ.get("GKSGD_GRAPH_WARMUP_SIDE", "0") == "1":
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(self.warmup):      # eager warm-up on a side stream (allocator / autotune caches)
                    self._body()
            torch.cuda.current_stream().wait_stream(s)
        else:
            for _ in range(self.warmup):
                self._body()
        self.mult.fill_(1.0)
        self.opt._lr_mult = self.mult
        # compressor seeds and dropout masks: device words the captured kernels
        # read at replay time (refreshed before every replay below)
        if hasattr(self.opt, "enable_device_seeds"):
            self.opt.enable_device_seeds()
        from .. import ops
        ops.graph_seed_word(self.x.device)
        self.graph = torch.cuda.CUDAGraph()
        self.opt._graph_sel = []
        it0 = getattr(self.opt, "train_iter", None)
        with torch.cuda.graph(self.graph):
            self._body()
        self.trainer.train_iter -= 1          # capture records the step; it did not run it
        if it0 is not None:
            self.opt.train_iter = it0         # (the captured synchronize() advanced it on the host)
        self.lr0 = self.trainer.lr
        self.density = self._density()
        self.captures += 1

    def __call__(self) -> None:
        t = self.trainer
        if t.train_iter % t.num_batches_per_epoch == 0 and t.train_iter > 0:
            t._on_epoch_boundary()          # host-side epoch logic (density schedule, logging)
        d = t.data_iter()
        self.x.copy_(d[0], non_blocking=True)
        _copy(self.y, d[1])
        if self.graph is None or self._density() != self.density:
            self.recapture()
        # lr schedule on the host -> device multiplier read by the captured update
        t.adjust_learning_rate(t.train_epoch, t.optimizer)
        self.mult.fill_(float(t.lr) / float(self.lr0) if self.lr0 else 1.0)   # async, stream-ordered
        # fresh random-k / DGC sample seeds (this iteration's seed_for) and a new
        # dropout replay word: nothing random is frozen into the graph
        if hasattr(self.opt, "refresh_device_seeds"):
            self.opt.refresh_device_seeds()
        from .. import ops
        self.replays += 1
        ops.set_graph_seed(self.x.device, self.replays * 0x9E3779B1 + 1)
        self.graph.replay()
        for slot in getattr(self.opt, "_graph_sel", ()):   # selected counts of this replay (stream-ordered copies)
            self.opt._log_selected(slot)
        t.train_iter += 1
        if hasattr(self.opt, "train_iter"):
            self.opt.train_iter += 1


def graphed(trainer, opt, clip: Optional[float] = None) -> Callable[[], None]:
    """A zero-argument callable running one captured training iteration."""
    return GraphedStep(trainer, opt, clip)
