"""Layer-wise backward profiler.

Parity: reference profiling.py:13-148 -- ``benchmark(trainer)`` runs
5 warm-up + 50 measured forward/backward passes, timestamps every
parameter's gradient in a hook and returns ``(seq_keys, layerwise_times,
sizes)`` in forward order for the MG-WFBP / MGS planners.  The reference
calls ``torch.cuda.synchronize()`` inside every hook; here each hook records
a HIP event on the current stream instead (no device-wide sync inside
backward), and the event deltas are read once after the pass.

Phase ranges (forward / backward / compress / exchange / update) are roctx
ranges emitted by ``utils/trace.py`` (rocprofv3 --marker-trace); the
optimizer's per-bucket timers are ``DistributedOptimizer(profiling=True)``.
"""
from __future__ import annotations

import contextlib
import time
from collections import defaultdict
from typing import Dict, List, Tuple

import numpy as np
import torch

from . import trace


class Profiling:
    def __init__(self, model: torch.nn.Module):
        if not isinstance(model, torch.nn.Module):
            raise ValueError("Not a valid model, please provide a 'nn.Module' instance.")
        self.model = model
        self._parameter_names = {v: k for k, v in model.named_parameters()}
        self._seq_keys = [k for k, _ in model.named_parameters()]
        self._backward_seq_keys: List[str] = []
        self._backward_key_sizes: List[int] = []
        self._events: Dict[str, list] = defaultdict(list)
        self._start = None
        self._is_profiling = False
        self._cuda = next(model.parameters()).is_cuda
        self._handles = [p.register_post_accumulate_grad_hook(self._make_hook(k)) for k, p in
                         model.named_parameters() if p.requires_grad]

    def _make_hook(self, name):
        def hook(p):
            if not self._is_profiling:
                return
            if len(self._backward_seq_keys) < len(self._seq_keys) and name not in self._backward_seq_keys:
                self._backward_seq_keys.append(name)
                self._backward_key_sizes.append(p.numel())
            self._events[name].append(self._stamp())
        return hook

    def _stamp(self):
        if self._cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            return e
        return time.time()

    def start(self):
        self._is_profiling = True
        self._start = self._stamp()

    def stop(self):
        self._is_profiling = False

    def remove(self):
        for h in self._handles:
            h.remove()

    def _delta(self, a, b) -> float:
        if self._cuda:
            return a.elapsed_time(b) / 1e3
        return b - a

    def get_layerwise_times(self) -> Tuple[np.ndarray, float]:
        if self._cuda:
            torch.cuda.synchronize()
        keys = self._backward_seq_keys
        ntrials = min(len(self._events[k]) for k in keys) if keys else 0
        starts = self._trial_starts
        table = []
        for j in range(ntrials):
            prev = starts[j]
            row = []
            for k in keys:
                t = self._events[k][j]
                row.append(max(self._delta(prev, t), 0.0))
                prev = t
            table.append(row)
        arr = np.array(table) if table else np.zeros((1, len(keys)))
        return arr.mean(axis=0), float(arr.sum(axis=1).mean())

    def get_backward_seq_keys(self):
        return self._backward_seq_keys

    def get_backward_key_sizes(self):
        return self._backward_key_sizes


def benchmark(trainer, warmup: int = 5, iterations: int = 50):
    """Per-layer backward times of ``trainer.net`` (forward order)."""
    p = Profiling(trainer.net)
    p._trial_starts = []
    hidden = None
    for i in range(iterations + warmup):
        inputs, labels = trainer.data_iter()
        outputs, loss, hidden = trainer.forward_loss(inputs, labels, None)
        if i >= warmup:
            p.start()
            p._trial_starts.append(p._start)
        loss.backward()
        p.stop()
        trainer.net.zero_grad(set_to_none=False)
    times, _ = p.get_layerwise_times()
    keys = p.get_backward_seq_keys()
    sizes = p.get_backward_key_sizes()
    p.remove()
    return keys[::-1], list(times[::-1]), sizes[::-1]
