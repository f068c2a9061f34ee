"""Hang watchdog and JSONL metrics (failure detection / observability).

The reference has no failure detection; a stuck collective simply hangs
every rank.  Here collectives already carry a timeout (torch.distributed
``timeout``, GKSGD_COLLECTIVE_TIMEOUT_S), and ``Watchdog`` adds a cheap
host-side detector: the training loop ``kick()``s it once per step; if no kick
arrives within ``timeout_s`` it logs the caller-provided state description
(bucket readiness / launch flags, selection counters) and every thread's
Python stack, once per stall, without touching the GPU.
"""
from __future__ import annotations

import faulthandler
import json
import os
import sys
import threading
import time
from typing import Callable, Optional

from ..settings import logger


class Watchdog:
    def __init__(self, timeout_s: float, describe: Optional[Callable[[], str]] = None, name: str = "gksgd"):
        self.timeout_s = float(timeout_s)
        self.describe = describe
        self.name = name
        self._last = time.monotonic()
        self._fired = False
        self._stop = threading.Event()
        self.stalls = 0
        self._thread = threading.Thread(target=self._run, name="%s-watchdog" % name, daemon=True)
        self._thread.start()

    def kick(self) -> None:
        self._last = time.monotonic()
        self._fired = False

    def _run(self) -> None:
        while not self._stop.wait(min(self.timeout_s / 4, 5.0)):
            idle = time.monotonic() - self._last
            if idle > self.timeout_s and not self._fired:
                self._fired = True
                self.stalls += 1
                msg = "[watchdog] no training step for %.1f s (limit %.1f s)" % (idle, self.timeout_s)
                try:
                    if self.describe is not None:
                        msg += "\n" + self.describe()
                except Exception as e:  # never let the watchdog itself crash
                    msg += "\n(state unavailable: %s)" % e
                logger.error(msg)
                try:
                    faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
                except Exception:
                    pass

    def stop(self) -> None:
        self._stop.set()
        self._thread.join(timeout=1.0)


class JsonlMetrics:
    """Append-only JSON-lines metrics file (one object per call)."""

    def __init__(self, path: str):
        self.path = path
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)

    def write(self, **fields) -> None:
        fields.setdefault("time", time.time())
        with open(self.path, "a") as f:
            f.write(json.dumps(fields, default=float) + "\n")
