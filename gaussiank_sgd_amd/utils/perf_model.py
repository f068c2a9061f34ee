"""Measured MI355X cost models for the bucket planners (MG-WFBP / MGS).

Parity: the reference ships per-world-size all-reduce alpha-beta tables
measured on its cluster (distributed_optimizer.py:164-169) and a fitted top-k
model for its GPU (utils.py:62,86-93).  Here every constant carries its
provenance in a JSON file:

    {"compress":  {"c0_s": ..., "c1_s_per_elem": ..., "measured": true, "source": "..."},
     "allgather": {"<P>": {"alpha_s": ..., "beta_s_per_byte": ..., "measured": ..., "source": "..."}},
     "allreduce": {"<P>": {...}}}

``compress`` is fitted by ``bench/kernels.py --fit-out`` (the fused Gaussian-k
pipeline at several bucket sizes on one MI355X); ``allgather`` / ``allreduce``
by ``bench/collectives.py --fit-out`` or by ``bench.py`` itself at N > 1 (the
driver's scaling run measures this node's xGMI fabric and prints the fit in
its JSON line).  Entries without a measurement are flagged ``"measured":
false`` -- the planners use them, but nothing claims they were measured.

Lookup order: ``$GKSGD_PERF_MODEL`` if set, else ``tuning/perf_model_mi355x.json``.
"""
from __future__ import annotations

import json
import os
from typing import Dict, Optional, Sequence, Tuple

_REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
DEFAULT_PATH = os.path.join(_REPO, "tuning", "perf_model_mi355x.json")

# Unmeasured fallbacks (used only when no JSON is available):
# compress ~ 5 fp32 passes over n at ~5 TB/s + ~12 us of launches;
# xGMI: a few tens of us latency, ~100 GB/s (all-gather) / 130 GB/s bus (all-reduce).
_FALLBACK = {
    "compress": {"c0_s": 12e-6, "c1_s_per_elem": 4e-12, "measured": False,
                 "source": "unmeasured default (5 fp32 passes at ~5 TB/s)"},
    "allgather": {str(P): {"alpha_s": a, "beta_s_per_byte": 1 / 100e9, "measured": False,
                           "source": "unmeasured default"} for P, a in ((2, 15e-6), (4, 20e-6), (8, 25e-6))},
    "allreduce": {str(P): {"alpha_s": a, "beta_s_per_byte": 2 / 130e9, "measured": False,
                           "source": "unmeasured default"} for P, a in ((2, 20e-6), (4, 30e-6), (8, 40e-6))},
}

_cache: Dict[str, dict] = {}


def path() -> str:
    return os.environ.get("GKSGD_PERF_MODEL") or DEFAULT_PATH


def load(p: Optional[str] = None) -> dict:
    p = p or path()
    if p in _cache:
        return _cache[p]
    model = json.loads(json.dumps(_FALLBACK))
    if os.path.isfile(p):
        with open(p) as f:
            got = json.load(f)
        for key in ("compress",):
            if key in got:
                model[key] = got[key]
        for key in ("allgather", "allreduce"):
            model[key].update(got.get(key, {}))
    _cache[p] = model
    return model


def reset() -> None:
    _cache.clear()


def compress_coeffs() -> Tuple[float, float]:
    c = load()["compress"]
    return float(c["c0_s"]), float(c["c1_s_per_elem"])


def _nearest(table: Dict[str, dict], P: int) -> dict:
    if str(P) in table:
        return table[str(P)]
    keys = sorted(int(k) for k in table)
    for k in keys:
        if k >= P:
            return table[str(k)]
    return table[str(keys[-1])]


def collective_ab(op: str, P: int) -> Tuple[float, float]:
    if P <= 1:
        return 0.0, 0.0
    e = _nearest(load()[op], P)
    return float(e["alpha_s"]), float(e["beta_s_per_byte"])


def fit_alpha_beta(sizes: Sequence[float], times: Sequence[float]) -> Tuple[float, float]:
    """Least-squares t = alpha + beta * x with non-negative coefficients."""
    import numpy as np
    x = np.asarray(sizes, dtype=np.float64)
    y = np.asarray(times, dtype=np.float64)
    A = np.stack([np.ones_like(x), x], axis=1)
    (a, b), *_ = np.linalg.lstsq(A, y, rcond=None)
    if b < 0:
        a, b = float(y.mean()), 0.0
    if a < 0:
        b = float((x * y).sum() / max((x * x).sum(), 1e-30))
        a = 0.0
    return float(a), float(b)


def update(p: str, section: str, entry: dict, key: Optional[str] = None) -> None:
    """Merge one measured entry into the JSON file at ``p`` (created if missing)."""
    data = {}
    if os.path.isfile(p):
        with open(p) as f:
            data = json.load(f)
    if key is None:
        data[section] = entry
    else:
        data.setdefault(section, {})[key] = entry
    os.makedirs(os.path.dirname(os.path.abspath(p)), exist_ok=True)
    with open(p, "w") as f:
        json.dump(data, f, indent=1, sort_keys=True)
    reset()
