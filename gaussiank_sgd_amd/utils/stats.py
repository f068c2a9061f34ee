"""Statistics helpers and the alpha-beta performance models.

Parity map (reference ``utils.py``):
  * ``gen_threshold_from_normal_distribution`` -> ``utils.py:136-138``
  * ``topk_perf_model`` / ``allgather_perf_model`` -> ``utils.py:86-107``
  * ``predict_allreduce_time_with_size`` -> ``utils.py:131-134``
  * ``predict_density_with_size_and_computation`` -> ``utils.py:110-129``
  * ``get_approximate_sigma_scale`` -> ``utils.py:42-52``
  * ``create_path`` / ``force_insert_item`` -> ``utils.py:13-21,55-58``

The reference calls ``scipy.stats.norm.ppf`` on the host inside every
compress call.  Here the quantile is a pure-python function (Acklam's rational
approximation polished by two Newton steps on ``math.erfc``; |err| < 1e-15)
that is evaluated once per density and cached, so the GPU path never waits on
the host.  The alpha/beta tables are kept for parity; ``fit_alpha_beta``
re-fits them from measurements taken on this machine (RCCL over xGMI).
"""
from __future__ import annotations

import functools
import math
import os
from typing import Dict, Iterable, Sequence, Tuple

import numpy as np

# --------------------------------------------------------------------------
# normal quantile
# --------------------------------------------------------------------------
_A = (-3.969683028665376e01, 2.209460984245205e02, -2.759285104469687e02,
      1.383577518672690e02, -3.066479806614716e01, 2.506628277459239e00)
_B = (-5.447609879822406e01, 1.615858368580409e02, -1.556989798598866e02,
      6.680131188771972e01, -1.328068155288572e01)
_C = (-7.784894002430293e-03, -3.223964580411365e-01, -2.400758277161838e00,
      -2.549732539343734e00, 4.374664141464968e00, 2.938163982698783e00)
_D = (7.784695709041462e-03, 3.224671290700398e-01, 2.445134137142996e00,
      3.754408661907416e00)


def _acklam(p: float) -> float:
    plow = 0.02425
    if p < plow:
        q = math.sqrt(-2 * math.log(p))
        return (((((_C[0] * q + _C[1]) * q + _C[2]) * q + _C[3]) * q + _C[4]) * q + _C[5]) / \
               ((((_D[0] * q + _D[1]) * q + _D[2]) * q + _D[3]) * q + 1)
    if p > 1 - plow:
        q = math.sqrt(-2 * math.log(1 - p))
        return -(((((_C[0] * q + _C[1]) * q + _C[2]) * q + _C[3]) * q + _C[4]) * q + _C[5]) / \
                ((((_D[0] * q + _D[1]) * q + _D[2]) * q + _D[3]) * q + 1)
    q = p - 0.5
    r = q * q
    return (((((_A[0] * r + _A[1]) * r + _A[2]) * r + _A[3]) * r + _A[4]) * r + _A[5]) * q / \
           (((((_B[0] * r + _B[1]) * r + _B[2]) * r + _B[3]) * r + _B[4]) * r + 1)


@functools.lru_cache(maxsize=4096)
def norm_ppf(p: float) -> float:
    """Inverse standard-normal CDF, double precision."""
    if not (0.0 < p < 1.0):
        if p == 0.0:
            return -math.inf
        if p == 1.0:
            return math.inf
        raise ValueError("p must be in [0, 1], got %r" % p)
    x = _acklam(p)
    # Newton polish on Phi(x) - p, Phi(x) = erfc(-x/sqrt2)/2
    for _ in range(2):
        e = 0.5 * math.erfc(-x / math.sqrt(2.0)) - p
        u = e * math.sqrt(2 * math.pi) * math.exp(x * x / 2.0)
        x = x - u / (1 + x * u / 2)
    return x


def gaussian_z(ratio: float) -> float:
    """|z| such that P(|N(0,1)| > z) = ratio (the reference's right multiplier).

    ``gen_threshold_from_normal_distribution(1-ratio, mu, sigma)`` returns
    ``mu - ppf(ratio/2)*sigma`` as the right threshold (utils.py:136-138).
    """
    return -norm_ppf(ratio / 2.0)


def gen_threshold_from_normal_distribution(p_value: float, mu: float, sigma: float) -> Tuple[float, float]:
    zvalue = norm_ppf((1 - p_value) / 2)
    return mu + zvalue * sigma, mu - zvalue * sigma


def get_approximate_sigma_scale(density: float) -> float:
    if density > 0.7:
        return 0.5
    if density > 0.05:
        return 1.5
    if density > 0.01:
        return 2.0
    return 3.0


# --------------------------------------------------------------------------
# performance models (reference constants kept for the planners' parity mode)
# --------------------------------------------------------------------------
TOPK_S_P102 = 2.18896957e-10  # P102-100 (reference utils.py:62)

GbE_multi_p_ab_small = {2: (1.6e-3, 1.0e-8), 4: (2.7e-3, 1.3e-8), 8: (4.0e-3, 1.5e-8), 16: (1.7e-3, 1.7e-8)}
GbE_multi_p_ab_large = {2: (4.4e-3, 5.8e-9), 4: (5.6e-3, 7.4e-9), 8: (7.68e-3, 8.2e-9), 16: (2.1e-3, 1.7e-8)}
tenGbE_multi_p_ab = {2: (1.5e-5, 5.7e-11), 4: (3.6e-5, 1.1e-10), 8: (8.5e-5, 1.4e-10), 16: (1.4e-4, 2.0e-10)}

# MI355X models: constants with provenance live in tuning/perf_model_mi355x.json
# (utils/perf_model.py; measured entries are flagged, unmeasured ones are
# labelled as defaults there).  Kept as functions so a re-fit file is picked up.
def _nearest(table: Dict[int, Tuple[float, float]], P: int) -> Tuple[float, float]:
    if P in table:
        return table[P]
    keys = sorted(table)
    for k in keys:
        if k >= P:
            return table[k]
    return table[keys[-1]]


def topk_perf_model(x: float, s: float = TOPK_S_P102) -> float:
    """Reference model of sort-based top-k: s * x * log2(x) (utils.py:86-93)."""
    if x == 0.0:
        return 0.0
    return s * x * np.log2(x)


def allgather_perf_model(x: float, P: int, density: float = 0.001, eth: str = "GbE") -> float:
    """Reference GbE all-gather model (utils.py:95-107)."""
    if x == 0:
        return 0.0
    size = x * P * 4 * density
    multi_p_ab = GbE_multi_p_ab_large if size >= 1024 * 1024 else GbE_multi_p_ab_small
    a, b = _nearest(multi_p_ab, P)
    return (a + b * size) * 2


def compress_perf_model_mi355x(x: float) -> float:
    """Fused compression pipeline time for a bucket of x gradients."""
    if x == 0:
        return 0.0
    from . import perf_model
    c0, c1 = perf_model.compress_coeffs()
    return c0 + c1 * x


def allgather_perf_model_xgmi(x: float, P: int, density: float = 0.001, kcap_factor: float = 4.0 / 3.0) -> float:
    """All-gather of one bucket's packed record: (4 + 2 k_cap) int32 words per rank."""
    if x == 0 or P <= 1:
        return 0.0
    from . import perf_model
    a, b = perf_model.collective_ab("allgather", P)
    rec_bytes = (4 + 2 * kcap_factor * max(x * density, 1.0)) * 4
    return a + b * rec_bytes


def allreduce_perf_model_xgmi(nbytes: float, P: int) -> float:
    if nbytes == 0 or P <= 1:
        return 0.0
    from . import perf_model
    a, b = perf_model.collective_ab("allreduce", P)
    return a + b * nbytes


def predict_density_with_size_and_computation(m, comp_time, P):
    """Reference returns 0.001 unconditionally (utils.py:110-129)."""
    return 0.001


def predict_allreduce_time_with_size(alpha: float, beta: float, size: float, P: int) -> float:
    if size == 0:
        return 0.0
    return alpha + beta * size


def fit_alpha_beta(sizes_bytes: Sequence[float], times_s: Sequence[float]) -> Tuple[float, float]:
    """Least-squares fit t = alpha + beta * bytes (non-negative)."""
    x = np.asarray(sizes_bytes, dtype=np.float64)
    y = np.asarray(times_s, dtype=np.float64)
    A = np.stack([np.ones_like(x), x], axis=1)
    (alpha, beta), *_ = np.linalg.lstsq(A, y, rcond=None)
    return float(max(alpha, 0.0)), float(max(beta, 0.0))


# --------------------------------------------------------------------------
# misc helpers
# --------------------------------------------------------------------------
def create_path(relative_path: str) -> None:
    os.makedirs(relative_path, exist_ok=True)


def force_insert_item(d: dict, key, val) -> None:
    d.setdefault(key, []).append(val)


def topk(tensor: np.ndarray, k: int):
    indexes = np.abs(tensor).argsort()[-k:]
    return indexes, tensor[indexes]


def effective_compression_ratio(numel: int, selected: float, value_bytes: int = 4, index_bytes: int = 4,
                                dense_bytes: int = 4) -> float:
    """Dense payload / sparse payload per rank (500x at density 0.001, fp32+int32)."""
    if selected <= 0:
        return float("inf")
    return (numel * dense_bytes) / (selected * (value_bytes + index_bytes))
