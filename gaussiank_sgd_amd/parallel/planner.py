"""Bucket planners driven by layer-wise backward times.

* ``plan_mgwfbp`` -- merged-gradient WFBP for dense all-reduce
  (reference distributed_optimizer.py:162-228): walk layers from the output
  side, merge layer l into its predecessor whenever the merged all-reduce
  would not start later than the separate one.
* ``plan_mgs`` -- merged-gradient sparsification (reference :230-310): merge
  when the extra compression time of the merged tensor is smaller than the
  all-gather start-up time it saves.

Both take explicit cost models so they can run with the reference's GbE /
P102 constants (parity) or with models fitted on MI355X (RCCL over xGMI, HIP
compression pipeline) -- see ``utils.stats``.  Inputs follow the reference:
``seq_layernames`` / ``layerwise_times`` / sizes in forward order; the
returned groups are in backward order (last layer first), like
``group_with_threshold``.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Sequence, Tuple

from ..utils import stats as perf

AllreduceModel = Callable[[float], float]    # bytes -> seconds
CompressModel = Callable[[float], float]     # elements -> seconds
AllgatherModel = Callable[[float], float]    # elements -> seconds


def _comm_start(tc: List[float], tb: List[float], taob: List[float]) -> List[float]:
    L = len(tb)
    taoc = [0.0] * L
    taoc[L - 1] = taob[L - 1] + tb[L - 1]
    for l in range(L - 2, -1, -1):
        taoc[l] = max(taoc[l + 1] + tc[l + 1], taob[l] + tb[l])
    return taoc


def plan_mgwfbp(seq_layernames: Sequence[str], layerwise_times: Sequence[float], sizes: Sequence[int],
                allreduce_time: AllreduceModel, alpha: float) -> Tuple[List[List[str]], Dict[str, int]]:
    L = len(sizes)
    if L == 1:
        return [[seq_layernames[0]]], {seq_layernames[0]: 0}
    p = [float(s) for s in sizes]
    tb = [float(t) for t in layerwise_times]
    tc = [allreduce_time(s * 4) for s in p]
    taob = [0.0] * L
    for l in range(L - 2, -1, -1):
        taob[l] = taob[l + 1] + tb[l + 1]
    taoc = _comm_start(tc, tb, taob)

    def merge(l: int) -> None:
        tc[l] = 0.0
        p[l - 1] += p[l]
        p[l] = 0.0
        tc[l - 1] = allreduce_time(p[l - 1] * 4)

    groups: List[List[str]] = []
    group: List[str] = [seq_layernames[L - 1]]
    idx = 0
    key_map = {seq_layernames[L - 1]: 0}
    for l in range(L - 2, 0, -1):
        key = seq_layernames[l]
        group.append(key)
        key_map[key] = idx
        cur = taob[l - 1] + tb[l - 1]
        if cur < taoc[l + 1] + tc[l + 1]:
            merge(l)
            taoc = _comm_start(tc, tb, taob)
        elif taoc[l + 1] + tc[l + 1] < cur < taoc[l] + tc[l] and taoc[l] + alpha > cur:
            merge(l)
            taoc = _comm_start(tc, tb, taob)
        else:
            idx += 1
            groups.append(group)
            group = []
    key_map[seq_layernames[0]] = idx
    group.append(seq_layernames[0])
    groups.append(group)
    return groups, key_map


def plan_mgs(seq_layernames: Sequence[str], layerwise_times: Sequence[float], sizes: Sequence[int],
             compress_time: CompressModel, allgather_time: AllgatherModel) -> Tuple[List[List[str]], Dict[str, int]]:
    L = len(sizes)
    if L == 1:
        return [[seq_layernames[0]]], {seq_layernames[0]: 0}
    p = [float(s) for s in sizes]
    tb = [float(t) for t in layerwise_times]

    def sparse_and_backward_start(tb_: List[float], p_: List[float], start: float = 0.0):
        n = len(tb_)
        ts = [compress_time(s) for s in p_]
        taob = [start] * n
        taos = [start] * n
        taos[n - 1] = taob[n - 1] + tb_[n - 1]
        for l in range(n - 2, -1, -1):
            taob[l] = taos[l + 1] + ts[l + 1]
            taos[l] = taob[l] + tb_[l]
        return taob, taos, ts

    def comm_start(ts: List[float], taos: List[float], p_: List[float]):
        n = len(p_)
        tc = [allgather_time(s) for s in p_]
        taoc = [0.0] * n
        taoc[n - 1] = taos[n - 1] + ts[n - 1]
        for l in range(n - 2, -1, -1):
            taoc[l] = max(taoc[l + 1] + tc[l + 1], taos[l] + ts[l])
        return taoc, tc

    taob, taos, ts = sparse_and_backward_start(tb, p)
    taoc, tc = comm_start(ts, taos, p)
    groups: List[List[str]] = []
    group: List[str] = [seq_layernames[L - 1]]
    idx = 0
    key_map = {seq_layernames[L - 1]: 0}
    for l in range(L - 2, 0, -1):
        key = seq_layernames[l]
        group.append(key)
        key_map[key] = idx
        tw = (tb[l - 1] + compress_time(p[l] + p[l - 1]) - compress_time(p[l]) - compress_time(p[l - 1])
              - (taoc[l] - (taos[l] + ts[l])))
        tsave = allgather_time(p[l]) + allgather_time(p[l - 1]) - allgather_time(p[l] + p[l - 1])
        if tw < tsave:
            tb[l - 1] += tb[l]
            tb[l] = 0.0
            p[l - 1] += p[l]
            p[l] = 0.0
            ts[l - 1] = compress_time(p[l - 1])
            ts[l] = 0.0
            tb2, ta2, _ = sparse_and_backward_start(tb[:l], p[:l], start=taob[l] + tb[l])
            taob[:l] = tb2
            taos[:l] = ta2
            taoc, tc = comm_start(ts, taos, p)
        else:
            idx += 1
            groups.append(group)
            group = []
    key_map[seq_layernames[0]] = idx
    group.append(seq_layernames[0])
    groups.append(group)
    return groups, key_map


# ---------------------------------------------------------------------------
# model presets
# ---------------------------------------------------------------------------
REFERENCE_ALPHA_BETA = {
    16: (0.00010632079996292579, 1.5 * 3.2713239529771973e-10),
    8: (9.75367204301171e-05, 3.0568230536676206e-10),
    4: (4.204298980348825e-05, 2.0589360830118177e-10),
    2: (2.554691138304671e-06, 9.837548167872609e-11),
}


def models_for(P: int, density: float, preset: str = "mi355x"):
    """Return (allreduce_time(bytes), alpha, compress_time(n), allgather_time(n))."""
    if preset == "reference":
        keys = sorted(REFERENCE_ALPHA_BETA)
        k = next((x for x in keys if x >= P), keys[-1])
        alpha, beta = REFERENCE_ALPHA_BETA[k]
        return ((lambda b: perf.predict_allreduce_time_with_size(alpha, beta, b, P)), alpha,
                (lambda n: perf.topk_perf_model(n)), (lambda n: perf.allgather_perf_model(n, max(P, 2), density)))
    from ..utils import perf_model
    a = perf_model.collective_ab("allreduce", max(P, 2))[0]
    return ((lambda b: perf.allreduce_perf_model_xgmi(b, P)), a, (lambda n: perf.compress_perf_model_mi355x(n)),
            (lambda n: perf.allgather_perf_model_xgmi(n, P, density)))
