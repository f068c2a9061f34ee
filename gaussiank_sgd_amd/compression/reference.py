"""Pure-torch oracles with the REFERENCE's exact selection semantics.

These re-state, as plain functions, what each compressor of the reference
(``compression.py``) computes, including its quirks, so the fused HIP
pipeline can be parity-tested against them.  They sync with the host and
allocate freely: tests and parity studies only, never the hot path.

  gaussian       compression.py:358-389   EC, <=3 refinement loops
  gaussian2      compression.py:405-435   no EC, <=5 loops
  topk2          compression.py:315-334   torch.topk, no EC
  uniform topk   compression.py:96-104,180-198   argsort(|x|)[::101][-k:]
  bucketized     compression.py:60-93    per-value-bin quota on argsort(|x|, desc)
  randomk        compression.py:461-474
  redsync        compression.py:638-679
  redsynctrim    compression.py:707-737
  dgcsampling    compression.py:570-603 (random sample supplied by caller)
  bucket (sign)  compression.py:243-265,298-312

Each returns ``(acc, indexes(int64), values, new_residual)``.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from ..utils.stats import gen_threshold_from_normal_distribution

Result = Tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]


def _k(numel: int, ratio: float) -> int:
    return max(int(numel * ratio), 1)


def _finish(acc: torch.Tensor, indexes: torch.Tensor) -> Result:
    values = acc[indexes]
    residual = acc + 0.0
    residual[indexes] = 0.0
    return acc, indexes, values, residual


def gaussian(tensor: torch.Tensor, residual: Optional[torch.Tensor], ratio: float, loops: int = 3,
             ec: bool = True, stats: Optional[Tuple[float, float]] = None) -> Result:
    """``stats=(mean, std)`` lets a test inject the statistics of the kernel."""
    acc = tensor + residual if (ec and residual is not None) else tensor.clone()
    k = _k(acc.numel(), ratio)
    if stats is None:
        std = float(torch.std(acc))
        mean = float(torch.mean(acc))
    else:
        mean, std = stats
    _, right = gen_threshold_from_normal_distribution(1 - ratio, mean, std)
    abs_t = torch.abs(acc)
    it = 0
    indexes = None
    while it < loops:
        indexes = (abs_t > right).nonzero().view(-1)
        if indexes.numel() < 2 * k / 3:
            right *= 0.5
        elif indexes.numel() > 4 * k / 3:
            right *= 1.5
        else:
            break
        it += 1
    return _finish(acc, indexes)


def topk_exact(tensor: torch.Tensor, residual: Optional[torch.Tensor], ratio: float, ec: bool = True) -> Result:
    """Exact top-|x| (ties broken by lowest index), returned in ascending index order."""
    acc = tensor + residual if (ec and residual is not None) else tensor.clone()
    k = min(_k(acc.numel(), ratio), acc.numel())
    keys = acc.contiguous().view(torch.int32).to(torch.int64) & 0x7FFFFFFF
    K = int(torch.topk(keys, k).values[-1])
    gt = keys > K
    eq_idx = (keys == K).nonzero().view(-1)[: k - int(gt.sum())]
    mask = gt.clone()
    mask[eq_idx] = True
    return _finish(acc, mask.nonzero().view(-1))


def topk2(tensor: torch.Tensor, ratio: float) -> Result:
    """topk2: torch.topk on |x|, residual neither added nor fed back (compression.py:315-334)."""
    k = _k(tensor.numel(), ratio)
    _, indexes = torch.topk(torch.abs(tensor), k=k)
    return _finish(tensor.clone(), indexes)


def uniform_abs_topk(tensor: torch.Tensor, residual: Optional[torch.Tensor], ratio: float,
                     ec: bool = True) -> Result:
    """The shipped 'topk' selection: every 101st element of argsort(|x|) (NOT top-k)."""
    acc = tensor + residual if (ec and residual is not None) else tensor.clone()
    k = _k(acc.numel(), ratio)
    sorted_index = torch.abs(acc).argsort()
    indexes = sorted_index[::101][-k:]
    return _finish(acc, indexes)


def bucketized_topk(tensor: torch.Tensor, residual: Optional[torch.Tensor], ratio: float,
                    ec: bool = True) -> Result:
    """The reference's ``TopKCompressor.bucketized_topk`` (compression.py:60-93)
    behind the ``topk`` compressor's EC, re-stated without its per-bin Python
    loop but with its exact semantics, quirk included:

    * positions of ``argsort(|x|, descending)`` are consumed bin by bin, in the
      ASCENDING order of the bins ``unique(int(100 x))`` -- so the chunk of
      positions charged to a bin is NOT that bin's members (the
      ascending bins are paired with descending-sorted indices);
    * a bin of count c takes its first ``c`` positions when c == 1, else
      ``round(c k / n)`` (Python's round: half to even);
    * if fewer than k were taken, the untaken positions (in order) fill up;
      the result is cut to k.

    Ties in |x| are broken by the stable sort (the reference's unstable
    argsort leaves them unspecified)."""
    acc = tensor + residual if (ec and residual is not None) else tensor.clone()
    flat = acc.reshape(-1)
    n = flat.numel()
    k = _k(n, ratio)
    sorted_index = torch.argsort(torch.abs(flat), descending=True, stable=True)
    sorted_int = (flat[sorted_index] * 100).int()          # truncation toward zero, as .int()
    _, counts = torch.unique(sorted_int, sorted=True, return_counts=True)
    counts = counts.to(torch.int64)
    # round((count * k) / n): the double quotient, rounded half to even (torch.round)
    take = torch.round((counts * k).to(torch.float64) / n).to(torch.int64)
    take = torch.where(counts == 1, counts, take)
    starts = torch.cumsum(counts, 0) - counts
    pos_bin = torch.repeat_interleave(torch.arange(counts.numel(), device=flat.device), counts)
    offset = torch.arange(n, device=flat.device) - starts[pos_bin]
    sel = offset < take[pos_bin]
    indexes = sorted_index[sel]
    if indexes.numel() < k:
        indexes = torch.cat([indexes, sorted_index[~sel][: k - indexes.numel()]])
    return _finish(acc, indexes[:k])


def randomk(tensor: torch.Tensor, residual: Optional[torch.Tensor], ratio: float, ec: bool = False,
            generator: Optional[torch.Generator] = None) -> Result:
    acc = tensor + residual if (ec and residual is not None) else tensor.clone()
    k = _k(acc.numel(), ratio)
    perm = torch.randperm(acc.numel(), device=acc.device, generator=generator)
    return _finish(acc, perm[:k])


def redsync(tensor: torch.Tensor, residual: Optional[torch.Tensor], ratio: float, ec: bool = True) -> Result:
    acc = tensor + residual if (ec and residual is not None) else tensor.clone()
    k = _k(acc.numel(), ratio)
    lo, hi, eps = 0.0, 1.0, 0.2
    abs_t = torch.abs(acc)
    mean_val = torch.mean(abs_t)
    max_val = torch.max(abs_t)
    indexes = None
    while hi - lo > eps:
        tmp = lo + (hi - lo) / 2
        thres = mean_val + tmp * (max_val - mean_val)
        indexes = (abs_t > thres).nonzero().view(-1)
        nnz = indexes.numel()
        if nnz > k and 2 * k > nnz:
            break
        elif nnz < k / 2:
            hi = tmp
        else:
            lo = tmp
    return _finish(acc, indexes)


def redsynctrim(tensor: torch.Tensor, residual: Optional[torch.Tensor], ratio: float, ec: bool = True,
                max_iters: int = 16) -> Result:
    acc = tensor + residual if (ec and residual is not None) else tensor.clone()
    k = _k(acc.numel(), ratio)
    abs_t = torch.abs(acc)
    mean_val = torch.mean(abs_t)
    max_val = torch.max(abs_t)
    eps = 0.2
    tmp = 1 - eps
    thres = mean_val + tmp * (max_val - mean_val)
    indexes = (abs_t > thres).nonzero().view(-1)
    nnz = indexes.numel()
    it = 0
    while nnz < k and it < max_iters:
        thres = mean_val + tmp * (max_val - mean_val)
        indexes = (abs_t > thres).nonzero().view(-1)
        nnz = indexes.numel()
        tmp = tmp - eps
        it += 1
    return _finish(acc, indexes)


def dgcsampling(tensor: torch.Tensor, residual: Optional[torch.Tensor], ratio: float,
                sampled_indexes: torch.Tensor, ec: bool = True) -> Result:
    acc = tensor + residual if (ec and residual is not None) else tensor.clone()
    k = _k(acc.numel(), ratio)
    abs_v = torch.abs(acc)
    sv = abs_v[sampled_indexes]
    kk = min(k, sv.numel())
    thres = torch.topk(sv, k=kk).values[kk - 1]
    indexes = (abs_v > thres).nonzero().view(-1)
    if indexes.numel() > 4 * k / 3:
        _, ti = torch.topk(abs_v[indexes], k=k)
        indexes = indexes[ti]
    return _finish(acc, indexes)


def sign_bucket_mean(tensor: torch.Tensor):
    """Returns (residual, means[2], positive_mask): BucketCompressor.bucket_mean_2."""
    x = tensor.clone()
    pos = x >= 0
    means = torch.zeros(2, dtype=x.dtype)
    if bool(pos.any()):
        means[0] = x[pos].mean()
    if bool((~pos).any()):
        means[1] = x[~pos].mean()
    x[pos] -= means[0]
    x[~pos] -= means[1]
    return x, means, pos


def sparse_aggregate(numel: int, per_rank: list, P: int) -> torch.Tensor:
    """Intended aggregation g = (1/P) sum_r scatter(idx_r, val_r)."""
    out = torch.zeros(numel, dtype=torch.float64)
    for idx, val in per_rank:
        out.index_add_(0, idx.long(), val.double())
    return (out / P).float()
