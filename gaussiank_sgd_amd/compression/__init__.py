"""Compressor registry with the reference's names and call signature.

Parity: ``compression.py:741-754`` -- ``compressors[name]`` is a class whose
``compress(tensor, name=None, ratio=...) -> (tensor, indexes, values)``
mutates ``tensor`` into the error-compensated gradient, keeps per-name
residuals in a class-level dict and exposes ``decompress`` / ``clear``.

Every sparse compressor here is a thin spec over ONE fused HIP pipeline
(``ops.compress_``: stats -> candidate ladder -> one-pass count -> decide ->
select/compact); the spec says which threshold mode, whether the residual is
added (EC) and how big the fixed-size send record is (``k_cap``).  The
DistributedOptimizer reads the spec and drives the pipeline directly on flat
gradient buckets with no host sync; the ``compress()`` classmethod below is the
reference-compatible per-tensor API (it syncs once to size its outputs).

Deliberate deviations:
  * ``topk`` is EXACT top-k (radix select); the shipped reference picks every
    101st element of argsort(|x|) -- available as ``topk_legacy``.
  * ``bucketized_topk`` (torch only) is the reference's bucketized variant
    that produced its two ``*_bucketized_topk`` logs, quirk included.
  * ``none`` returns a 3-tuple (the reference's 2-tuple crashes its own caller).
  * variable-count selectors send at most ``k_cap`` entries per bucket; the
    rest stays in the residual (no gradient mass is dropped).  The record
    holds ``ceil(4k/3)`` entries for Gaussian-k and DGC,
    2k for RedSync (k < nnz < 2k).  When the reference rule's threshold
    passes more than k_cap entries (heavy-tailed buckets: the reference's
    <=3-loop tree stops at up to 18x k), the pipeline re-selects by
    magnitude -- the evaluated candidate threshold with the largest count
    in [2k/3, k_cap], else the exact radix key at k_cap -- so the record always holds
    the LARGEST entries; the header's ``total`` keeps the reference count.
  * ``gaussian_cal`` (new, opt-in): calibrated Gaussian-k -- the one-pass
    count evaluates 8 thresholds around a per-bucket adaptive centre and
    picks the count closest to k inside [2k/3, 4k/3], falling back to the
    exact radix key when none qualifies.  ``gaussian`` stays bit-faithful to
    the reference's <=3-loop tree (compression.py:372-381).
  * random-k seeds are a pure function of (iteration, bucket, rank) -- the
    reference's class-level counter (compression.py:439-553) would be shared
    by every virtual rank of an in-process world.
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import torch

from .. import ops
from ..utils.stats import gaussian_z
from . import reference


class _SparseCompressor:
    name = "sparse"
    mode = ops.MODE_GAUSSIAN
    ec = True
    loops = 3
    exact_k = False          # record capacity k (True) or ceil(kcap_factor * k)
    kcap_factor = 4.0 / 3.0
    dense = False
    fused = True             # drives the fused HIP pipeline
    same_seed = False        # random-k: identical indices on every rank
    sample_p = 0.01          # DGC sampling ratio
    residuals: Dict[str, torch.Tensor] = {}
    _bufs: Dict[str, "ops.CompressBuffers"] = {}
    counter = 0

    @classmethod
    def clear(cls) -> None:
        cls.residuals = {}
        cls._bufs = {}

    @classmethod
    def k_of(cls, numel: int, ratio: float) -> int:
        return max(int(numel * ratio), 1)

    @classmethod
    def k_cap_for(cls, k: int, numel: int) -> int:
        if cls.exact_k:
            return max(1, min(k, numel))
        return max(1, min(int(math.ceil(cls.kcap_factor * k)), numel))

    @classmethod
    def z_for(cls, ratio: float) -> float:
        return gaussian_z(ratio) if cls.mode == ops.MODE_GAUSSIAN else 0.0

    @classmethod
    def next_seed(cls, rank: int = 0) -> int:
        """Seed for the per-tensor class API (reference-style call counter)."""
        cls.counter += 1
        return cls.seed_for(cls.counter, 0, rank)

    @classmethod
    def seed_for(cls, step: int, bucket: int, rank: int = 0) -> int:
        """Stateless seed: identical on every rank for the *same* variants."""
        h = (int(step) * 1000003 + int(bucket) * 2654435761 + 17) & 0xFFFFFFFF
        if not cls.same_seed:
            h = (h + int(rank) * 7919 * 40503) & 0xFFFFFFFF
        h ^= h >> 16
        h = (h * 0x7FEB352D) & 0xFFFFFFFF
        h ^= h >> 15
        return h

    @classmethod
    def get_residuals(cls, name, like_tensor):
        if name not in cls.residuals:
            cls.residuals[name] = torch.zeros_like(like_tensor.data)
        return cls.residuals[name]

    @classmethod
    def compress(cls, tensor: torch.Tensor, name=None, sigma_scale=3, ratio=0.05, seed=None):
        with torch.no_grad():
            flat = tensor.data.view(-1)
            numel = flat.numel()
            k = cls.k_of(numel, ratio)
            k_cap = cls.k_cap_for(k, numel)
            res = cls.get_residuals(name, flat)
            if cls.ec:
                flat.add_(res)
            bufs = cls._bufs.get(name)
            if bufs is None or bufs.k_cap != k_cap or bufs.device != flat.device:
                bufs = ops.CompressBuffers(k_cap, flat.device)
                cls._bufs[name] = bufs
            seed = cls.next_seed() if seed is None else int(seed)
            ops.compress_(flat, res, bufs, cls.mode, ec=False, zero_g=False, loops=cls.loops,
                          z=cls.z_for(ratio), k=k, k_cap=k_cap, seed=seed, sample_p=cls.sample_p)
            sent = int(bufs.record[0])
            indexes = bufs.indices()[:sent].long()
            values = bufs.values()[:sent].clone()
            return tensor, indexes, values

    @staticmethod
    def decompress(tensor, ctc=None, name=None):
        return tensor


class GaussianCompressor(_SparseCompressor):
    """Gaussian-k (compression.py:337-403), EC, <=3 refinement loops.

    Record capacity k_cap = k: at most k entries go on the wire -- the
    reference's 500x at d = 0.001 (fp32 values + int32 indices,
    distributed_optimizer.py:426-427) -- and when the reference rule's
    threshold passes more (it accepts up to 4k/3) the largest k are sent (an
    overflow-extension threshold, else exact top-k) and the rest stays in the
    residual.  Measured on MI355X (r6c2, profiles/r06_kcap_ab.txt): the
    ResNet-50 bs512 step within noise of k_cap = 4k/3, bs32 -0.9%."""
    name = "gaussion"  # sic, reference :347
    mode = ops.MODE_GAUSSIAN
    ec = True
    loops = 3
    kcap_factor = 1.0


class GaussianCalCompressor(GaussianCompressor):
    """Calibrated Gaussian-k (new): 8-candidate adaptive ladder, exact fallback."""
    name = "gaussian_cal"
    mode = ops.MODE_GAUSSIAN_CAL
    kcap_factor = 4.0 / 3.0      # its decision accepts any count in [2k/3, 4k/3]

    @classmethod
    def z_for(cls, ratio: float) -> float:
        return gaussian_z(ratio)


class GaussianCompressor2(GaussianCompressor):
    """No residual add, <=5 loops (compression.py:405-435)."""
    name = "gaussion2"
    ec = False
    loops = 5


class TopKCompressor(_SparseCompressor):
    """Exact top-k with EC (radix select)."""
    name = "topk"
    mode = ops.MODE_TOPK
    ec = True
    exact_k = True


class TopKCompressor2(TopKCompressor):
    """torch.topk without residual feedback (compression.py:315-334)."""
    name = "topk2"
    ec = False


class TopKLegacyCompressor(_SparseCompressor):
    """The reference's shipped 'topk': uniform_abs_topk (argsort[::101][-k:]), torch only."""
    name = "topk_legacy"
    ec = True
    exact_k = True
    fused = False

    @classmethod
    def compress(cls, tensor, name=None, sigma_scale=2.5, ratio=0.05):
        with torch.no_grad():
            flat = tensor.data.view(-1)
            res = cls.get_residuals(name, flat)
            acc, idx, vals, new_res = reference.uniform_abs_topk(flat, res, ratio, ec=True)
            flat.copy_(acc)
            res.copy_(new_res)
            return tensor, idx, vals


class BucketizedTopKCompressor(TopKLegacyCompressor):
    """The reference's 'bucketized' topk (compression.py:60-93: per-value-bin
    quota of the |x|-sorted positions, with its bin/index pairing quirk), EC,
    torch only -- the selection behind the reference's
    logs/results/{SGD,LARS}_1024_*_bucketized_topk runs."""
    name = "bucketized_topk"

    @classmethod
    def compress(cls, tensor, name=None, sigma_scale=2.5, ratio=0.05):
        with torch.no_grad():
            flat = tensor.data.view(-1)
            res = cls.get_residuals(name, flat)
            acc, idx, vals, new_res = reference.bucketized_topk(flat, res, ratio, ec=True)
            flat.copy_(acc)
            res.copy_(new_res)
            return tensor, idx, vals


class RandomKCompressor(_SparseCompressor):
    """k uniformly random indices, no EC (compression.py:439-489)."""
    name = "randomk"
    mode = ops.MODE_RANDOMK
    ec = False
    exact_k = True


class RandomKECCompressor(RandomKCompressor):
    name = "randomkec"
    ec = True


class RandomKSameCompressor(RandomKCompressor):
    """Identical indices on every rank (compression.py:512-533), without reseeding the global RNG."""
    name = "randomksame"
    same_seed = True


class RandomKSameECCompressor(RandomKSameCompressor):
    name = "randomksameec"
    ec = True


class DGCSamplingCompressor(_SparseCompressor):
    """1% sample threshold, exact top-k when > 4k/3 (compression.py:555-620)."""
    name = "dgcsampling"
    mode = ops.MODE_DGC
    ec = True


class RedSyncCompressor(_SparseCompressor):
    name = "redsync"
    mode = ops.MODE_REDSYNC
    ec = True
    kcap_factor = 2.0          # stops once k < nnz < 2k (compression.py:653-672)


class RedSyncTrimCompressor(_SparseCompressor):
    name = "redsynctrim"
    mode = ops.MODE_REDSYNCTRIM
    ec = True
    kcap_factor = 4.0


class BucketCompressor:
    """Sign-bucket means (compression.py:227-312): all-reduce 2 floats per group.

    ``compress`` subtracts the per-sign mean in place and returns the means;
    ``decompress`` adds the (all-reduced) means back per original sign.
    """
    name = "bucket"
    dense = True
    fused = True
    _state: Dict[str, dict] = {}
    _last: Optional[str] = None

    @classmethod
    def clear(cls):
        cls._state = {}
        cls._last = None

    @classmethod
    def buffers(cls, name, flat: torch.Tensor) -> dict:
        st = cls._state.get(name)
        if st is None or st["mask"].numel() != flat.numel() or st["mask"].device != flat.device:
            st = {
                "mask": torch.zeros(flat.numel(), dtype=torch.uint8, device=flat.device),
                "means": torch.zeros(2, dtype=torch.float32, device=flat.device),
                "ws": ops.sign_bucket_ws(flat.device),
                "tensor": flat,
            }
            cls._state[name] = st
        st["tensor"] = flat
        return st

    @classmethod
    def compress(cls, tensor, name=None, ratio=None):
        with torch.no_grad():
            flat = tensor.data.view(-1)
            st = cls.buffers(name, flat)
            ops.sign_bucket_compress_(flat, st["mask"], st["means"], st["ws"])
            cls._last = name
            return tensor, None, st["means"]

    @classmethod
    def decompress(cls, tensor, ctc=None, name=None):
        name = cls._last if name is None else name
        st = cls._state[name]
        ops.sign_bucket_decompress_(st["tensor"], st["mask"], st["means"])
        return st["tensor"]


class NoneCompressor:
    name = "none"
    dense = True
    fused = True

    @staticmethod
    def clear():
        pass

    @staticmethod
    def compress(tensor, name=None, ratio=None):
        return tensor, None, tensor

    @staticmethod
    def decompress(tensor, ctc=None, name=None):
        return tensor


compressors = {
    "topk": TopKCompressor,
    "topk2": TopKCompressor2,
    "topk_legacy": TopKLegacyCompressor,
    "bucketized_topk": BucketizedTopKCompressor,
    "bucket": BucketCompressor,
    "gaussian": GaussianCompressor,
    "gaussian2": GaussianCompressor2,
    "gaussian_cal": GaussianCalCompressor,
    "randomk": RandomKCompressor,
    "randomkec": RandomKECCompressor,
    "randomksame": RandomKSameCompressor,
    "randomksameec": RandomKSameECCompressor,
    "dgcsampling": DGCSamplingCompressor,
    "redsync": RedSyncCompressor,
    "redsynctrim": RedSyncTrimCompressor,
    "none": NoneCompressor,
    None: NoneCompressor,
}

__all__ = ["compressors", "reference"] + [c.__name__ for c in set(compressors.values())]
