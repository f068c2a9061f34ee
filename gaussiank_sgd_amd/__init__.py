"""gaussiank_sgd_amd -- MI355X-native communication-compressed data-parallel SGD.

Capabilities of GaussianK-SGD (Shi et al., "Understanding Top-k
Sparsification in Distributed Deep Learning"), rebuilt for AMD Instinct
MI355X: fused gfx950 HIP kernels for error-feedback sparsification
(Gaussian-k, exact top-k, random-k, DGC, RedSync, sign-bucket), a packed
sparse all-gather over RCCL/xGMI overlapped with backward, and fused
SGD/LARS updates over flat parameter arenas.

Sub-packages: ``ops`` (HIP kernels + bindings), ``compression``,
``parallel`` (comm, buckets, DistributedOptimizer), ``optim``, ``models``,
``data``, ``train``, ``utils``.
"""
__version__ = "0.1.0"

from . import settings  # noqa: F401
