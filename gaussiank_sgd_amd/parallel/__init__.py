"""Data parallelism: comm facade (RCCL / gloo / native RCCL engine), flat
gradient arenas + buckets, bucket planners and the compressed
DistributedOptimizer."""
from . import comm
from .buckets import GradArena, group_with_threshold
from .distributed_optimizer import DistributedOptimizer
from .shadow import install_bf16_shadow, install_direct_grads

__all__ = ["comm", "GradArena", "group_with_threshold", "DistributedOptimizer", "install_bf16_shadow", "install_direct_grads"]
