"""Statistics / perf models, checkpointing, profiling and metrics helpers."""
from . import stats
from .stats import create_path, force_insert_item, gen_threshold_from_normal_distribution

__all__ = ["stats", "create_path", "force_insert_item", "gen_threshold_from_normal_distribution"]
