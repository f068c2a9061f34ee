"""Trainer (DLTrainer), LR schedules and the CLI entry points."""
from .trainer import DLTrainer, _support_datasets, _support_dnns

__all__ = ["DLTrainer", "_support_datasets", "_support_dnns"]
