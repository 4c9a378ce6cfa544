"""Utilities: model partitioning helpers, timing and memory reporting."""
from .partition import partition_model

__all__ = ["partition_model"]
