"""Utilities: model partitioning, LM data pipeline, profiling/memory instrumentation."""
from .partition import partition_model
from . import data, profiling

__all__ = ["partition_model", "data", "profiling"]
