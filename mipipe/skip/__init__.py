"""Cross-partition skip connections: ``@skippable``, ``stash``, ``pop``."""
from .namespace import Namespace
from .skippable import pop, skippable, stash, verify_skippables
from .layout import SkipLayout, inspect_skip_layout
from .tracker import SkipTracker, SkipTrackerThroughPortals, current_skip_tracker, use_skip_tracker

__all__ = [
    "skippable",
    "stash",
    "pop",
    "verify_skippables",
    "Namespace",
    "SkipLayout",
    "inspect_skip_layout",
    "SkipTracker",
    "SkipTrackerThroughPortals",
    "use_skip_tracker",
    "current_skip_tracker",
]
