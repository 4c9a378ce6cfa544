"""Optimal contiguous partitioning of a cost sequence.

``solve(costs, partitions)`` splits ``costs`` into ``partitions`` contiguous,
non-empty blocks minimising the largest block sum -- the pipeline's slowest
stage.  Exact: binary search over the achievable bottleneck values (all
contiguous sums) with a greedy feasibility check, O(n^2 log n) for n layers,
which is instantaneous for any realistic layer count.  Among optimal splits it
returns the one that packs earlier blocks fullest (deterministic).
"""
from __future__ import annotations

from typing import List, Sequence, TypeVar

__all__ = ["solve", "solve_balance"]

T = TypeVar("T", int, float)


def _feasible(costs: Sequence[float], parts: int, limit: float) -> bool:
    used, acc = 1, 0.0
    for c in costs:
        if c > limit:
            return False
        if acc + c > limit:
            used += 1
            acc = c
            if used > parts:
                return False
        else:
            acc += c
    return True


def _split(costs: Sequence[float], parts: int, limit: float) -> List[int]:
    """Greedy split under ``limit`` that still leaves >=1 item per remaining block."""
    n = len(costs)
    sizes: List[int] = []
    i = 0
    for b in range(parts):
        remaining_blocks = parts - b - 1
        acc = 0.0
        size = 0
        while i < n - remaining_blocks and (size == 0 or acc + costs[i] <= limit):
            acc += costs[i]
            size += 1
            i += 1
        sizes.append(size)
    sizes[-1] += n - i
    return sizes


def solve_balance(costs: Sequence[float], partitions: int) -> List[int]:
    """Block sizes (a ``balance`` list) for the optimal split."""
    n = len(costs)
    if partitions < 1:
        raise ValueError("partitions must be a positive integer")
    if n < partitions:
        raise ValueError(f"sequence is shorter than intended partitions ({n} < {partitions})")
    prefix = [0.0]
    for c in costs:
        prefix.append(prefix[-1] + float(c))
    candidates = sorted({prefix[j] - prefix[i] for i in range(n) for j in range(i + 1, n + 1)})
    lo, hi = 0, len(candidates) - 1
    while lo < hi:
        mid = (lo + hi) // 2
        if _feasible(costs, partitions, candidates[mid]):
            hi = mid
        else:
            lo = mid + 1
    return _split(costs, partitions, candidates[lo])


def solve(sequence: List[T], partitions: int = 1) -> List[List[T]]:
    """Splits ``sequence`` into ``partitions`` blocks with the smallest max sum."""
    sizes = solve_balance(sequence, partitions)
    out: List[List[T]] = []
    start = 0
    for s in sizes:
        out.append(list(sequence[start : start + s]))
        start += s
    return out
