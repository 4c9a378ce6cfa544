"""Long cross-stage residuals for the LM: BASELINE.json config #5.

"TransformerEncoder with @skippable cross-stage residuals": layer ``a``'s
output is stashed and added to layer ``b``'s output (``b > a``), U-Net style --
the skips of U-ViT-like encoders.  With the layers spread over pipeline stages
these skips cross stage boundaries, which is exactly the reference's
skip_layout / copy_policy / portal path (``/root/reference/pipe.py:334-348``,
``pipeline.py:136-138``); in the multi-process engine they ride
:class:`~mipipe.parallel.p2p.DirectLinks` (stash rank -> pop rank, one xGMI
hop).

The skip modules are parameter-free and sit right after the pipeline unit
that ends a layer (its MLP output half), so they do not disturb the stage
planner's unit indices: :func:`insert_long_skips` places them into any list
of units (a whole model, or one stage's slice).
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

from torch import nn

from ..skip import Namespace, pop, skippable, stash

__all__ = ["StashSkip", "AddSkip", "unet_pairs", "layer_end_unit", "long_skip_modules", "insert_long_skips"]


@skippable(stash=["skip"])
class StashSkip(nn.Module):
    """Identity that stashes its input for a later :class:`AddSkip`."""

    def forward(self, x):
        yield stash("skip", x)
        return x


@skippable(pop=["skip"])
class AddSkip(nn.Module):
    """``x + skip``."""

    def forward(self, x):
        s = yield pop("skip")
        return x + s


def unet_pairs(num_layers: int) -> List[Tuple[int, int]]:
    """Mirror pairs ``(i, L-1-i)``: the outer layers' outputs reach the furthest."""
    return [(i, num_layers - 1 - i) for i in range(num_layers // 2)]


def layer_end_unit(layer: int) -> int:
    """Pipeline-unit index of layer ``layer``'s last unit (unit 0 is the
    encoder; 4 units per layer, see ``mipipe.parallel.stage.block_costs``)."""
    return 4 * layer + 4


def long_skip_modules(pairs: Sequence[Tuple[int, int]]) -> Dict[int, List[nn.Module]]:
    """unit index -> skip modules to run right after that unit (adds before
    stashes, so a layer that ends one skip and starts another passes the sum
    on).  Namespaces are LABELLED so every pipeline rank keys a skip alike."""
    after: Dict[int, List[Tuple[int, nn.Module]]] = {}
    for a, b in pairs:
        if not 0 <= a < b:
            raise ValueError(f"skip ({a}, {b}) must go forward")
        ns = Namespace(label=f"L{a}->L{b}")
        after.setdefault(layer_end_unit(a), []).append((1, StashSkip().isolate(ns)))
        after.setdefault(layer_end_unit(b), []).append((0, AddSkip().isolate(ns)))
    return {u: [m for _, m in sorted(ms, key=lambda t: t[0])] for u, ms in after.items()}


def insert_long_skips(units: Sequence[nn.Module], pairs: Sequence[Tuple[int, int]], start: int = 0) -> List[nn.Module]:
    """``units`` (pipeline units ``start, start+1, ...``) with the skip modules of
    ``pairs`` inserted after the units that end their layers."""
    after = long_skip_modules(pairs)
    out: List[nn.Module] = []
    for k, u in enumerate(units):
        out.append(u)
        out += after.get(start + k, [])
    return out
