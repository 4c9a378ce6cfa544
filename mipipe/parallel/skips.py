"""Cross-stage ``@skippable`` skips in the multi-process engine.

In the single-process :class:`mipipe.Pipe` a skip tensor rides a portal: it is
hidden from the intermediate partitions and copied once, stash device -> pop
device, at the pop partition's fence (``/root/reference/pipeline.py:136-138``,
``mipipe/skip/portal.py``).  The engine does the same across processes:

* the routes -- which virtual stage stashes each skip and which pops it -- are
  discovered once at construction, every rank contributing its chunks'
  declarations (:func:`gather_routes`);
* the stashing rank sends the tensor straight to the popping rank on a
  communicator of its own (:class:`~mipipe.parallel.p2p.DirectLinks`): every
  MI355X pair of a node has its own xGMI link, so a skip takes one hop on a
  link the activation traffic does not use, however many stages it spans;
* the popping rank hands the skip's gradient back the same way after its
  backward, and the stashing rank's backward seeds the stashed tensor with it
  (``torch.autograd.backward([y, *stashed], [dy, *dskips])``) -- the portal's
  Orange -> Copy -> Blue gradient hand-off, without phony edges, because each
  stage's backward is one explicit call here.

Skips between two chunks of the SAME rank (looping placement) are handed over
in memory; a stash and pop inside one chunk use the plain tracker.

Keys are ``"<namespace label or id>:<name>"`` strings so that they mean the
same on every rank: ranks build their modules with the same skip names, and
namespaced layers either in the same construction order on every rank or with
labelled namespaces (``Namespace(label=...)``).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist
from torch import Tensor, nn

from ..skip.skippable import Skippable
from ..skip.tracker import SkipTracker

__all__ = ["skip_key", "SkipRoute", "local_declarations", "routes_from_declarations", "gather_routes",
           "EngineSkipTracker"]


def skip_key(ns, name: str) -> str:
    if ns is None:
        return f":{name}"
    label = getattr(ns, "label", None)
    return f"{label if label is not None else ns.id}:{name}"


@dataclass
class SkipRoute:
    key: str
    stash_vstage: int
    pop_vstage: int
    shape: Optional[Tuple[int, ...]] = None  # per micro-batch, as sent
    dtype: Optional[torch.dtype] = None

    @property
    def has_grad(self) -> bool:
        return self.dtype is not None and self.dtype.is_floating_point


def _layers(module: nn.Module) -> Iterable[nn.Module]:
    if isinstance(module, nn.Sequential):
        for layer in module:
            yield from _layers(layer)
    else:
        yield module


def local_declarations(chunks: Sequence[nn.Module], vstages: Sequence[int]) -> List[Tuple[int, int, str, str]]:
    """``(vstage, layer position, 'stash' | 'pop', key)`` of every skippable layer of this rank's chunks."""
    out: List[Tuple[int, int, str, str]] = []
    for chunk, vs in zip(chunks, vstages):
        for pos, layer in enumerate(_layers(chunk)):
            if not isinstance(layer, Skippable):
                continue
            for ns, name in layer.poppable():
                out.append((vs, pos, "pop", skip_key(ns, name)))
            for ns, name in layer.stashable():
                out.append((vs, pos, "stash", skip_key(ns, name)))
    return out


def routes_from_declarations(decls: Iterable[Tuple[int, int, str, str]]) -> Dict[str, SkipRoute]:
    """Pairs every pop with the latest earlier stash of its key and returns the
    pairs that cross virtual stages (the cross-process form of
    :func:`~mipipe.skip.verify_skippables`; raises ``TypeError`` on a pop
    without a stash or a stash without a pop)."""
    # A layer reads its pops before it publishes its stashes (Skippable.forward).
    order = sorted(decls, key=lambda d: (d[0], d[1], d[2] != "pop"))
    open_stash: Dict[str, int] = {}
    routes: Dict[str, SkipRoute] = {}
    problems: List[str] = []
    for vs, _, kind, key in order:
        if kind == "stash":
            if key in open_stash:
                problems.append(f"'{key}' is stashed again (stage {vs}) before it was popped")
            open_stash[key] = vs
            continue
        if key not in open_stash:
            problems.append(f"'{key}' is popped at stage {vs} but was not stashed before")
            continue
        src = open_stash.pop(key)
        if src != vs:
            if key in routes:
                problems.append(f"'{key}' crosses stages twice; isolate the layers with namespaces")
            routes[key] = SkipRoute(key, src, vs)
    for key, vs in sorted(open_stash.items()):
        problems.append(f"'{key}' is stashed at stage {vs} but never popped")
    if problems:
        raise TypeError("skip connections do not match across pipeline stages:\n" +
                        "\n".join(f"* {p}" for p in problems))
    return routes


def gather_routes(chunks: Sequence[nn.Module], vstages: Sequence[int], act_shapes: Sequence[Tuple[int, ...]],
                  act_dtype: torch.dtype, group=None,
                  skip_shapes: Optional[Dict[str, Tuple[Sequence[int], torch.dtype]]] = None) -> Dict[str, SkipRoute]:
    """Cross-stage routes of the whole pipeline (collective over ``group`` when
    torch.distributed is initialised).  A skip travels with the shape and dtype
    of the activation its POP stage receives, unless ``skip_shapes`` names it
    (by skip name or by key)."""
    mine = (local_declarations(chunks, vstages), {vs: tuple(s) for vs, s in zip(vstages, act_shapes)})
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        every: List = [None] * dist.get_world_size(group)
        dist.all_gather_object(every, mine, group=group)
    else:
        every = [mine]
    decls = [d for part in every for d in part[0]]
    shapes = {vs: s for part in every for vs, s in part[1].items()}
    routes = routes_from_declarations(decls)
    spec_of = skip_shapes or {}
    for key, r in routes.items():
        spec = spec_of.get(key) or spec_of.get(key.split(":", 1)[1])
        if spec is not None:
            r.shape, r.dtype = tuple(spec[0]), spec[1]
        else:
            r.shape, r.dtype = shapes[r.pop_vstage], act_dtype
    return routes


class EngineSkipTracker(SkipTracker):
    """Tracker of one (chunk, micro-batch) run inside the engine.

    Cross-stage stashes are collected in :attr:`outgoing` (the engine ships
    them); cross-stage pops are served from :attr:`incoming` (what the engine
    received, as leaves that collect the skip's gradient)."""

    def __init__(self, cross: Dict[str, SkipRoute], incoming: Optional[Dict[str, Tensor]] = None) -> None:
        super().__init__()
        self.cross = cross
        self.incoming: Dict[str, Tensor] = dict(incoming or {})
        self.outgoing: Dict[str, Tensor] = {}

    def save(self, batch, ns, name: str, tensor: Optional[Tensor]) -> None:
        key = skip_key(ns, name)
        if key in self.cross:
            if tensor is None:
                raise TypeError(f"cross-stage skip '{key}' must stash a tensor, not None")
            self.outgoing[key] = tensor
        else:
            super().save(batch, ns, name, tensor)

    def load(self, batch, ns, name: str) -> Optional[Tensor]:
        key = skip_key(ns, name)
        if key in self.cross:
            try:
                return self.incoming[key]
            except KeyError:
                raise RuntimeError(f"skip '{key}' has not arrived at this stage") from None
        return super().load(batch, ns, name)
