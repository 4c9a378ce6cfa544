"""``@skippable`` modules and the ``stash`` / ``pop`` commands.

A skippable module's ``forward`` is a generator.  It ``yield stash(name, t)`` to
publish a tensor for a later layer and ``t = yield pop(name)`` to receive one.
The tensors bypass the intermediate layers -- and, inside a :class:`~mipipe.Pipe`,
the intermediate *partitions*: they are carried by portals (portal.py) straight
from the stashing partition's device to the popping partition's device.

Outside a pipe, a thread-local in-memory tracker is used, so the same
``nn.Sequential`` also runs unpartitioned (the transparency property).

Parity: ``verify_skippables`` is called by ``Pipe.__init__``
(``/root/reference/pipe.py:334-336``).
"""
from __future__ import annotations

from typing import (
    Any,
    Callable,
    ClassVar,
    Dict,
    FrozenSet,
    Generator,
    Iterable,
    List,
    Optional,
    Set,
    Tuple,
    Type,
    cast,
)

import torch
from torch import Tensor, nn

from ..microbatch import Batch
from .namespace import Namespace
from .tracker import current_skip_tracker

__all__ = ["skippable", "stash", "pop", "verify_skippables", "Skippable"]


class stash:
    """Command: ``yield stash('name', tensor)``."""

    __slots__ = ("name", "tensor")

    def __init__(self, name: str, tensor: Optional[Tensor]) -> None:
        self.name = name
        self.tensor = tensor


class pop:
    """Command: ``tensor = yield pop('name')``."""

    __slots__ = ("name",)

    def __init__(self, name: str) -> None:
        self.name = name


class Skippable(nn.Module):
    """Base of the classes produced by :func:`skippable`.

    Wraps an instance of the user's module class; ``self.module`` is it.
    """

    module_cls: ClassVar[Type[nn.Module]]
    stashable_names: ClassVar[FrozenSet[str]]
    poppable_names: ClassVar[FrozenSet[str]]

    def __init__(self, *args: Any, **kwargs: Any) -> None:
        super().__init__()
        self.module = self.module_cls(*args, **kwargs)  # type: ignore[call-arg]
        self.namespaces: Dict[str, Namespace] = {}

    def __repr__(self) -> str:
        return f"@skippable({self.module})"

    # -- naming ------------------------------------------------------------
    def namespaced(self, name: str) -> Tuple[Optional[Namespace], str]:
        return self.namespaces.get(name), name

    def stashable(self) -> Iterable[Tuple[Optional[Namespace], str]]:
        for name in sorted(self.stashable_names):
            yield self.namespaced(name)

    def poppable(self) -> Iterable[Tuple[Optional[Namespace], str]]:
        for name in sorted(self.poppable_names):
            yield self.namespaced(name)

    def isolate(self, ns: Namespace, *, only: Optional[Iterable[str]] = None) -> "Skippable":
        """Puts this layer's skip names (or just ``only``) into namespace ``ns``.

        Returns ``self`` so it chains: ``Layer().isolate(ns)``.
        """
        names: Iterable[str] = only if only is not None else (self.stashable_names | self.poppable_names)
        for name in names:
            self.namespaces[name] = ns
        return self

    # -- execution ---------------------------------------------------------
    def _drive(
        self,
        args: Tuple[Any, ...],
        on_stash: Callable[[str, Optional[Tensor]], None],
        on_pop: Callable[[str], Optional[Tensor]],
    ) -> Any:
        """Runs the user's forward, serving its stash/pop commands."""
        result = self.module(*args)
        if not isinstance(result, Generator):
            return result
        gen = cast(Generator, result)
        reply: Any = None
        while True:
            try:
                command = gen.send(reply)
            except StopIteration as stop:
                return stop.value
            if isinstance(command, stash):
                on_stash(command.name, command.tensor)
                reply = None
            elif isinstance(command, pop):
                reply = on_pop(command.name)
            else:
                raise TypeError(f"{command!r} is not a command from @skippable")

    def forward(self, *inputs: Any) -> Any:  # type: ignore[override]
        tracker = current_skip_tracker()

        # Pull every poppable tensor up front: portals attach their autograd
        # edges to the batch's first tensor.
        batch = Batch(inputs[0] if len(inputs) == 1 and torch.is_tensor(inputs[0]) else list(inputs))
        incoming: Dict[str, Optional[Tensor]] = {}
        for ns, name in self.poppable():
            try:
                incoming[name] = tracker.load(batch, ns, name)
            except KeyError:
                raise RuntimeError(f"'{name}' has not been stashed")
        args = (batch.values,) if batch.atomic else tuple(batch.values)

        outgoing: Dict[str, Optional[Tensor]] = {}

        def on_stash(name: str, tensor: Optional[Tensor]) -> None:
            if name not in self.stashable_names:
                raise RuntimeError(f"'{name}' has not been declared as stashable")
            outgoing[name] = tensor

        def on_pop(name: str) -> Optional[Tensor]:
            if name not in self.poppable_names:
                raise RuntimeError(f"'{name}' has not been declared as poppable")
            return incoming.pop(name)

        output = self._drive(args, on_stash, on_pop)

        missing = sorted(self.stashable_names - outgoing.keys())
        if missing:
            raise RuntimeError(", ".join(f"'{n}'" for n in missing) + " must be stashed but have not")
        leftover = sorted(incoming.keys())
        if leftover:
            raise RuntimeError(", ".join(f"'{n}'" for n in leftover) + " must be popped but have not")

        out_batch = Batch(output)
        for ns, name in self.stashable():
            tracker.save(out_batch, ns, name, outgoing[name])
        return out_batch.values


def skippable(
    stash: Iterable[str] = (), pop: Iterable[str] = ()
) -> Callable[[Type[nn.Module]], Type[Skippable]]:
    """Class decorator declaring which skip names a module stashes and pops.

    ::

        @skippable(stash=['1to3'])
        class Layer1(nn.Module):
            def forward(self, x):
                yield stash('1to3', x)
                return f(x)

        @skippable(pop=['1to3'])
        class Layer3(nn.Module):
            def forward(self, x):
                skip = yield pop('1to3')
                return f(x) + skip
    """
    stashable_names = frozenset(stash)
    poppable_names = frozenset(pop)

    def wrap(module_cls: Type[nn.Module]) -> Type[Skippable]:
        attrs = {
            "module_cls": module_cls,
            "stashable_names": stashable_names,
            "poppable_names": poppable_names,
            "__doc__": module_cls.__doc__,
            "__module__": module_cls.__module__,
            "__qualname__": module_cls.__qualname__,
        }
        return cast(Type[Skippable], type(module_cls.__name__, (Skippable,), attrs))

    return wrap


def verify_skippables(module: nn.Sequential) -> None:
    """Checks statically that every stash has exactly one later pop.

    Raises ``TypeError`` listing every mismatch.
    """
    stashed: Set[Tuple[Optional[Namespace], str]] = set()
    popped: Set[Tuple[Optional[Namespace], str]] = set()
    problems: List[str] = []

    for layer_name, layer in module.named_children():
        if not isinstance(layer, Skippable):
            continue

        for name in sorted(layer.stashable_names & layer.poppable_names):
            problems.append(f"'{layer_name}' declared '{name}' both as stashable and as poppable")

        for ns, name in layer.stashable():
            if name in layer.poppable_names:
                continue
            if (ns, name) in stashed:
                problems.append(f"'{layer_name}' redeclared '{name}' as stashable but not isolated by namespace")
                continue
            stashed.add((ns, name))

        for ns, name in layer.poppable():
            if name in layer.stashable_names:
                continue
            if (ns, name) in popped:
                problems.append(f"'{layer_name}' redeclared '{name}' as poppable but not isolated by namespace")
                continue
            if (ns, name) not in stashed:
                problems.append(f"'{layer_name}' declared '{name}' as poppable but it was not stashed")
                continue
            popped.add((ns, name))

    for _, name in sorted(stashed - popped, key=lambda k: k[1]):
        problems.append(f"no module declared '{name}' as poppable but stashed")

    if problems:
        raise TypeError(
            "one or more pairs of stash and pop do not match:\n\n" + "\n".join(f"* {p}" for p in problems)
        )
