"""RRef facade for ``Pipe.forward``.

Upstream ``Pipe.forward`` returns ``torch.distributed.rpc.RRef(output)`` and
requires ``init_rpc`` (``/root/reference/README.md:59,373``); the reference
removed both because pipelining is intra-node (``/root/reference/pipe.py:318-323,
491-494``, ``README.md:545``).  Here the result is a real RPC ``RRef`` when an RPC
agent is running and a :class:`LocalRRef` otherwise -- both expose
``local_value()`` / ``to_here()`` -- so upstream user code runs without
``init_rpc``.
"""
from __future__ import annotations

from typing import Any, Generic, TypeVar

__all__ = ["LocalRRef", "make_rref", "rpc_agent_running"]

T = TypeVar("T")


class LocalRRef(Generic[T]):
    """An owner-local reference to a value, API-compatible with ``rpc.RRef``'s
    read side."""

    __slots__ = ("_value",)

    def __init__(self, value: T) -> None:
        self._value = value

    def local_value(self) -> T:
        return self._value

    def to_here(self, timeout: float = 0.0) -> T:
        return self._value

    def is_owner(self) -> bool:
        return True

    def confirmed_by_owner(self) -> bool:
        return True

    def owner_name(self) -> str:
        return "local"

    def __repr__(self) -> str:
        return f"LocalRRef({type(self._value).__name__})"


def rpc_agent_running() -> bool:
    try:
        from torch.distributed import rpc

        if not rpc.is_available():
            return False
        return bool(rpc.api._is_current_rpc_agent_set())  # type: ignore[attr-defined]
    except Exception:
        return False


def make_rref(value: Any):
    """``rpc.RRef(value)`` if an RPC agent exists, else :class:`LocalRRef`."""
    if rpc_agent_running():
        from torch.distributed.rpc import RRef

        return RRef(value)
    return LocalRRef(value)
