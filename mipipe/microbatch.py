"""Micro-batch containers, scatter and gather.

Behaviour from the reference's ``Pipe.forward`` contract
(``/root/reference/pipe.py:436-475``) and its uses of ``Batch``
(``/root/reference/pipeline.py:44-60``, ``README.md:318-322,382``):

* a mini-batch is split on dim 0 with ``Tensor.chunk``; like ``chunk`` this can
  produce *fewer* than ``chunks`` micro-batches (batch 20, chunks 8 -> 7);
* non-tensor inputs and :class:`NoChunk`-wrapped tensors are replicated into
  every micro-batch;
* gather concatenates tensor outputs on dim 0 and returns non-tensor outputs as
  a list with one element per micro-batch (``[5, 5]``);
* every input tensor must live on the first partition's device.

On top of that, :func:`gather` can write straight into a preallocated output
(avoiding a second copy of the logits) -- see :func:`gather_into`.
"""
from __future__ import annotations

import typing
from typing import Any, Callable, Iterator, List, Sequence, Tuple, Union, cast

import torch
from torch import Tensor

__all__ = ["NoChunk", "Batch", "check", "scatter", "gather", "gather_into"]

Tensors = Sequence[Tensor]
TensorOrTensors = Union[Tensor, Tensors]


class NoChunk:
    """Marks a tensor input that is *not* split: every micro-batch sees all of it."""

    def __init__(self, inp: Tensor):
        if not torch.is_tensor(inp):
            raise TypeError(f"NoChunk only supported for tensors, found: {inp}")
        self._tensor = inp

    @property
    def tensor(self) -> Tensor:
        return self._tensor

    def __repr__(self) -> str:
        return f"NoChunk({tuple(self._tensor.shape)})"


class Batch:
    """One micro-batch: a single tensor ("atomic") or a tuple of values."""

    __slots__ = ("_values", "atomic")

    def __init__(self, values: Union[Any, List[Any], Tuple[Any, ...]]):
        if torch.is_tensor(values):
            self._values: Tuple[Any, ...] = (values,)
            self.atomic = True
        elif isinstance(values, (list, tuple)):
            self._values = tuple(values)
            self.atomic = False
            # Every partition boundary must carry at least one tensor
            # (/root/reference/pipe.py:436-438): dependencies attach to it.
            if not any(torch.is_tensor(v) for v in self._values):
                raise TypeError(f"No tensors found in batch: {self._values}")
        else:
            raise TypeError(f"No tensors found in batch: {values!r}")

    # -- views ---------------------------------------------------------------
    @property
    def tensor(self) -> Tensor:
        if not self.atomic:
            raise AttributeError("not atomic batch")
        return cast(Tensor, self._values[0])

    @property
    def values(self):
        """What a partition receives: the tensor itself when atomic, else the tuple."""
        if self.atomic:
            return self._values[0]
        return self._values

    @property
    def tensors(self) -> Tuple[Tensor, ...]:
        return tuple(v for v in self._values if torch.is_tensor(v))

    def find_tensor_idx(self) -> int:
        """Index of the first tensor -- where dependency edges are attached."""
        for idx, value in enumerate(self._values):
            if torch.is_tensor(value):
                return idx
        raise TypeError("No tensor found!")

    def get_device(self) -> torch.device:
        return self._values[self.find_tensor_idx()].device

    # -- computation ------------------------------------------------------------
    def call(self, function: Callable[..., Any]) -> "Batch":
        """Runs ``function`` on the values and wraps the result as a Batch."""
        if self.atomic:
            return Batch(function(self._values[0]))
        return Batch(function(*self._values))

    # -- sequence protocol ------------------------------------------------------
    def __repr__(self) -> str:
        return f"Batch[atomic={self.atomic!r}]({self._values!r})"

    def __iter__(self) -> Iterator[Any]:
        return iter(self._values)

    def __len__(self) -> int:
        return len(self._values)

    def __getitem__(self, index: int) -> Any:
        return self._values[index]

    @typing.overload
    def __setitem__(self, index: int, value: Any) -> None: ...

    @typing.overload
    def __setitem__(self, index: slice, value: Sequence[Any]) -> None: ...

    def __setitem__(self, index, value) -> None:
        if isinstance(index, int):
            if self.atomic and index != 0:
                raise IndexError("atomic batch allows index 0 only")
            items = list(self._values)
            items[index] = value
            self._values = tuple(items)
            return
        if isinstance(index, slice):
            if index != slice(None):
                raise NotImplementedError("only slice [:] supported")
            value = tuple(value)
            if self.atomic and len(value) != 1:
                raise IndexError("atomic batch cannot be replaced with multiple values")
            self._values = value
            return
        raise TypeError(f"invalid index type: {type(index).__name__}")


def check(first_device: torch.device, *inputs: Any) -> None:
    """Validates a mini-batch before scattering (``/root/reference/pipe.py:476-477``)."""
    first_device = torch.device(first_device)
    found_tensor = False
    for value in inputs:
        tensor = value.tensor if isinstance(value, NoChunk) else value
        if not torch.is_tensor(tensor):
            continue
        found_tensor = True
        if not _same_device(tensor.device, first_device):
            raise ValueError(
                "All inputs should be on the same device as the first partition "
                f"({first_device}); found input on {tensor.device}"
            )
    if not found_tensor:
        raise TypeError("inputs do not have any tensors")


def _same_device(a: torch.device, b: torch.device) -> bool:
    if a.type != b.type:
        return False
    if a.type != "cuda":
        return True
    ia = a.index if a.index is not None else torch.cuda.current_device()
    ib = b.index if b.index is not None else torch.cuda.current_device()
    return ia == ib


def scatter(*inputs: Any, chunks: int) -> List[Batch]:
    """Splits a mini-batch into micro-batches along dim 0."""
    if len(inputs) == 1 and torch.is_tensor(inputs[0]):
        return [Batch(piece) for piece in cast(Tensor, inputs[0]).chunk(chunks)]

    columns: List[List[Any]] = []
    n_chunks = None
    for value in inputs:
        if torch.is_tensor(value):
            pieces = list(cast(Tensor, value).chunk(chunks))
            if n_chunks is not None and len(pieces) != n_chunks:
                raise RuntimeError(
                    f"Found different number of chunks produced for inputs: {n_chunks} and {len(pieces)}"
                )
            n_chunks = len(pieces)
            columns.append(pieces)
        else:
            columns.append([])  # filled below once the micro-batch count is known

    if n_chunks is None:
        # Only NoChunk / non-tensor inputs: the batch is replicated `chunks` times.
        n_chunks = chunks

    for col, value in zip(columns, inputs):
        if col:
            continue
        shared = value.tensor if isinstance(value, NoChunk) else value
        col.extend([shared] * n_chunks)

    return [Batch([col[i] for col in columns]) for i in range(n_chunks)]


def gather(outputs: List[Batch]) -> Any:
    """Concatenates micro-batch outputs back into a mini-batch."""
    if outputs[0].atomic:
        return torch.cat([b.tensor for b in outputs])

    merged: List[Any] = []
    for pos in range(len(outputs[0])):
        kind = type(outputs[0][pos])
        column = []
        for b in outputs:
            if type(b[pos]) is not kind:
                raise TypeError(f"Types for microbatch outputs do not match, found: {kind} and {type(b[pos])}")
            column.append(b[pos])
        merged.append(torch.cat(column) if torch.is_tensor(outputs[0][pos]) else column)
    return tuple(merged)


def gather_into(outputs: List[Batch], out: Tensor) -> Tensor:
    """Like :func:`gather` for atomic outputs but writes into ``out`` (no autograd)."""
    offset = 0
    for b in outputs:
        t = b.tensor
        n = t.shape[0]
        out[offset : offset + n].copy_(t)
        offset += n
    return out
