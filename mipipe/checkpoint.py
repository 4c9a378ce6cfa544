"""Activation checkpointing with deterministic recompute.

Graph shape (``/root/reference/pipeline.py:161-185``, ``README.md:452-537``)::

    Wait[1] -> Checkpoint -> Wait[3] -> fork --+-- Recompute(phony) --+-> join -> Copy
                                               +----------------------+

* ``Checkpoint.forward`` runs the partition under ``no_grad`` and stashes the RNG
  state; only the *inputs* are saved.
* ``Recompute`` hangs off a phony branch.  Its backward needs no gradient, so
  the autograd engine can run it as soon as the join's gradient arrives -- i.e.
  *before* ``Wait[3].backward`` makes the compute stream wait for the incoming
  gradient copy.  Recomputation therefore overlaps the gradient transfer.
* ``Checkpoint.backward`` pops the recomputed ``(output, leaf inputs)`` and runs
  the real backward through them.

RNG: dropout in ``mipipe.ops`` draws its Philox (seed, offset) from the torch
device generator, so saving/restoring ``torch.cuda.get_rng_state`` here makes
the recomputed masks bit-identical to the forward ones (§2.2 N6).
"""
from __future__ import annotations

import threading
from collections import deque
from contextlib import contextmanager
from typing import Any, Callable, Deque, Generator, List, Optional, Tuple, Union

import torch
from torch import Tensor

from .dependency import fork, join
from .microbatch import Batch
from .phony import get_phony

__all__ = [
    "is_checkpointing",
    "is_recomputing",
    "enable_checkpointing",
    "enable_recomputing",
    "Checkpointing",
    "Checkpoint",
    "Recompute",
    "checkpoint",
    "save_rng_states",
    "restore_rng_states",
]

Recomputed = Tuple[Any, Tuple[Any, ...]]
RNGStates = Tuple[Tensor, Optional[Tensor]]


class _ThreadFlags(threading.local):
    def __init__(self) -> None:
        self.checkpointing = False
        self.recomputing = False
        # a checkpointed forward whose recompute will run (grad was enabled around it)
        self.recompute_expected = True


_flags = _ThreadFlags()


@contextmanager
def enable_checkpointing() -> Generator[None, None, None]:
    prev = _flags.checkpointing
    _flags.checkpointing = True
    try:
        yield
    finally:
        _flags.checkpointing = prev


@contextmanager
def enable_recomputing() -> Generator[None, None, None]:
    prev = _flags.recomputing
    _flags.recomputing = True
    try:
        yield
    finally:
        _flags.recomputing = prev


def is_checkpointing() -> bool:
    """True while a partition runs its first (no-grad) forward under checkpointing."""
    return _flags.checkpointing


def recompute_expected() -> bool:
    """True while a checkpointed forward runs whose backward will recompute it:
    state kept for the recompute (ops.attention's dropout keep words) is then
    worth keeping.  False for a training-mode forward under ``torch.no_grad()``
    (checkpointed, but never backpropagated)."""
    return _flags.checkpointing and _flags.recompute_expected


@contextmanager
def _recompute_expected(on: bool) -> Generator[None, None, None]:
    prev = _flags.recompute_expected
    _flags.recompute_expected = on
    try:
        yield
    finally:
        _flags.recompute_expected = prev


def is_recomputing() -> bool:
    """True while a partition re-runs its forward during backward.

    Layers with side effects on forward (DeferredBatchNorm's statistics) must
    skip them when this is set.
    """
    return _flags.recomputing


def save_rng_states(device: torch.device, rng_states: Deque[RNGStates]) -> None:
    cpu_state = torch.get_rng_state()
    dev_state = torch.cuda.get_rng_state(device) if device.type == "cuda" else None
    rng_states.append((cpu_state, dev_state))


@contextmanager
def restore_rng_states(device: torch.device, rng_states: Deque[RNGStates]) -> Generator[None, None, None]:
    """Restores the saved RNG state for the block; the ambient state is
    preserved so recompute does not perturb later random draws."""
    cpu_state, dev_state = rng_states.pop()
    devices = [device] if device.type == "cuda" else []
    with torch.random.fork_rng(devices=devices, enabled=True):
        torch.set_rng_state(cpu_state)
        if dev_state is not None:
            torch.cuda.set_rng_state(dev_state, device)
        yield


def _first_device(values) -> torch.device:
    for v in values:
        if torch.is_tensor(v):
            return v.device
    raise RuntimeError(f"No tensors found in {values}")


def _float_only(output):
    if isinstance(output, tuple):
        return tuple(x.detach() if torch.is_tensor(x) and not x.is_floating_point() else x for x in output)
    return output


class Checkpointing:
    """Pairs one ``Checkpoint`` with the ``Recompute`` that will feed it."""

    def __init__(self, function: Callable[..., Any], batch: Batch) -> None:
        self.function = function
        self.batch = batch
        # Exactly one recompute result and one RNG snapshot travel between the
        # two autograd nodes.
        self.recomputed: Deque[Recomputed] = deque(maxlen=1)
        self.rng_states: Deque[RNGStates] = deque(maxlen=1)

    def checkpoint(self) -> Batch:
        """Runs the function without keeping activations."""
        # A phony that requires grad keeps Checkpoint in the graph even when no
        # input requires grad (e.g. token ids into the first partition).
        phony = get_phony(self.batch.get_device(), requires_grad=True)
        with _recompute_expected(torch.is_grad_enabled()):
            output = Checkpoint.apply(
                phony, self.recomputed, self.rng_states, self.function, self.batch.atomic, *self.batch
            )
        return Batch(_float_only(output))

    def recompute(self, batch: Batch) -> None:
        """Schedules recomputation as a side branch of ``batch``'s graph."""
        idx = batch.find_tensor_idx()
        batch[idx], phony = fork(batch[idx])
        phony = Recompute.apply(
            phony, self.recomputed, self.rng_states, self.function, self.batch.atomic, *self.batch
        )
        batch[idx] = join(batch[idx], phony)


class Checkpoint(torch.autograd.Function):
    @staticmethod
    def forward(ctx, phony, recomputed, rng_states, function, input_atomic, *inputs):  # type: ignore[override]
        ctx.recomputed = recomputed
        save_rng_states(_first_device(inputs), rng_states)
        ctx.save_for_backward(*[x for x in inputs if torch.is_tensor(x)])
        with torch.no_grad(), enable_checkpointing():
            if input_atomic:
                return function(inputs[0])
            return function(*inputs)

    @staticmethod
    def backward(ctx, *grad_outputs):  # type: ignore[override]
        output, leaves = ctx.recomputed.pop()
        outputs = output if isinstance(output, tuple) else (output,)
        pairs = [
            (y, g)
            for y, g in zip(outputs, grad_outputs)
            if torch.is_tensor(y) and y.requires_grad and g is not None
        ]
        if pairs:
            torch.autograd.backward([y for y, _ in pairs], [g for _, g in pairs])
        grads: List[Optional[Tensor]] = [None] * 5
        grads.extend(x.grad if torch.is_tensor(x) else None for x in leaves)
        return tuple(grads)


class Recompute(torch.autograd.Function):
    @staticmethod
    def forward(ctx, phony, recomputed, rng_states, function, input_atomic, *inputs):  # type: ignore[override]
        ctx.recomputed = recomputed
        ctx.rng_states = rng_states
        ctx.function = function
        ctx.input_atomic = input_atomic
        ctx.inputs = inputs
        ctx.save_for_backward(*[x for x in inputs if torch.is_tensor(x)])
        return phony

    @staticmethod
    def backward(ctx, *grad_outputs):  # type: ignore[override]
        inputs = ctx.inputs
        leaves = tuple(
            x.detach().requires_grad_(x.requires_grad) if torch.is_tensor(x) else x for x in inputs
        )
        device = _first_device(inputs)
        with restore_rng_states(device, ctx.rng_states):
            with torch.enable_grad(), enable_recomputing():
                if ctx.input_atomic:
                    output = ctx.function(leaves[0])
                else:
                    output = ctx.function(*leaves)
        ctx.recomputed.append((output, leaves))
        return tuple([None] * (5 + len(inputs)))


def checkpoint(function: Callable[..., Any], input: Union[Tensor, Tuple[Any, ...]]):
    """Checkpoints ``function(input)`` outside a pipeline (upstream helper)."""
    batch = Batch(input)
    chk = Checkpointing(function, batch)
    batch = chk.checkpoint()
    chk.recompute(batch)
    return batch.values
