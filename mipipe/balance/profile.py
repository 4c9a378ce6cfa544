"""Per-layer profiling for automatic balancing.

* :func:`profile_times` -- wall time of forward+backward per layer, measured on a
  sandboxed copy of each layer until ``timeout`` seconds have elapsed.  On a GPU
  each measurement is bracketed by device synchronisation, so it measures
  kernel time, not launch time.
* :func:`profile_sizes` -- activation memory per layer (peak allocated during
  the forward of a one-sample batch, scaled to one micro-batch of
  ``batch / chunks`` samples) plus parameter memory scaled by ``param_scale``
  (weights + grads + optimizer state).
"""
from __future__ import annotations

import copy
import time
from typing import Any, Generator, List, Sequence, Union

import torch
from torch import Tensor, nn

from ..microbatch import Batch

__all__ = ["profile_times", "profile_sizes", "layerwise_sandbox", "detach"]

Device = Union[torch.device, int, str]


def layerwise_sandbox(module: nn.Sequential, device: torch.device) -> Generator[nn.Module, None, None]:
    """Yields a deep copy of each layer on ``device`` (the model itself is untouched)."""
    for layer in module:
        sandbox = copy.deepcopy(layer).to(device)
        sandbox.train(module.training)
        yield sandbox


def detach(batch: Batch) -> None:
    """Makes each tensor of ``batch`` a fresh leaf that requires grad (floats only)."""
    for i, x in enumerate(batch):
        if torch.is_tensor(x):
            leaf = x.detach()
            if leaf.is_floating_point():
                leaf.requires_grad_(True)
            batch[i] = leaf


def _sync(device: torch.device) -> None:
    if device.type == "cuda":
        torch.cuda.synchronize(device)


def _as_batch(sample: Any) -> Batch:
    if isinstance(sample, (list, tuple)):
        return Batch(list(sample))
    return Batch(sample)


def profile_times(module: nn.Sequential, sample: Union[List[Any], Tensor], timeout: float, device: torch.device) -> List[int]:
    """Microseconds per layer (summed over repeated passes until ``timeout``)."""
    if any(p.grad is not None for p in module.parameters()):
        raise ValueError("some parameter already has gradient")
    device = torch.device(device)
    batch = _as_batch(sample)
    for i, x in enumerate(batch):
        if torch.is_tensor(x):
            batch[i] = x.to(device)

    layers = list(layerwise_sandbox(module, device))
    totals = [0.0] * len(layers)

    def one_pass(record: bool) -> None:
        b = _as_batch(list(batch) if not batch.atomic else batch.tensor)
        for k, layer in enumerate(layers):
            detach(b)
            _sync(device)
            t0 = time.perf_counter()
            out = b.call(layer)
            outs = [y for y in out if torch.is_tensor(y) and y.requires_grad]
            if outs:
                torch.autograd.backward(outs, [torch.ones_like(y) for y in outs])
            _sync(device)
            if record:
                totals[k] += time.perf_counter() - t0
            b = out

    # One untimed pass first: the first layer would otherwise absorb one-time
    # costs (autograd engine start-up, kernel loading, allocator growth).
    one_pass(record=False)
    begun = time.perf_counter()
    while time.perf_counter() - begun < timeout:
        one_pass(record=True)
    return [max(1, int(t * 1e6)) for t in totals]


def profile_sizes(
    module: nn.Sequential,
    input: Union[List[Any], Tensor],
    chunks: int,
    param_scale: float,
    device: torch.device,
) -> List[int]:
    """Bytes per layer: activations of one micro-batch + scaled parameter bytes."""
    device = torch.device(device)
    if device.type != "cuda":
        raise ValueError("size profiler supports only CUDA device")

    batch = _as_batch(input)
    sizes: List[int] = []
    latent_scale = batch[0].size(0) / chunks
    for i, x in enumerate(batch):
        if torch.is_tensor(x):
            batch[i] = x[:1].detach().to(device).requires_grad_(x.is_floating_point())

    for layer in layerwise_sandbox(module, device):
        detach(batch)
        torch.cuda.synchronize(device)
        torch.cuda.reset_peak_memory_stats(device)
        base = torch.cuda.memory_allocated(device)
        batch = batch.call(layer)
        peak = torch.cuda.max_memory_allocated(device)
        latent = max(0, peak - base)
        latent = int(latent * latent_scale)
        params = sum(p.numel() * p.element_size() for p in layer.parameters())
        sizes.append(latent + int(params * param_scale))
    return sizes
