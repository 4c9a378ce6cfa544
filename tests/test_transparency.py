"""Pipe is transparent: outputs and gradients equal the plain nn.Sequential
(SURVEY §4 'Transparency tests'), including the reference driver's
Transformer (BASELINE config #1: 2-stage, 2-layer nn.TransformerEncoder, chunks=2,
checkpoint='never', CPU devices)."""
import copy
import math

import pytest
import torch
from torch import nn

from mipipe import Pipe
from mipipe.balance import balance_by_time
from mipipe.balance.blockpartition import solve, solve_balance
from mipipe.utils import partition_model


@pytest.mark.parametrize("checkpoint", ["never", "except_last", "always"])
def test_simple_linears(checkpoint):
    def sum_grad(parameters):
        return sum(p.grad.sum() for p in parameters if p.grad is not None)

    def zero_grad(parameters):
        for p in parameters:
            p.grad = None

    inputs = torch.rand(8, 1)
    model = nn.Sequential(nn.Linear(1, 2), nn.Linear(2, 4), nn.Linear(4, 2), nn.Linear(2, 1))

    outputs = model(inputs)
    loss = outputs.mean()
    loss.backward()
    grad_without_pipe = sum_grad(model.parameters())
    zero_grad(model.parameters())

    model = Pipe(model, chunks=4, checkpoint=checkpoint)
    outputs = model(inputs).local_value()
    loss = outputs.mean()
    loss.backward()
    grad_with_pipe = sum_grad(model.parameters())
    assert torch.allclose(grad_with_pipe, grad_without_pipe)


class _Stage(nn.Module):
    """nn.Sequential of encoder layers as one partition (seq-first layout)."""

    def __init__(self, layers):
        super().__init__()
        self.layers = nn.ModuleList(layers)

    def forward(self, x):
        # Micro-batching is on dim 0 (batch-first); layers are seq-first.
        x = x.transpose(0, 1)
        for layer in self.layers:
            x = layer(x)
        return x.transpose(0, 1)


@pytest.mark.parametrize("checkpoint", ["never", "except_last", "always"])
def test_baseline_config1_transformer_cpu(checkpoint):
    """BASELINE.json config #1: 2-stage 2-layer TransformerEncoder, chunks=2, CPU."""
    d, h = 32, 4
    layers = [nn.TransformerEncoderLayer(d, h, 64, dropout=0.0) for _ in range(2)]
    seq = nn.Sequential(_Stage([layers[0]]), _Stage([layers[1]]))
    ref = copy.deepcopy(seq)
    x = torch.randn(6, 5, d, requires_grad=True)
    xr = x.detach().clone().requires_grad_(True)

    pipe = Pipe(seq, chunks=2, checkpoint=checkpoint)
    assert len(pipe.partitions) == 2
    out = pipe(x).local_value()
    expect = ref(xr)
    assert torch.allclose(out, expect, atol=1e-5)
    out.pow(2).mean().backward()
    expect.pow(2).mean().backward()
    assert torch.allclose(x.grad, xr.grad, atol=1e-5)
    for (n, p), (_, q) in zip(seq.named_parameters(), ref.named_parameters()):
        assert torch.allclose(p.grad, q.grad, atol=1e-5), n


def test_dropout_recompute_matches_never():
    """With dropout, 'always' (recompute) must give the same grads as 'never'."""
    torch.manual_seed(1)
    base = nn.Sequential(nn.Linear(8, 8), nn.Dropout(0.3), nn.Linear(8, 8), nn.Dropout(0.3))
    x = torch.randn(12, 8)

    grads = {}
    for mode in ("never", "always"):
        model = copy.deepcopy(base)
        pipe = Pipe(model, chunks=3, checkpoint=mode)
        torch.manual_seed(123)
        out = pipe(x).local_value()
        out.square().sum().backward()
        grads[mode] = [p.grad.clone() for p in model.parameters()]
    for a, b in zip(grads["never"], grads["always"]):
        assert torch.allclose(a, b)


def test_inplace_on_requires_grad():
    model = nn.Sequential(nn.Linear(1, 1), nn.ReLU(inplace=True))
    model = Pipe(model, checkpoint="always")
    x = torch.rand(1)
    y = model(x).local_value()
    message = r"a leaf Variable that requires grad .* used in an in-place operation."
    with pytest.raises(RuntimeError, match=message):
        y.backward()


def test_blockpartition():
    assert solve([1, 2, 3, 4, 5, 6], partitions=2) == [[1, 2, 3, 4], [5, 6]]
    assert solve([1, 2, 3, 4, 5, 6], partitions=3) == [[1, 2, 3], [4, 5], [6]]
    assert solve([1, 1, 1, 1], partitions=4) == [[1], [1], [1], [1]]
    assert solve([5, 1, 1, 1, 1, 1], partitions=2) == [[5], [1, 1, 1, 1, 1]]
    with pytest.raises(ValueError):
        solve([1], partitions=2)
    # Optimal for every split of a random sequence (brute force check).
    import itertools
    import random

    rng = random.Random(0)
    for _ in range(20):
        seq = [rng.randint(1, 20) for _ in range(7)]
        for parts in (2, 3, 4):
            best = min(
                max(sum(seq[a:b]) for a, b in zip((0,) + cut, cut + (len(seq),)))
                for cut in itertools.combinations(range(1, len(seq)), parts - 1)
            )
            sizes = solve_balance(seq, parts)
            assert sum(sizes) == len(seq) and all(s > 0 for s in sizes)
            starts = [sum(sizes[:k]) for k in range(parts)]
            got = max(sum(seq[s : s + n]) for s, n in zip(starts, sizes))
            assert got == best


def test_balance_by_time_cpu():
    class Delay(nn.Module):
        def __init__(self, seconds):
            super().__init__()
            self.seconds = seconds
            self.w = nn.Parameter(torch.ones(1))

        def forward(self, x):
            import time

            time.sleep(self.seconds)
            return x * self.w

    model = nn.Sequential(*[Delay(s) for s in (0.001, 0.001, 0.001, 0.001, 0.01, 0.01)])
    balance = balance_by_time(2, model, torch.rand(1, 1), timeout=0.3, device="cpu")
    assert balance == [5, 1]


def test_balance_by_size_mocked_profile(monkeypatch):
    """balance_by_size forwards its arguments to profile_sizes and balances the
    returned per-layer sizes (no GPU: the profiler is mocked)."""
    import mipipe.balance as B

    seen = {}

    def fake_profile_sizes(module, input, chunks, param_scale, device):
        seen.update(n=len(module), chunks=chunks, param_scale=param_scale, device=device)
        return [10, 10, 10, 10, 40, 40][: len(module)]

    monkeypatch.setattr(B, "profile_sizes", fake_profile_sizes)
    model = nn.Sequential(*[nn.Linear(2, 2) for _ in range(6)])
    balance = B.balance_by_size(2, model, torch.rand(4, 2), chunks=4, param_scale=4.0, device="cpu")
    assert balance == [5, 1] or balance == [4, 2]
    assert sum(balance) == 6
    # the largest partition cost is minimal: [4,2] -> max(40,80)=80; [5,1] -> max(80,40)=80
    assert seen == {"n": 6, "chunks": 4, "param_scale": 4.0, "device": torch.device("cpu")}
    assert B.balance_by_size(3, model, torch.rand(4, 2), device="cpu") == [4, 1, 1]


def test_partition_model():
    model = nn.Sequential(*[nn.Linear(2, 2) for _ in range(5)])
    grouped = partition_model(model, [2, 3], devices=["cpu", "cpu"])
    assert len(grouped) == 2 and len(grouped[0]) == 2 and len(grouped[1]) == 3
    from mipipe import BalanceError

    with pytest.raises(BalanceError):
        partition_model(model, [2, 2], devices=["cpu", "cpu"])
