"""@skippable / stash / pop / portals (BASELINE config #5 plumbing)."""
import pytest
import torch
from torch import nn

from mipipe import Pipe
from mipipe.skip import Namespace, inspect_skip_layout, pop, skippable, stash, verify_skippables
from mipipe.skip.layout import SkipLayout
from mipipe.skip.portal import Portal
from mipipe.skip.tracker import SkipTracker, SkipTrackerThroughPortals, current_skip_tracker, use_skip_tracker
from mipipe.microbatch import Batch


@skippable(stash=["skip"])
class Stash(nn.Module):
    def forward(self, x):
        yield stash("skip", x)
        return x


@skippable(pop=["skip"])
class Pop(nn.Module):
    def forward(self, x):
        skip = yield pop("skip")
        return x + skip


@skippable(stash=["1to3"])
class Layer1(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv = nn.Linear(3, 3)

    def forward(self, input):
        yield stash("1to3", input)
        return self.conv(input)


class Layer2(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv = nn.Linear(3, 3)

    def forward(self, input):
        return self.conv(input)


@skippable(pop=["1to3"])
class Layer3(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv = nn.Linear(3, 3)

    def forward(self, input):
        skip_1to3 = yield pop("1to3")
        return self.conv(input) + skip_1to3


def test_skippable_outside_pipe():
    model = nn.Sequential(Layer1(), Layer2(), Layer3())
    x = torch.rand(4, 3)
    l1, l2, l3 = model[0].module, model[1], model[2].module
    expect = l3.conv(l2.conv(l1.conv(x))) + x
    assert torch.allclose(model(x), expect)


@pytest.mark.parametrize("checkpoint", ["never", "always", "except_last"])
@pytest.mark.parametrize("balance_cpu", [True])
def test_1to3_through_pipe(checkpoint, balance_cpu):
    model = nn.Sequential(Layer1(), Layer2(), Layer3())
    x = torch.rand(6, 3, requires_grad=True)
    ref = model(x)
    ref.sum().backward()
    gx = x.grad.clone()
    gw = [p.grad.clone() for p in model.parameters()]
    x.grad = None
    model.zero_grad()

    pipe = Pipe(model, chunks=3, checkpoint=checkpoint)
    assert len(pipe.partitions) == 3  # CPU children -> one partition each
    out = pipe(x).local_value()
    assert torch.allclose(out, ref, atol=1e-6)
    out.sum().backward()
    assert torch.allclose(x.grad, gx, atol=1e-6)
    for p, g in zip(model.parameters(), gw):
        assert torch.allclose(p.grad, g, atol=1e-6)


def test_namespace_isolation():
    ns1, ns2 = Namespace(), Namespace()
    model = nn.Sequential(
        Stash().isolate(ns1), Stash().isolate(ns2), Pop().isolate(ns2), Pop().isolate(ns1)
    )
    verify_skippables(model)
    x = torch.ones(2, 1)
    # x -> stash1(x) -> stash2(x) -> x + x -> 2x + x
    assert torch.allclose(model(x), x * 3)
    pipe = Pipe(model, chunks=2)
    assert torch.allclose(pipe(x).local_value(), x * 3)


def test_namespace_repr_and_order():
    a, b = Namespace(), Namespace()
    assert a != b and a == a
    assert a < b
    assert "Namespace" in repr(a)
    assert len({a, b, a}) == 2


def test_verify_skippables_errors():
    @skippable(stash=["foo"], pop=["foo"])
    class StashPopFoo(nn.Module):
        def forward(self, x):
            return x

    with pytest.raises(TypeError, match="both as stashable and as poppable"):
        verify_skippables(nn.Sequential(StashPopFoo()))

    with pytest.raises(TypeError, match="as poppable but it was not stashed"):
        verify_skippables(nn.Sequential(Pop()))

    with pytest.raises(TypeError, match="no module declared 'skip' as poppable but stashed"):
        verify_skippables(nn.Sequential(Stash()))

    with pytest.raises(TypeError, match="redeclared 'skip' as stashable but not isolated by namespace"):
        verify_skippables(nn.Sequential(Stash(), Stash(), Pop()))

    with pytest.raises(TypeError, match="redeclared 'skip' as poppable"):
        verify_skippables(nn.Sequential(Stash(), Pop(), Pop()))

    # Pipe verifies at construction.
    with pytest.raises(TypeError):
        Pipe(nn.Sequential(Stash()))


def test_undeclared_commands():
    @skippable(stash=["a"])
    class Bad(nn.Module):
        def forward(self, x):
            yield stash("b", x)
            return x

    with pytest.raises(RuntimeError, match="has not been declared as stashable"):
        Bad()(torch.zeros(1))

    @skippable(stash=["a"])
    class NoStash(nn.Module):
        def forward(self, x):
            return x

    with pytest.raises(RuntimeError, match="must be stashed but have not"):
        NoStash()(torch.zeros(1))

    @skippable()
    class BadCmd(nn.Module):
        def forward(self, x):
            yield "junk"
            return x

    with pytest.raises(TypeError, match="is not a command"):
        BadCmd()(torch.zeros(1))


def test_inspect_skip_layout():
    a, b, c, d = Stash(), nn.Linear(1, 1), Pop(), nn.Linear(1, 1)
    partitions = [nn.Sequential(a, b), nn.Sequential(c), nn.Sequential(d)]
    layout = inspect_skip_layout(partitions)
    assert layout.requires_copy(None, "skip")
    assert list(layout.copy_policy(0)) == []
    assert list(layout.copy_policy(1)) == [(0, None, "skip")]
    assert list(layout.copy_policy(2)) == []

    same = inspect_skip_layout([nn.Sequential(Stash(), Pop())])
    assert not same.requires_copy(None, "skip")
    assert list(same.copy_policy(0)) == []


def test_portal_tensor_life():
    t = torch.zeros(1)
    p = Portal(t, 2)
    assert p.use_tensor() is t
    assert p.use_tensor() is t
    assert p.tensor is None
    with pytest.raises(RuntimeError):
        p.use_tensor()
    p.put_grad(torch.ones(1))
    assert p.use_grad() is not None and p.use_grad() is None


def test_tracker_default_is_plain_and_scoped():
    t = current_skip_tracker()
    assert type(t) is SkipTracker
    tp = SkipTrackerThroughPortals(SkipLayout(1, {}))
    with use_skip_tracker(tp):
        assert current_skip_tracker() is tp
    assert current_skip_tracker() is t
    with pytest.raises(TypeError):
        t.copy(Batch(torch.zeros(1)), None, None, None, "x")


def test_skip_memory_freed_after_pop():
    # Portal drops its tensor once used (no leak across iterations).
    model = nn.Sequential(Layer1(), Layer2(), Layer3())
    pipe = Pipe(model, chunks=2, checkpoint="never")
    x = torch.rand(4, 3, requires_grad=True)
    out = pipe(x).local_value()
    out.sum().backward()
    out2 = pipe(x).local_value()
    out2.sum().backward()
