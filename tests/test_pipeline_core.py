"""Clock cycles, dependency, phony, stream, worker, checkpoint plumbing (CPU)."""
import threading

import pytest
import torch
from torch import nn

from mipipe.checkpoint import (
    Checkpointing,
    checkpoint,
    is_checkpointing,
    is_recomputing,
)
from mipipe.dependency import Fork, Join, fork, join
from mipipe.microbatch import Batch
from mipipe.phony import get_phony
from mipipe.pipeline import checkpoint_stop_for, clock_cycles
from mipipe.stream import (
    CPUStream,
    current_stream,
    default_stream,
    get_device,
    is_cuda,
    new_stream,
    record_stream,
    use_device,
    use_stream,
    wait_stream,
)
from mipipe.worker import Task, create_workers, release_workers


def test_clock_cycles():
    assert list(clock_cycles(1, 1)) == [[(0, 0)]]
    assert list(clock_cycles(1, 3)) == [[(0, 0)], [(0, 1)], [(0, 2)]]
    assert list(clock_cycles(3, 1)) == [[(0, 0)], [(1, 0)], [(2, 0)]]
    assert list(clock_cycles(3, 3)) == [
        [(0, 0)],
        [(1, 0), (0, 1)],
        [(2, 0), (1, 1), (0, 2)],
        [(2, 1), (1, 2)],
        [(2, 2)],
    ]
    assert list(clock_cycles(4, 2)) == [
        [(0, 0)],
        [(1, 0), (0, 1)],
        [(2, 0), (1, 1)],
        [(3, 0), (2, 1)],
        [(3, 1)],
    ]


@pytest.mark.parametrize("m,n", [(1, 1), (4, 2), (8, 8), (32, 8), (3, 5)])
def test_clock_cycles_cover_every_cell_once(m, n):
    seen = [c for tick in clock_cycles(m, n) for c in tick]
    assert sorted(seen) == sorted((i, j) for i in range(m) for j in range(n))
    assert len(list(clock_cycles(m, n))) == m + n - 1


def test_checkpoint_stop():
    assert checkpoint_stop_for("always", 4) == 4
    assert checkpoint_stop_for("except_last", 4) == 3
    assert checkpoint_stop_for("never", 4) == 0
    # derived from the actual micro-batch count (README.md:398 fix)
    assert checkpoint_stop_for("except_last", 1) == 0
    with pytest.raises(ValueError):
        checkpoint_stop_for("sometimes", 4)


# -- phony / dependency -------------------------------------------------------
def test_phony_cached_and_empty():
    p1 = get_phony(torch.device("cpu"), requires_grad=False)
    p2 = get_phony(torch.device("cpu"), requires_grad=False)
    p3 = get_phony(torch.device("cpu"), requires_grad=True)
    assert p1 is p2
    assert p1 is not p3
    assert p1.numel() == 0 and p3.requires_grad


def test_fork_join_identity_and_edge():
    x = torch.ones(2, requires_grad=True)
    y, phony = fork(x)
    assert y.grad_fn.__class__.__name__.startswith("Fork")
    z = join(torch.zeros(2, requires_grad=True), phony)
    (y.sum() + z.sum()).backward()
    assert torch.equal(x.grad, torch.ones(2))


def test_fork_without_grad_is_passthrough():
    x = torch.ones(2)
    y, phony = fork(x)
    assert y is x
    assert join(y, phony) is y


def test_fork_join_orders_backward():
    order = []

    class Log(torch.autograd.Function):
        @staticmethod
        def forward(ctx, tag, x):
            ctx.tag = tag
            return x.detach()

        @staticmethod
        def backward(ctx, g):
            order.append(ctx.tag)
            return None, g

    a = torch.ones(1, requires_grad=True)
    b = torch.ones(1, requires_grad=True)
    a1 = Log.apply("a", a)
    b1 = Log.apply("b", b)
    a2, phony = fork(a1)
    b2 = join(b1, phony)
    # b's backward must finish before a's Fork can run.
    (a2 + b2).backward()
    assert order == ["b", "a"]


# -- stream (CPU) -------------------------------------------------------------
def test_cpu_stream_api():
    cpu = torch.device("cpu")
    assert new_stream(cpu) is CPUStream
    assert current_stream(cpu) is CPUStream
    assert default_stream(cpu) is CPUStream
    assert not is_cuda(CPUStream)
    assert get_device(CPUStream) == cpu
    with use_device(cpu), use_stream(CPUStream):
        pass
    wait_stream(CPUStream, CPUStream)
    record_stream(torch.zeros(1), CPUStream)


# -- worker -------------------------------------------------------------------
def test_worker_runs_and_reports_errors():
    ins, outs, entries = create_workers([torch.device("cpu"), torch.device("cpu")])
    assert ins[0] is ins[1]  # one worker per unique device

    def ok():
        return Batch(torch.tensor(threading.current_thread().name != "MainThread"))

    def bad():
        raise ValueError("boom")

    ins[0].put(Task(CPUStream, compute=ok, finalize=None))
    ins[0].put(Task(CPUStream, compute=bad, finalize=None))
    good, payload = outs[0].get()
    assert good and payload[1].tensor.item()
    good, exc = outs[0].get()
    assert not good and exc[0] is ValueError
    release_workers(entries)
    good, payload = outs[0].get(timeout=5)
    assert not good and payload is None


def test_task_captures_grad_mode():
    with torch.no_grad():
        t = Task(CPUStream, compute=lambda: Batch(torch.tensor(torch.is_grad_enabled())), finalize=None)
    assert not t.compute().tensor.item()


# -- checkpoint ---------------------------------------------------------------
def test_checkpoint_function_matches():
    lin = nn.Linear(3, 3)
    x = torch.randn(4, 3, requires_grad=True)
    y_ref = torch.tanh(lin(x)).sum()
    y_ref.backward()
    g_ref = x.grad.clone()
    w_ref = lin.weight.grad.clone()
    x.grad = None
    lin.weight.grad = None
    y = checkpoint(lambda t: torch.tanh(lin(t)), x).sum()
    y.backward()
    assert torch.allclose(x.grad, g_ref)
    assert torch.allclose(lin.weight.grad, w_ref)


def test_checkpoint_flags():
    flags = []

    def f(x):
        flags.append((is_checkpointing(), is_recomputing()))
        return x * 2

    x = torch.ones(1, requires_grad=True)
    checkpoint(f, x).sum().backward()
    assert flags == [(True, False), (False, True)]
    assert not is_checkpointing() and not is_recomputing()


def test_checkpoint_dropout_deterministic():
    drop = nn.Dropout(0.5)
    x = torch.ones(1000, requires_grad=True)
    y = checkpoint(drop, x)
    y.sum().backward()
    # gradient mask equals the forward mask because the RNG state was replayed
    assert torch.equal((x.grad != 0), (y.detach() != 0))


def test_checkpoint_non_float_outputs_detached():
    def f(x):
        return x * 2, torch.arange(3)

    b = Batch(torch.ones(2, requires_grad=True))
    chk = Checkpointing(f, b)
    out = chk.checkpoint()
    assert not out[1].requires_grad


def test_recompute_expected_only_when_backward_will_recompute():
    """recompute_expected() (ops.attention keeps its dropout keep words for the recompute only then): True inside a
    checkpointed forward taken with grad enabled, False for a training-mode forward under no_grad, False outside."""
    from mipipe.checkpoint import checkpoint, recompute_expected

    seen = []

    def f(t):
        seen.append((is_checkpointing(), is_recomputing(), recompute_expected()))
        return t * 2

    x = torch.ones(3, requires_grad=True)
    y = checkpoint(f, x)
    y.sum().backward()
    assert seen == [(True, False, True), (False, True, False)]
    seen.clear()
    with torch.no_grad():
        checkpoint(f, torch.ones(3))
    assert seen == [(True, False, False)]
    assert not recompute_expected()
