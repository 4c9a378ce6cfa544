"""FlatAdam(defer_wgrad=True): the process-wide weight-gradient queue with
several optimizers (ownership of the deferral).

The GEMMs are replaced by a host fake with the same contract as the native
``linear_wgrad`` (``main = dy^T x`` or ``main += dy^T x``), so the queueing,
flushing and dropping logic runs on CPU."""
import pytest
import torch
from torch import nn

import importlib

lin = importlib.import_module("mipipe.ops.linear")  # the module (mipipe.ops.linear is also a function)
from mipipe.optim import FlatAdam


class _FakeK:
    def linear_wgrad(self, dy, x, main, accumulate):
        g = dy.t().float() @ x.float()
        if accumulate:
            main.add_(g)
        else:
            main.copy_(g)

    def linear_wgrad_segments(self, dys, xs, main, accumulate):
        for i, (d, x) in enumerate(zip(dys, xs)):
            self.linear_wgrad(d, x, main, accumulate or i > 0)

    def column_sum_segments(self, dys, main, accumulate):
        s = sum(d.float().sum(0) for d in dys)
        if accumulate:
            main.add_(s)
        else:
            main.copy_(s)


@pytest.fixture
def fake_kernels(monkeypatch):
    monkeypatch.setattr(lin, "kernels_for", lambda t: _FakeK())
    yield
    lin._DEFERRED = None


def _queue(p, dy, x):
    """What the tile-path backward does for a weight inside a deferral."""
    lin._defer(p, dy, x)


def _lazy_weight(n, k):
    w = nn.Parameter(torch.randn(n, k))
    lin.mark_gemm_weight(w)
    return w


def test_second_deferring_optimizer_flushes_shared_queue(fake_kernels):
    w1, w2 = _lazy_weight(4, 8), _lazy_weight(4, 8)
    o1 = FlatAdam([w1], lr=0.1, defer_wgrad=True)
    o2 = FlatAdam([w2], lr=0.1, defer_wgrad=True)
    o1.zero_grad()
    o2.zero_grad()  # the deferral is o1's; o2 joins the shared queue
    assert o1._deferring and not o2._deferring
    dy, x = torch.randn(64, 4), torch.randn(64, 8)
    _queue(w1, dy, x)
    _queue(w2, 2 * dy, x)
    # o2 steps first: it must flush the queue holding its weight instead of
    # stepping on zeroed "fresh" gradients
    o2.fold_grads()
    assert torch.allclose(w2.main_grad, (2 * dy).t() @ x, atol=1e-5)
    assert lin._DEFERRED == {}  # flushed, still open for the owner
    assert torch.allclose(w1.main_grad, dy.t() @ x, atol=1e-5)  # flushed together
    o1.fold_grads()
    assert lin._DEFERRED is None
    assert torch.allclose(w1.main_grad, dy.t() @ x, atol=1e-5)


def test_zero_grad_drops_queue_without_running_it(fake_kernels):
    w = _lazy_weight(4, 8)
    o = FlatAdam([w], lr=0.1, defer_wgrad=True)
    o.zero_grad()
    calls = []
    _FakeK.linear_wgrad_segments, orig = (lambda self, *a: calls.append(a)), _FakeK.linear_wgrad_segments
    try:
        _queue(w, torch.randn(64, 4), torch.randn(64, 8))
        o.zero_grad()  # an eval / aborted backward: drop, do not run
        assert not calls
        assert id(w) not in lin.deferred_param_ids()
        assert o._deferring
        o.fold_grads()  # nothing queued: the fresh weight is zeroed
        assert torch.count_nonzero(w.main_grad) == 0
    finally:
        _FakeK.linear_wgrad_segments = orig


def test_zero_grad_keeps_other_optimizers_queue(fake_kernels):
    w1, w2 = _lazy_weight(4, 8), _lazy_weight(4, 8)
    o1 = FlatAdam([w1], lr=0.1, defer_wgrad=True)
    o2 = FlatAdam([w2], lr=0.1, defer_wgrad=True)
    o1.zero_grad()
    o2.zero_grad()
    dy, x = torch.randn(64, 4), torch.randn(64, 8)
    _queue(w1, dy, x)
    _queue(w2, dy, x)
    o2.zero_grad()  # drops only w2's entry
    assert lin.deferred_param_ids() == {id(w1)}
    o1.fold_grads()
    assert torch.allclose(w1.main_grad, dy.t() @ x, atol=1e-5)
