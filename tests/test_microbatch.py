import pytest
import torch
from torch import nn

from mipipe.microbatch import Batch, NoChunk, check, gather, scatter


def test_batch_atomic():
    x = torch.tensor(42)
    b = Batch(x)
    assert b.atomic
    assert b.tensor is x
    assert b.tensors == (x,)
    assert list(b) == [x]
    assert len(b) == 1
    assert b[0] is x


def test_batch_non_atomic():
    x, y = torch.tensor(42), torch.tensor(21)
    b = Batch((x, y))
    assert not b.atomic
    with pytest.raises(AttributeError):
        b.tensor
    assert list(b) == [x, y]
    assert b.values == (x, y)
    assert len(b) == 2


def test_batch_requires_a_tensor():
    with pytest.raises(TypeError):
        Batch((1, 2))
    with pytest.raises(TypeError):
        Batch(3)


def test_batch_call():
    a = Batch(torch.tensor(42))
    b = Batch((torch.tensor(42), torch.tensor(21)))

    def f(x):
        return x

    def g(x, y):
        return x, y

    assert a.call(f).atomic
    assert not b.call(g).atomic


def test_batch_setitem_by_index():
    a = Batch(torch.tensor(42))
    b = Batch((torch.tensor(42), torch.tensor(21)))
    a[0] = torch.tensor(0)
    b[0] = torch.tensor(0)
    assert a.atomic and a[0].item() == 0
    assert not b.atomic and len(b) == 2 and b[0].item() == 0
    with pytest.raises(IndexError):
        a[1] = torch.tensor(1)


def test_batch_setitem_by_slice():
    a = Batch(torch.tensor(42))
    b = Batch((torch.tensor(42), torch.tensor(21)))
    a[:] = (torch.tensor(0),)
    b[:] = (torch.tensor(0),)
    assert a.atomic and a[0].item() == 0
    assert not b.atomic and len(b) == 1
    with pytest.raises(NotImplementedError):
        b[0:1] = (torch.tensor(1),)


def test_find_tensor_idx_and_device():
    b = Batch([1, torch.zeros(2), torch.ones(1)])
    assert b.find_tensor_idx() == 1
    assert b.get_device() == torch.device("cpu")


def test_check():
    check(torch.device("cpu"), torch.tensor(7))
    check(torch.device("cpu"), torch.tensor(7), 3)
    with pytest.raises(TypeError):
        check(torch.device("cpu"), 7)
    with pytest.raises(TypeError):
        check(torch.device("cpu"), "str")


def test_scatter_tensor():
    x = torch.zeros(1, 1)
    batches = scatter(x, chunks=4)
    assert len(batches) == 1
    assert batches[0].atomic


def test_scatter_fewer_chunks_than_requested():
    # chunk() semantics: 20 rows into 8 chunks gives 7 micro-batches
    # (/root/reference/README.md:398).
    x = torch.zeros(20, 3)
    assert len(scatter(x, chunks=8)) == 7


def test_scatter_multiple_tensors():
    a = torch.zeros(2, 1)
    b = torch.zeros(2, 2)
    a0, a1 = scatter(a, b, chunks=2)
    assert a0[0].shape == (1, 1) and a0[1].shape == (1, 2)
    assert a1[0].shape == (1, 1)


def test_scatter_nochunk_and_non_tensor():
    x = torch.arange(8.0).view(4, 2)
    w = torch.ones(3)
    bs = scatter(x, NoChunk(w), 5, chunks=2)
    assert len(bs) == 2
    for b in bs:
        assert b[1] is w
        assert b[2] == 5
        assert b[0].shape == (2, 2)


def test_scatter_mismatched_chunks():
    with pytest.raises(RuntimeError):
        scatter(torch.zeros(4, 1), torch.zeros(2, 1), chunks=4)


def test_nochunk_requires_tensor():
    with pytest.raises(TypeError):
        NoChunk(3)


def test_gather_tensors():
    a = torch.zeros(1, 1)
    b = torch.zeros(1, 1)
    ab = gather([Batch(a), Batch(b)])
    assert ab.size() == (2, 1)


def test_gather_tuples_and_non_tensors():
    a = (torch.zeros(1, 1), torch.zeros(2, 2), 5)
    b = (torch.zeros(1, 1), torch.zeros(2, 2), 5)
    out = gather([Batch(a), Batch(b)])
    assert isinstance(out, tuple)
    assert out[0].size() == (2, 1)
    assert out[1].size() == (4, 2)
    assert out[2] == [5, 5]


def test_gather_type_mismatch():
    with pytest.raises(TypeError):
        gather([Batch((torch.zeros(1), 5)), Batch((torch.zeros(1), "x"))])
