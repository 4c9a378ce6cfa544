"""Pipe API behaviour on CPU partitions (BASELINE config #1 plumbing).

Every CPU child becomes its own partition, so these run real multi-stage
pipelines with no GPU (SURVEY §4 'CPU devices as a fake backend')."""
import copy
from collections import OrderedDict
import time

import pytest
import torch
from torch import nn

from mipipe import LocalRRef, NoChunk, Pipe, WithDevice
from mipipe.pipe import PipeSequential


def _out(pipe, *x):
    return pipe(*x).local_value()


def test_parameters():
    model = nn.Sequential(nn.Linear(1, 1))
    pipe = Pipe(model, chunks=1)
    assert list(pipe.parameters()) != []


def test_public_attrs():
    class MyString:
        def __init__(self, value):
            self.value = value

        def __str__(self):
            return self.value

    model = nn.Sequential(nn.Linear(1, 1))
    pipe = Pipe(model, chunks=42.000, checkpoint=MyString("always"))
    assert pipe.devices == [torch.device("cpu")]
    assert pipe.chunks == 42
    assert isinstance(pipe.chunks, int)
    assert pipe.checkpoint == "always"
    assert isinstance(pipe.checkpoint, str)


def test_sequential_like():
    a = nn.Linear(1, 1)
    b = nn.Linear(1, 1)
    model = nn.Sequential(a, b)
    pipe = Pipe(model)
    assert len(pipe) == 2
    assert list(pipe) == [a, b]
    assert pipe[0] is a
    assert pipe[1] is b
    with pytest.raises(IndexError):
        _ = pipe[2]
    assert pipe[-1] is b
    assert pipe[-2] is a
    with pytest.raises(IndexError):
        _ = pipe[-3]


def test_chunks_less_than_1():
    model = nn.Sequential(nn.Linear(1, 1))
    with pytest.raises(ValueError):
        Pipe(model, chunks=0)
    with pytest.raises(ValueError):
        Pipe(model, chunks=-1)


def test_batch_size_indivisible():
    model = nn.Sequential(nn.Linear(1, 1))
    pipe = Pipe(model, chunks=4)
    _out(pipe, torch.rand(7, 1))


def test_batch_size_small():
    model = nn.Sequential(nn.Linear(1, 1))
    pipe = Pipe(model, chunks=4)
    _out(pipe, torch.rand(2, 1))


@pytest.mark.parametrize("mode,expected", [("always", 2), ("except_last", 1), ("never", 0)])
def test_checkpoint_modes(mode, expected):
    def count_grad_fn(grad_fn, name, visited=None):
        visited = visited or set()
        if grad_fn in visited:
            return 0
        visited.add(grad_fn)
        if grad_fn is None:
            return 0
        if grad_fn.__class__.__name__ == name:
            return 1
        return sum(count_grad_fn(f, name, visited) for f, _ in grad_fn.next_functions)

    model = nn.Sequential(nn.Linear(1, 1))
    input = torch.rand(2, 1)
    pipe = Pipe(model, chunks=2, checkpoint=mode)
    output = _out(pipe, input)
    assert count_grad_fn(output.grad_fn, "CheckpointBackward") == expected


def test_checkpoint_mode_invalid():
    model = nn.Sequential(nn.Linear(1, 1))
    with pytest.raises(ValueError, match="checkpoint is not one of 'always', 'except_last', or 'never'"):
        Pipe(model, chunks=2, checkpoint="INVALID_CHECKPOINT")


def test_checkpoint_mode_when_chunks_1():
    model = nn.Sequential(nn.Linear(1, 1))
    # All checkpoint modes are fine.
    for mode in ("except_last", "always", "never"):
        _out(Pipe(model, chunks=1, checkpoint=mode), torch.rand(2, 1))


def test_checkpoint_eval():
    model = nn.Sequential(nn.Linear(1, 1))
    pipe = Pipe(model, chunks=2)
    input = torch.rand(2, 1)

    def find_grad_fn(grad_fn, name):
        if grad_fn is None:
            return False
        if grad_fn.__class__.__name__ == name:
            return True
        return any(find_grad_fn(f, name) for f, _ in grad_fn.next_functions)

    pipe.train()
    assert find_grad_fn(_out(pipe, input).grad_fn, "RecomputeBackward")
    pipe.eval()
    assert not find_grad_fn(_out(pipe, input).grad_fn, "RecomputeBackward")


def test_checkpoint_non_float_input():
    class ForkNonFloat(nn.Module):
        def forward(self, input):
            return (input * 2, torch.tensor([False]))

    class JoinNonFloat(nn.Module):
        def forward(self, input, non_float):
            return input * 2

    model = nn.Sequential(ForkNonFloat(), JoinNonFloat())
    pipe = Pipe(model, chunks=1, checkpoint="always")
    input = torch.rand(1, requires_grad=True)
    output = _out(pipe, input)
    output.backward()


def test_no_grad():
    model = nn.Sequential(nn.Linear(1, 1))
    pipe = Pipe(model, chunks=2)
    input = torch.rand(2, 1)
    latent = None

    def hook(module, input, output):
        nonlocal latent
        latent = output

    partition = pipe.partitions[0]
    partition.register_forward_hook(hook)
    with torch.no_grad():
        _out(pipe, input)
    assert latent.grad_fn is None


def test_exception():
    class ExpectedException(Exception):
        pass

    class Raise(nn.Module):
        def forward(self, *_):
            raise ExpectedException()

    model = nn.Sequential(Raise())
    pipe = Pipe(model, chunks=1)
    with pytest.raises(ExpectedException):
        pipe(torch.rand(1))


def test_exception_early_stop_asap():
    """Even if the first partitions have finished to process, the partition
    before the failed partition should be killed as soon as possible."""

    class ExpectedException(Exception):
        pass

    class Pass(nn.Module):
        def forward(self, x):
            return x

    counter = 0

    class Counter(nn.Module):
        def forward(self, x):
            time.sleep(0.05)
            nonlocal counter
            counter += 1
            return x

    class Raise(nn.Module):
        def forward(self, x):
            raise ExpectedException()

    model = nn.Sequential(Pass(), Pass(), Counter(), Raise())
    pipe = Pipe(model, chunks=3)
    with pytest.raises(ExpectedException):
        pipe(torch.rand(3))
    # If the early stop doesn't work, it would be 3 instead.
    assert counter == 2


def test_nested_input():
    class NestedInput(nn.Module):
        def __init__(self):
            super().__init__()
            self.fc_a = nn.Linear(1, 1)
            self.fc_b = nn.Linear(1, 1)

        def forward(self, inp):
            return inp

    model = nn.Sequential(NestedInput())
    pipe = Pipe(model, chunks=2)
    a = torch.rand(10, 1, requires_grad=True)
    b = torch.rand(10, 1, requires_grad=True)
    # TypeError: expected Tensor, but got tuple
    with pytest.raises(TypeError):
        _out(pipe, (a, (a, b)))


def test_input_pair():
    class Two(nn.Module):
        def __init__(self):
            super().__init__()
            self.fc_a = nn.Linear(1, 1)
            self.fc_b = nn.Linear(1, 1)

        def forward(self, a, b):
            return (self.fc_a(a), self.fc_b(b))

    model = nn.Sequential(Two())
    pipe = Pipe(model, chunks=2)
    a = torch.rand(10, 1, requires_grad=True)
    b = torch.rand(10, 1, requires_grad=True)
    a_out, b_out = _out(pipe, a, b)
    loss = (a_out + b_out).mean()
    loss.backward()
    assert a.grad is not None
    assert b.grad is not None


def test_multi_sequence_input():
    class MultiSeq(nn.Module):
        def forward(self, tup1, tup2):
            return tup1, tup2

    model = Pipe(nn.Sequential(MultiSeq()))
    with pytest.raises(TypeError):
        model([torch.rand(10), torch.rand(10)], [torch.rand(10), torch.rand(10)])


def test_input_singleton():
    class One(nn.Module):
        def __init__(self):
            super().__init__()
            self.fc = nn.Linear(1, 1)

        def forward(self, a):
            return (self.fc(a),)

    model = nn.Sequential(One())
    pipe = Pipe(model, chunks=2)
    a = torch.rand(10, 1, requires_grad=True)
    (a_out,) = _out(pipe, a)
    a_out.mean().backward()
    assert all(p.grad is not None for p in model.parameters())
    assert a.grad is not None


def test_input_varargs():
    model = nn.Sequential(nn.Linear(1, 1))
    pipe = Pipe(model)
    a = torch.rand(1)
    b = torch.rand(1)
    # TypeError: forward() takes 2 positional arguments but 3 were given
    with pytest.raises(TypeError):
        pipe(a, b)


def test_non_tensor():
    class NonTensor(nn.Module):
        def forward(self, _):
            return "hello"

    model = nn.Sequential(NonTensor())
    pipe = Pipe(model)
    x = torch.rand(1)
    with pytest.raises(TypeError):
        pipe(x)
    with pytest.raises(TypeError):
        pipe("hello")


def test_non_tensor_sequence():
    class NonTensorTuple(nn.Module):
        def forward(self, x):
            return (x, "hello")

    class NonTensorArgs(nn.Module):
        def forward(self, x: str, y: bool):
            return x, y

    model = nn.Sequential(NonTensorTuple())
    pipe = Pipe(model)
    x = torch.rand(1)
    with pytest.raises(TypeError):
        pipe((x, "hello"))
    with pytest.raises(TypeError):
        pipe([x, "hello"])

    model = nn.Sequential(NonTensorArgs())
    pipe = Pipe(model)
    with pytest.raises(TypeError):
        # Need at least one Tensor.
        pipe("hello", True)


@pytest.mark.parametrize("checkpoint", ["never", "always", "except_last"])
def test_valid_non_tensor(checkpoint):
    class NonTensor1(nn.Module):
        def forward(self, a: int, b, c: str, d: bool):
            return (a, c, b, d)

    class NonTensor2(nn.Module):
        def forward(self, a: int, c: str, b, d: bool):
            if isinstance(b, torch.Tensor):
                b = b + 1.0
            return a, c, b, d

    model = nn.Sequential(NonTensor1(), NonTensor2())
    pipe = Pipe(model, chunks=2, checkpoint=checkpoint)
    t = torch.rand(10, 1)
    a, c, b, d = _out(pipe, 1, t, "x", True)
    assert a == [1, 1]
    assert c == ["x", "x"]
    assert torch.allclose(b, t + 1.0)
    assert d == [True, True]


def test_deferred_batch_norm():
    bn = nn.BatchNorm2d(3)
    pipe_bn = nn.BatchNorm2d(3)
    pipe = Pipe(nn.Sequential(pipe_bn), chunks=2, deferred_batch_norm=True)
    x = torch.rand(4, 3, 10, 10)
    _out(pipe, x).mean().backward()
    bn(x).mean().backward()
    assert torch.allclose(pipe[0].running_mean, bn.running_mean, atol=1e-4)
    assert torch.allclose(pipe[0].running_var, bn.running_var, atol=1e-4)


def test_deferred_batch_norm_params():
    bn = nn.BatchNorm2d(3)
    pipe_bn = nn.BatchNorm2d(3)
    pipe = Pipe(nn.Sequential(pipe_bn), chunks=1, deferred_batch_norm=True)
    x = torch.rand(4, 3, 10, 10)
    _out(pipe, x).mean().backward()
    bn(x).mean().backward()
    assert pipe[0].weight.grad is not None
    assert pipe[0].bias.grad is not None
    assert torch.allclose(pipe[0].weight.grad, bn.weight.grad, atol=1e-4)
    assert torch.allclose(pipe[0].bias.grad, bn.bias.grad, atol=1e-4)


def test_partitions():
    a = nn.Linear(1, 1)
    b = nn.Linear(1, 1)
    model = nn.Sequential(a, b)
    pipe = Pipe(model)
    assert isinstance(pipe.partitions, nn.ModuleList)
    assert isinstance(pipe.partitions[0], nn.Sequential)
    assert isinstance(pipe.partitions[1], nn.Sequential)
    assert "partitions.0.0.weight" in pipe.state_dict()


def test_deny_moving():
    a = nn.Linear(1, 1)
    b = nn.Linear(1, 1)
    model = nn.Sequential(a, b)
    pipe = Pipe(model)
    # Moving is denied.
    with pytest.raises(TypeError):
        pipe.cuda()
    with pytest.raises(TypeError):
        pipe.cpu()
    with pytest.raises(TypeError):
        pipe.to(torch.device("cuda"))
    with pytest.raises(TypeError):
        pipe.to(0)
    with pytest.raises(TypeError):
        pipe.to("cuda")
    with pytest.raises(TypeError):
        pipe.to(device=0)
    with pytest.raises(TypeError):
        pipe.to(torch.rand(1))
    with pytest.raises(TypeError):
        pipe.to(tensor=torch.rand(1))
    # Casting is allowed.
    pipe.half()
    pipe.to(torch.double)
    pipe.to(dtype=torch.float)


def test_empty_module():
    # Empty sequential module is not illegal.
    model = nn.Sequential()
    model = Pipe(model)
    assert model(torch.tensor(42)).local_value() == torch.tensor(42)
    # But only tensor or tensors is legal in Pipe.
    with pytest.raises(TypeError):
        model(42)


def test_named_children():
    a = nn.Linear(1, 1)
    b = nn.Linear(1, 1)
    model = nn.Sequential(OrderedDict([("a", a), ("b", b)]))
    pipe = Pipe(model)
    names = {n for n, _ in pipe.named_modules()}
    assert "partitions.0.0" in names
    assert "partitions.1.0" in names
    # Pipe doesn't support __getattr__. Unlike nn.Sequential, Pipe requires
    # several methods in its namespace.
    with pytest.raises(AttributeError):
        pipe.a


def test_verify_module_non_sequential():
    with pytest.raises(TypeError, match="module must be nn.Sequential to be partitioned"):
        Pipe(nn.Module())


def test_verify_module_duplicate_children():
    conv = nn.Conv2d(3, 3, 1)
    model = nn.Sequential(conv, conv)
    with pytest.raises(ValueError, match="module with duplicate children is not supported"):
        Pipe(model)


def test_return_plain_output():
    model = nn.Sequential(nn.Linear(2, 2))
    pipe = Pipe(model, chunks=2, return_rref=False)
    out = pipe(torch.rand(4, 2))
    assert torch.is_tensor(out)
    rref = Pipe(model, chunks=2)(torch.rand(4, 2))
    assert isinstance(rref, LocalRRef)
    assert torch.is_tensor(rref.to_here())


def test_with_device_wrapper_cpu():
    fc1 = nn.Linear(16, 8)
    fc2 = nn.Linear(8, 4)
    dropout = nn.Dropout()
    model = nn.Sequential(fc1, fc2, WithDevice(dropout, "cpu"))
    model = Pipe(model, chunks=8)
    assert torch.device("cpu") == model(torch.rand(16, 16)).local_value().device
    assert [torch.device("cpu")] * 3 == model.devices


def test_pipe_sequential_multiple_inputs():
    class Add(nn.Module):
        def forward(self, a, b):
            return a + b

    class Split(nn.Module):
        def forward(self, x):
            return x, x * 2

    seq = PipeSequential(Split(), Add())
    assert torch.equal(seq(torch.ones(2)), torch.full((2,), 3.0))


def test_nochunk_replicated():
    class UseWeight(nn.Module):
        def forward(self, x, w):
            assert w.shape == (3,)
            return x * w.sum()

    pipe = Pipe(nn.Sequential(UseWeight()), chunks=4)
    x = torch.rand(8, 1)
    w = torch.ones(3)
    out = pipe(x, NoChunk(w)).local_value()
    assert torch.allclose(out, x * 3)


def test_shared_params_same_device_ok():
    lin = nn.Linear(2, 2)
    model = nn.Sequential(lin, nn.Sequential(lin))
    # Both on CPU -> each its own partition, but same device -> allowed.
    Pipe(model)


# ------------------------------------------------------------------ explicit balance
def test_balance_groups_children():
    """balance=[2, 2]: two partitions of two children each (the reference rule
    alone would make four CPU partitions)."""
    model = nn.Sequential(nn.Linear(4, 4), nn.ReLU(), nn.Linear(4, 4), nn.Linear(4, 4))
    pipe = Pipe(model, chunks=2, balance=[2, 2])
    assert len(pipe.partitions) == 2
    assert [len(p) for p in pipe.partitions] == [2, 2]
    assert len(Pipe(model, chunks=2).partitions) == 4
    pipe.close()


@pytest.mark.parametrize("balance", [[1, 1], [2, 3], [0, 4], [-1, 5]])
def test_balance_errors(balance):
    from mipipe import BalanceError

    model = nn.Sequential(*[nn.Linear(2, 2) for _ in range(4)])
    with pytest.raises(BalanceError):
        Pipe(model, balance=balance)


def test_balance_partition_spanning_devices():
    model = nn.Sequential(nn.Linear(2, 2), nn.Linear(2, 2, device="meta"))
    with pytest.raises(ValueError, match="spans several devices"):
        Pipe(model, balance=[2])


def test_balance_parameterless_child_joins_partition():
    """An unpinned activation has no device of its own: it runs in its partition."""
    model = nn.Sequential(nn.Linear(2, 2), nn.ReLU(), nn.Linear(2, 2))
    pipe = Pipe(model, chunks=1, balance=[2, 1])
    assert [type(m) for m in pipe.partitions[0]] == [nn.Linear, nn.ReLU]
    pipe.close()


@pytest.mark.parametrize("checkpoint", ["never", "except_last", "always"])
@pytest.mark.parametrize("balance", [[1, 2, 1], [2, 2], [4]])
def test_balance_transparency(checkpoint, balance):
    torch.manual_seed(0)
    model = nn.Sequential(nn.Linear(8, 8), nn.Tanh(), nn.Linear(8, 8), nn.Linear(8, 4))
    ref = copy.deepcopy(model)
    x = torch.randn(12, 8)
    pipe = Pipe(model, chunks=3, checkpoint=checkpoint, balance=balance, copy_same_device=True)
    assert len(pipe.partitions) == len(balance)
    out = pipe(x).local_value()
    out.sum().backward()
    y = ref(x)
    y.sum().backward()
    assert torch.allclose(out, y, atol=1e-6)
    for p, q in zip(model.parameters(), ref.parameters()):
        assert torch.allclose(p.grad, q.grad, atol=1e-6)
    pipe.close()


def test_copy_engine_validation():
    with pytest.raises(ValueError, match="copy_engine"):
        Pipe(nn.Sequential(nn.Linear(2, 2)), copy_engine="tcp")


def test_transfer_policy_kept_for_backward():
    """Copy keeps the policy in force at forward for its backward (which runs
    later on an autograd thread, outside the pipeline's context)."""
    from mipipe.copy import Copy, current_policy, transfer_policy
    from mipipe.stream import CPUStream

    x = torch.randn(3, requires_grad=True)
    with transfer_policy(True, "blit"):
        assert current_policy() == (True, 1)
        (y,) = Copy.apply(CPUStream, CPUStream, x)
    assert current_policy()[0] is False
    y.sum().backward()
    assert torch.equal(x.grad, torch.ones(3))
    with pytest.raises(ValueError):
        with transfer_policy(True, "pcie"):
            pass
