"""The chunk layout of FlatAdam's overlapped step (CPU: pure arithmetic; the
GPU behaviour is tests/test_gpu_optim_overlap.py)."""
import random

import torch

from mipipe.optim import FlatAdam, overlap_chunks


def _check(sizes, n_lazy_params, min_chunk):
    chunks, owner = overlap_chunks(sizes, n_lazy_params, min_chunk)
    n_lazy, n = sum(sizes[:n_lazy_params]), sum(sizes)
    if n > n_lazy:
        assert chunks[0] == (n_lazy, n)
        lazy = chunks[1:]
    else:
        lazy = chunks
    if n_lazy:
        assert lazy[0][0] == 0 and lazy[-1][1] == n_lazy
        assert all(a[1] == b[0] for a, b in zip(lazy, lazy[1:]))
        assert all(s % 64 == 0 and e > s for s, e in lazy)
        assert all(e - s >= min_chunk for s, e in lazy[:-1])
    off = 0
    for i, k in enumerate(sizes):
        a, b = off, off + k
        off = b
        s, e = chunks[owner[i]]
        if i >= n_lazy_params:
            assert owner[i] == 0
        else:  # the owner chunk updates the parameter's last element
            assert s < b <= e, (i, a, b, chunks[owner[i]])


def test_overlap_chunks_examples():
    assert overlap_chunks([100, 200, 70, 5, 5], 3, 64) == ([(370, 380), (0, 64), (64, 256), (256, 370)],
                                                         [2, 3, 3, 0, 0])
    assert overlap_chunks([10], 0, 8) == ([(0, 10)], [0])


def test_overlap_chunks_random_layouts():
    rng = random.Random(0)
    for _ in range(300):
        nl = rng.randint(1, 12)
        sizes = [rng.choice([64, 4096, rng.randint(1, 5000)]) for _ in range(nl)]
        sizes += [rng.randint(1, 300) for _ in range(rng.randint(0, 4))]
        _check(sizes, nl, rng.choice([1, 64, 1000, 10 ** 6]))


def test_overlap_is_off_on_cpu():
    lin = torch.nn.Linear(8, 8)
    opt = FlatAdam(lin.parameters(), lr=1e-3, overlap_modules=[lin])
    assert opt._overlap is None  # CPU groups: the plain step
    opt.zero_grad()
    lin(torch.randn(2, 8)).sum().backward()
    opt.step()
