"""FlatAdam(overlap_modules=...): the update on a side stream, chunk by chunk in
forward order, with the next step's forward waiting per module.  The result
must be bit-identical to the serial step (the same elementwise kernel over the
same elements), over several steps, with and without recompute, with dropout."""
import dataclasses

import pytest
import torch

from mipipe import ops
from mipipe.models import CONFIGS, TargetSequential, build_lm_blocks, lm_pipeline_units
from mipipe.models.transformer import merge_units
from mipipe.optim import FlatAdam, _Overlap
from mipipe.parallel import PipelineEngine

pytestmark = pytest.mark.gpu


def _cfg():
    return dataclasses.replace(CONFIGS["tiny"], dropout=0.1, num_layers=4, d_model=256, nhead=4,
                               dim_feedforward=512, vocab=512, seq_len=64)


def _train(overlap: bool, checkpoint: str, steps: int = 4):
    cfg = _cfg()
    dev = torch.device("cuda", 0)
    m, mb = 4, 2
    torch.manual_seed(0)
    units = lm_pipeline_units(list(torch.nn.Sequential(*build_lm_blocks(cfg)).children()))
    model = TargetSequential(*merge_units(units)).train().to(dev, torch.bfloat16)
    opt = FlatAdam(model.parameters(), lr=1e-3, max_grad_norm=0.5, overlap_modules=[model] if overlap else None)
    assert (opt._overlap is not None) == overlap
    eng = PipelineEngine(model, chunks=m, checkpoint=checkpoint, act_shape=(mb, cfg.seq_len),
                         act_dtype=torch.bfloat16, device=dev,
                         loss_fn=lambda y, t: ops.cross_entropy(y.reshape(-1, cfg.vocab), t.reshape(-1)))
    g = torch.Generator().manual_seed(7)
    tok = torch.randint(0, cfg.vocab, (m, mb, cfg.seq_len + 1), generator=g)
    inputs = [tok[i, :, :-1].to(dev) for i in range(m)]
    targets = [tok[i, :, 1:].contiguous().to(dev) for i in range(m)]
    losses = []
    for s in range(steps):
        torch.manual_seed(100 + s)
        opt.zero_grad()
        st = eng.step(inputs, targets)
        opt.step(opt.grad_sumsq())
        losses.append(st.loss.detach().clone())
    torch.cuda.synchronize()
    state = opt.state_dict()
    return ([float(x) for x in losses], [p.detach().clone() for p in model.parameters()],
            [t.clone() for grp in state["groups"] for t in grp.values()], opt, model)


def _embedding_range(opt, model):
    """Flat-buffer range of the embedding table: its gradient is summed with float atomics (embed_bwd_kernel),
    so its last bits depend on the order the atomics land in -- between two SERIAL runs too."""
    emb = next(m for m in model.modules() if type(m).__name__ == "Encoder")
    off = 0
    for p in opt.groups[0].params:
        if p is emb.weight:
            return off, off + p.numel()
        off += p.numel()
    raise AssertionError("no embedding parameter")


def _same(a, b, rng):
    lo, hi = rng
    ok = torch.equal(a[:lo], b[:lo]) and torch.equal(a[hi:], b[hi:])
    return ok and torch.allclose(a[lo:hi], b[lo:hi], rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("checkpoint", ["never", "except_last"])
def test_overlapped_step_bit_identical(monkeypatch, checkpoint):
    """Bit-identical everywhere but the embedding table (atomics), which matches to rounding."""
    monkeypatch.setattr(_Overlap, "MIN_CHUNK", 4096)  # many chunks at this size
    l0, p0, s0, *_ = _train(False, checkpoint)
    l1, p1, s1, opt, model = _train(True, checkpoint)
    assert len(opt._overlap.chunks[0]) > 8, opt._overlap.chunks
    assert l0 == l1
    for a, b in zip(p0, p1):
        assert torch.equal(a, b)
    rng = _embedding_range(opt, model)
    for a, b in zip(s0, s1):  # master, exp_avg, exp_avg_sq: flat buffers
        assert _same(a, b, rng)


def test_overlap_chunks_cover_the_buffer_in_forward_order(monkeypatch):
    monkeypatch.setattr(_Overlap, "MIN_CHUNK", 4096)
    *_, opt, model = _train(True, "never", steps=1)
    g = opt.groups[0]
    chunks = opt._overlap.chunks[0]
    assert chunks[0] == (g.n_lazy, g.numel)  # non-GEMM parameters (embedding, norms, biases) first
    lazy = chunks[1:]
    assert lazy[0][0] == 0 and lazy[-1][1] == g.n_lazy
    assert all(a[1] == b[0] for a, b in zip(lazy, lazy[1:]))
    assert all(a % 64 == 0 for a, _ in chunks)
    # every hooked module waits for the chunk that updates the last element of each of its parameters
    off = {}
    o = 0
    for p in g.params:
        off[id(p)] = (o, o + p.numel())
        o += p.numel()
    for mod in model.modules():
        if id(mod) not in opt._overlap.need:
            continue
        need = opt._overlap.need[id(mod)][0]
        for p in mod.parameters(recurse=mod is not model):  # a block's hook covers its whole subtree
            a, b = off[id(p)]
            if a >= g.n_lazy:
                assert need >= 0
            else:
                ci = next(i for i, (s, e) in enumerate(chunks) if s < b <= e and i > 0)
                assert need >= ci
