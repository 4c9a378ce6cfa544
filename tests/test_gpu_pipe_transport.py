"""The single-process ``Pipe``'s stage transport on ONE MI355X.

Several partitions on ``cuda:0`` (``Pipe(balance=...)``): every stage boundary
runs the reference's machinery for real -- ``Copy`` on the per-(partition,
micro-batch) copy streams (with ``copy_same_device=True`` a native
device-to-device copy fenced by pooled events, i.e. ``peer_copy``),
``Wait`` events between copy and compute streams, ``record_stream`` on the
streams that consume, portals for cross-partition skips, and recompute on the
stage streams (``/root/reference/pipeline.py:119-142,186-192,253-254``;
``README.md:193-237,332-369``).  With ``stage_streams="dedicated"`` every later
partition on the GPU computes on a stream of its own, so stage j's micro-batch i
really overlaps stage j-1's micro-batch i+1 (sleep-kernel test); the default,
``"shared"``, computes every partition of a GPU on its current stream, as the
reference does (one stream per device).
"""
import copy
import dataclasses
import time

import pytest
import torch

from mipipe import Pipe, ops
from mipipe.models import CONFIGS, build_lm_blocks
from mipipe.models.long_skip import AddSkip, StashSkip
from mipipe.optim import FlatAdam
from mipipe.skip import Namespace

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def _cfg(dropout=0.0):
    return dataclasses.replace(CONFIGS["tiny"], dropout=dropout, num_layers=2, d_model=256, nhead=4,
                               dim_feedforward=512, vocab=512, seq_len=64)


def _data(cfg, m, mb, seed=7):
    g = torch.Generator().manual_seed(seed)
    tok = torch.randint(0, cfg.vocab, (m * mb, cfg.seq_len + 1), generator=g)
    return tok[:, :-1].to(DEV), tok[:, 1:].contiguous().to(DEV)


def _loss(cfg, y, t):
    return ops.cross_entropy(y.reshape(-1, cfg.vocab), t.reshape(-1))


_BALANCE = {2: [3, 3], 4: [2, 1, 1, 2]}  # 6 LM blocks: encoder, 2 x (attention, FFN), decoder


def _pipe_step(nparts, checkpoint, dropout, copy_same_device, seed=99, engine=None, stage_streams="dedicated"):
    cfg = _cfg(dropout)
    torch.manual_seed(0)
    model = torch.nn.Sequential(*build_lm_blocks(cfg, dtype=torch.bfloat16)).to(DEV).train()
    opt = FlatAdam(model.parameters(), lr=1e-3)
    pipe = Pipe(model, chunks=4, checkpoint=checkpoint, balance=_BALANCE[nparts],
                copy_same_device=copy_same_device, copy_engine=engine, return_rref=False, stage_streams=stage_streams)
    x, t = _data(cfg, 4, 2)
    try:
        assert len(pipe.partitions) == nparts and all(d == DEV for d in pipe.devices)
        # dedicated: later partitions of the GPU compute on streams of their own;
        # shared: all on the device's current stream (the reference's one per device)
        streams = pipe.pipeline.compute_streams()
        assert len({s.cuda_stream for s in streams}) == (nparts if stage_streams == "dedicated" else 1)
        opt.zero_grad()
        torch.manual_seed(seed)
        out = pipe(x)
        loss = _loss(cfg, out, t)
        loss.backward()
        opt.fold_grads()
        torch.cuda.synchronize()
    finally:
        pipe.close()
    return float(loss), {n: p.main_grad.clone() for n, p in model.named_parameters()}


@pytest.mark.parametrize("nparts", [2, 4])
@pytest.mark.parametrize("copy_same_device", [True, False])
def test_pipe_partitions_one_gpu_match_sequential(nparts, copy_same_device):
    """2 / 4 partitions on cuda:0, bf16 HIP-kernel LM blocks, no dropout:
    output and gradients == the same blocks as one nn.Sequential."""
    cfg = _cfg(0.0)
    torch.manual_seed(0)
    blocks = build_lm_blocks(cfg, dtype=torch.bfloat16)
    ref = torch.nn.Sequential(*copy.deepcopy(blocks)).to(DEV).train()
    ref_opt = FlatAdam(ref.parameters(), lr=1e-3)
    x, t = _data(cfg, 4, 2)
    ref_opt.zero_grad()
    loss_ref = _loss(cfg, ref(x), t)
    loss_ref.backward()
    ref_opt.fold_grads()
    loss, grads = _pipe_step(nparts, "never", 0.0, copy_same_device)
    assert abs(loss - float(loss_ref)) < 2e-3 * abs(float(loss_ref))
    for n, q in ref.named_parameters():
        g, gr = grads[n].float(), q.main_grad.float()
        assert (g - gr).abs().max().item() < 2e-2 * (gr.abs().max().item() + 1e-6), n


@pytest.mark.parametrize("nparts", [2, 4])
def test_pipe_partitions_one_gpu_checkpoint_modes_bit_identical(nparts):
    """Dropout 0.2 everywhere, stage boundaries as native D2D copies: 'always'
    and 'except_last' (recompute on the stage streams) give gradients BIT-
    IDENTICAL to 'never'; handing tensors over in place gives the same bits as
    copying them (SDMA and blit engines alike)."""
    loss0, g0 = _pipe_step(nparts, "never", 0.2, True)
    _, g_other = _pipe_step(nparts, "never", 0.2, True, seed=100)
    assert any(not torch.equal(g0[n], g_other[n]) for n in g0)  # dropout is live
    runs = [("except_last", True, None), ("always", True, None), ("never", False, None), ("always", True, "blit")]
    for mode, copy_sd, engine in runs:
        loss, g = _pipe_step(nparts, mode, 0.2, copy_sd, engine=engine)
        assert loss == loss0, (mode, copy_sd, engine)
        for n in g0:
            assert torch.equal(g[n], g0[n]), (mode, copy_sd, engine, n, (g[n] - g0[n]).abs().max().item())


def test_check_pipe_four_partitions_one_gpu():
    """The stream-race checker on a Pipe that HAS copy streams to race: four
    partitions on cuda:0, native D2D boundaries, dropout 0.2 -- scheduled step
    (copy / stage streams overlapping) == serialised step."""
    from mipipe.debug import check_pipe

    cfg = _cfg(0.2)
    torch.manual_seed(0)
    model = torch.nn.Sequential(*build_lm_blocks(cfg, dtype=torch.bfloat16)).to(DEV).train()
    FlatAdam(model.parameters(), lr=1e-3)
    pipe = Pipe(model, chunks=4, checkpoint="except_last", balance=_BALANCE[4], copy_same_device=True,
                stage_streams="dedicated")
    x, t = _data(cfg, 4, 2)
    try:
        assert len(pipe.partitions) == 4
        torch.manual_seed(3)
        rep = check_pipe(pipe, x, loss_fn=lambda y: _loss(cfg, y, t))
    finally:
        pipe.close()
    assert rep.ok, rep.worst()
    assert len(rep.max_rel) > 10


def _skip_model(cfg, dtype=torch.bfloat16):
    """[enc, Stash, A0, F0, A1, F1, Add, dec]: layer-0 input added to layer-1 output."""
    blocks = build_lm_blocks(cfg, dtype=dtype)
    ns = Namespace(label="enc->L1")
    mods = [blocks[0], StashSkip().isolate(ns)] + blocks[1:5] + [AddSkip().isolate(ns), blocks[5]]
    return torch.nn.Sequential(*mods)


@pytest.mark.parametrize("checkpoint", ["never", "except_last", "always"])
def test_skippable_portals_across_partitions_one_gpu(checkpoint):
    """@skippable stash in partition 0, pop in partition 3 on cuda:0: the portal
    copies the skip once (stash stage -> pop stage, native D2D on the copy
    streams) and its gradient comes back; == the model run unpartitioned."""
    cfg = _cfg(0.0)
    torch.manual_seed(0)
    model = _skip_model(cfg).to(DEV).train()
    ref = copy.deepcopy(model)
    opt, ref_opt = FlatAdam(model.parameters(), lr=1e-3), FlatAdam(ref.parameters(), lr=1e-3)
    x, t = _data(cfg, 4, 2)
    ref_opt.zero_grad()
    loss_ref = _loss(cfg, ref(x), t)
    loss_ref.backward()
    ref_opt.fold_grads()
    pipe = Pipe(model, chunks=4, checkpoint=checkpoint, balance=[2, 2, 2, 2], copy_same_device=True,
                return_rref=False, stage_streams="dedicated")
    try:
        assert len(pipe.partitions) == 4
        layout = pipe._skip_layout
        assert list(layout.copy_policy(3)) and not list(layout.copy_policy(1))  # stash in 0, pop in 3
        opt.zero_grad()
        loss = _loss(cfg, pipe(x), t)
        loss.backward()
        opt.fold_grads()
        torch.cuda.synchronize()
    finally:
        pipe.close()
    assert abs(float(loss) - float(loss_ref)) < 2e-3 * abs(float(loss_ref))
    for (n, p), q in zip(model.named_parameters(), ref.parameters()):
        g, gr = p.main_grad.float(), q.main_grad.float()
        assert (g - gr).abs().max().item() < 2e-2 * (gr.abs().max().item() + 1e-6), n


class _Sleep(torch.autograd.Function):
    """Forward and backward each enqueue a busy-wait kernel on the current stream."""

    @staticmethod
    def forward(ctx, x, us):
        from mipipe import _native_loader

        ctx.us = us
        _native_loader.kernels().gpu_sleep(us)
        return x * 1.0

    @staticmethod
    def backward(ctx, g):
        from mipipe import _native_loader

        _native_loader.kernels().gpu_sleep(ctx.us)
        return g * 1.0, None


class _SleepLayer(torch.nn.Module):
    def __init__(self, us):
        super().__init__()
        self.us = us
        self.w = torch.nn.Parameter(torch.ones(1))  # places the layer on its device

    def forward(self, x):
        return _Sleep.apply(x * self.w, self.us)


def _timed(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return time.perf_counter() - t0


def test_stage_overlap_on_one_gpu():
    """Two partitions on cuda:0, 4 micro-batches, every cell a 20 ms sleep:
    serial = 8 cells = 160 ms; the GPipe wavefront needs 5 ticks = 100 ms,
    which is only reachable if partition 1's micro-batch i runs WHILE
    partition 0's micro-batch i+1 does (stage streams + copy streams).  The
    backward (autograd, phony ordering) must overlap the same way."""
    us = 20000
    model = torch.nn.Sequential(_SleepLayer(us), _SleepLayer(us)).to(DEV)
    pipe = Pipe(model, chunks=4, checkpoint="never", balance=[1, 1], copy_same_device=True, return_rref=False,
                stage_streams="dedicated")
    x = torch.randn(8, 1024, device=DEV, requires_grad=True)
    out = {}
    try:
        pipe(x)  # warm-up (streams, kernels)
        torch.cuda.synchronize()
        fwd = _timed(lambda: out.__setitem__("y", pipe(x)))
        bwd = _timed(lambda: out["y"].sum().backward())
    finally:
        pipe.close()
    serial = 8 * us * 1e-6
    assert fwd < 0.8 * serial, f"forward {fwd * 1e3:.1f} ms: stages did not overlap (serial {serial * 1e3:.0f} ms)"
    assert fwd > 0.95 * 5 * us * 1e-6, fwd  # sanity: 5 ticks is the floor
    assert bwd < 0.85 * serial, f"backward {bwd * 1e3:.1f} ms: stages did not overlap"
    assert torch.allclose(x.grad, torch.ones_like(x))


def test_shared_stage_streams_match_sequential():
    """The default (stage_streams='shared', the reference's one stream per
    device): the partitions of cuda:0 all compute on its current stream, the
    boundaries still copy on the copy streams -- same loss and gradients as
    the plain model."""
    cfg = _cfg(0.0)
    torch.manual_seed(0)
    blocks = build_lm_blocks(cfg, dtype=torch.bfloat16)
    ref = torch.nn.Sequential(*copy.deepcopy(blocks)).to(DEV).train()
    ref_opt = FlatAdam(ref.parameters(), lr=1e-3)
    x, t = _data(cfg, 4, 2)
    ref_opt.zero_grad()
    loss_ref = _loss(cfg, ref(x), t)
    loss_ref.backward()
    ref_opt.fold_grads()
    loss, grads = _pipe_step(4, "never", 0.0, True, stage_streams="shared")
    assert abs(loss - float(loss_ref)) < 2e-3 * abs(float(loss_ref))
    for n, q in ref.named_parameters():
        g, gr = grads[n].float(), q.main_grad.float()
        assert (g - gr).abs().max().item() < 2e-2 * (gr.abs().max().item() + 1e-6), n
