"""The pipeline on MI355X with the HIP kernels: Pipe and engine end to end.

* ``mipipe.Pipe`` running the bf16 LM blocks (MFMA GEMMs, flash attention,
  fused LN, FlatAdam) against the same blocks as one ``nn.Sequential``
  (SURVEY §4 transparency, on our kernels, not ``nn.Linear``);
* activation-checkpoint recompute replays dropout bit-exactly on our kernels
  (LN / GEMM-epilogue / attention / embedding dropout): ``always`` and
  ``except_last`` gradients are BIT-IDENTICAL to ``never``, for the engine and
  for ``Pipe`` (``/root/reference/README.md:517-537``);
* multi-GPU: ``Pipe`` over ``cuda:0..N-1`` (native peer copies over xGMI) and
  the engine over RCCL (``nccl`` backend, one rank per GPU) against the
  single-rank engine -- skipped on a one-GPU box (``multigpu``).
"""
import copy
import dataclasses

import pytest
import torch

from mipipe import Pipe, ops
from mipipe.models import CONFIGS, build_lm_blocks
from mipipe.optim import FlatAdam
from mipipe.parallel import PipelineEngine

from helpers.engine_cases import ENGINE_CASES, run_dropout_recompute_case, run_engine_case

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def _cfg(dropout=0.0, layers=2):
    base = CONFIGS["tiny"]
    cfg = dataclasses.replace(base, dropout=dropout, num_layers=layers, d_model=256, nhead=4, dim_feedforward=512,
                              vocab=512, seq_len=64)
    return cfg


def _data(cfg, m, mb, seed=7):
    g = torch.Generator().manual_seed(seed)
    tok = torch.randint(0, cfg.vocab, (m, mb, cfg.seq_len + 1), generator=g)
    return [tok[i, :, :-1] for i in range(m)], [tok[i, :, 1:].contiguous() for i in range(m)]


def _loss_fn(cfg):
    return lambda y, t: ops.cross_entropy(y.reshape(-1, cfg.vocab), t.reshape(-1))


def _ngpu():
    return torch.cuda.device_count() if torch.cuda.is_available() else 0


# ------------------------------------------------------------------ Pipe on our kernels
def _pipe_vs_sequential(devices, checkpoint, copy_streams=None, dropout=0.0, defer_wgrad=False):
    cfg = _cfg(dropout=dropout)
    m, mb = 4, 2
    torch.manual_seed(0)
    blocks = build_lm_blocks(cfg, dtype=torch.bfloat16)
    ref_blocks = copy.deepcopy(blocks)
    # reference: one device, the whole mini-batch in one pass
    ref = torch.nn.Sequential(*ref_blocks).to(DEV).train()
    ref_opt = FlatAdam(ref.parameters(), lr=1e-3)
    inputs, targets = _data(cfg, m, mb)
    x = torch.cat(inputs).to(DEV)
    t = torch.cat(targets)
    ref_opt.zero_grad()
    loss_ref = _loss_fn(cfg)(ref(x), t.to(DEV))
    loss_ref.backward()
    ref_opt.fold_grads()

    # pipe: blocks spread evenly over the devices
    n = len(devices)
    per = (len(blocks) + n - 1) // n
    parts = [torch.nn.Sequential(*blocks[i * per:(i + 1) * per]).to(devices[i]) for i in range(n)
             if blocks[i * per:(i + 1) * per]]
    model = torch.nn.Sequential(*parts).train()
    opt = FlatAdam(model.parameters(), lr=1e-3, defer_wgrad=defer_wgrad)
    pipe = Pipe(model, chunks=m, checkpoint=checkpoint, copy_streams=copy_streams)
    try:
        opt.zero_grad()
        out = pipe(x).local_value()
        loss = _loss_fn(cfg)(out, t.to(out.device))
        loss.backward()
        if defer_wgrad:
            import importlib

            _lin = importlib.import_module("mipipe.ops.linear")  # the module, not ops.linear()

            queued = len(_lin._DEFERRED or {})
            assert queued > 0, "no weight gradient was deferred"
        opt.fold_grads()
        if defer_wgrad:
            assert _lin._DEFERRED is None
    finally:
        pipe.close()
    assert abs(float(loss) - float(loss_ref)) < 2e-3 * abs(float(loss_ref))
    for (name, p), q in zip(model.named_parameters(), ref.parameters()):
        g, gr = p.main_grad.float().cpu(), q.main_grad.float().cpu()
        scale = gr.abs().max().item() + 1e-6
        assert (g - gr).abs().max().item() < 2e-2 * scale, name
    return pipe


@pytest.mark.parametrize("checkpoint", ["never", "except_last"])
def test_pipe_deferred_wgrad_one_gpu(checkpoint):
    """FlatAdam(defer_wgrad=True) around a Pipe: the backward queues the weight
    gradients of every micro-batch and fold_grads runs one K-segmented GEMM per
    weight -- same gradients as the unsplit model."""
    _pipe_vs_sequential([DEV], checkpoint, defer_wgrad=True)


@pytest.mark.parametrize("checkpoint", ["never", "except_last", "always"])
def test_pipe_lm_bf16_one_gpu(checkpoint):
    """Pipe on one MI355X (one partition: scatter, worker thread, checkpoint /
    recompute, gather) with the HIP-kernel LM blocks == nn.Sequential."""
    _pipe_vs_sequential([DEV], checkpoint)


@pytest.mark.multigpu
@pytest.mark.parametrize("ngpu", [2, 4])
def test_pipe_deferred_wgrad_multi_gpu(ngpu):
    """Deferred weight gradients queued by several devices' autograd threads are
    each launched on their own device at fold_grads."""
    if _ngpu() < ngpu:
        pytest.skip(f"needs {ngpu} GPUs")
    _pipe_vs_sequential([torch.device("cuda", d) for d in range(ngpu)], "except_last", defer_wgrad=True)


@pytest.mark.multigpu
@pytest.mark.parametrize("ngpu", [2, 4, 8])
@pytest.mark.parametrize("checkpoint,copy_streams", [("never", None), ("except_last", None), ("always", 2),
                                                     ("except_last", 1)])
def test_pipe_lm_bf16_multi_gpu(ngpu, checkpoint, copy_streams):
    """Pipe over cuda:0..N-1 (peer copies over xGMI on copy streams) == nn.Sequential on one GPU."""
    if _ngpu() < ngpu:
        pytest.skip(f"needs {ngpu} GPUs")
    pipe = _pipe_vs_sequential([torch.device("cuda", d) for d in range(ngpu)], checkpoint, copy_streams)
    assert len(pipe.devices) == ngpu


def test_pipe_copy_stream_pool():
    """copy_streams=k: each partition gets k distinct streams shared round-robin."""
    lin = torch.nn.Linear(8, 8).to(DEV)
    pipe = Pipe(torch.nn.Sequential(lin), chunks=5, copy_streams=2)
    (row,) = pipe._copy_streams
    assert len(row) == 5 and len({id(s) for s in row}) == 2 and row[0] is row[2] is row[4]
    pipe.close()
    pipe = Pipe(torch.nn.Sequential(lin), chunks=5)  # default: one copy stream per partition
    assert len({id(s) for s in pipe._copy_streams[0]}) == 1
    pipe.close()
    pipe = Pipe(torch.nn.Sequential(lin), chunks=5, copy_streams=None)  # the reference's: one per micro-batch
    assert len({id(s) for s in pipe._copy_streams[0]}) == 5
    pipe.close()
    with pytest.raises(ValueError):
        Pipe(torch.nn.Sequential(lin), chunks=2, copy_streams=0)


# ------------------------------------------------------------------ bit-exact recompute
def _engine_grads(checkpoint, cfg, m, mb, seed=99):
    torch.manual_seed(0)
    full = torch.nn.Sequential(*build_lm_blocks(cfg)).train().to(DEV, torch.bfloat16)
    opt = FlatAdam(full.parameters(), lr=1e-3)
    eng = PipelineEngine(full, chunks=m, checkpoint=checkpoint, act_shape=(mb, cfg.seq_len),
                         act_dtype=torch.bfloat16, loss_fn=_loss_fn(cfg), device=DEV)
    inputs, targets = _data(cfg, m, mb)
    opt.zero_grad()
    torch.manual_seed(seed)
    st = eng.step([x.to(DEV) for x in inputs], [t.to(DEV) for t in targets])
    opt.fold_grads()
    torch.cuda.synchronize()
    _note_embeddings(full)
    return float(st.loss), {n: p.main_grad.clone() for n, p in full.named_parameters()}


_EMBED_NAMES = set()  # parameter names of token-embedding tables, filled by the grad helpers


def _note_embeddings(model):
    from mipipe.models.lm import Encoder

    for mn, mod in model.named_modules():
        if isinstance(mod, Encoder):
            _EMBED_NAMES.add(f"{mn}.weight" if mn else "weight")


def _assert_same_grad(g, g0, name, mode):
    """Bit-identical gradients -- except the token embedding's: its backward adds rows
    with float atomics, so a token repeated within a micro-batch lands in main_grad in
    an arbitrary order (the last bit may differ between ANY two runs, checkpointed or
    not).  Everything recomputed (dropout masks included) must match exactly."""
    if name in _EMBED_NAMES:
        assert torch.allclose(g, g0, rtol=1e-5, atol=1e-8), (mode, name, (g - g0).abs().max().item())
    else:
        assert torch.equal(g, g0), (mode, name, (g - g0).abs().max().item())


def test_engine_recompute_bit_identical_with_dropout():
    """Engine, dropout 0.2 everywhere (embedding, attention, GEMM epilogues, LN):
    recomputed micro-batches regenerate the same Philox masks, so the gradients
    of 'always' / 'except_last' equal 'never' bit for bit."""
    cfg = _cfg(dropout=0.2)
    m, mb = 4, 2
    loss0, g0 = _engine_grads("never", cfg, m, mb)
    # dropout is live: a different RNG seed gives different gradients
    _, g_other = _engine_grads("never", cfg, m, mb, seed=100)
    assert any(not torch.equal(g0[n], g_other[n]) for n in g0)
    for mode in ("except_last", "always"):
        loss, g = _engine_grads(mode, cfg, m, mb)
        assert loss == loss0, mode
        for n in g0:
            _assert_same_grad(g[n], g0[n], n, mode)


def _pipe_grads(checkpoint, cfg, m, mb, seed=99):
    torch.manual_seed(0)
    blocks = build_lm_blocks(cfg, dtype=torch.bfloat16)
    model = torch.nn.Sequential(torch.nn.Sequential(*blocks).to(DEV)).train()
    opt = FlatAdam(model.parameters(), lr=1e-3)
    pipe = Pipe(model, chunks=m, checkpoint=checkpoint)
    inputs, targets = _data(cfg, m, mb)
    try:
        opt.zero_grad()
        torch.manual_seed(seed)
        out = pipe(torch.cat(inputs).to(DEV)).local_value()
        loss = _loss_fn(cfg)(out, torch.cat(targets).to(DEV))
        loss.backward()
        opt.fold_grads()
        torch.cuda.synchronize()
    finally:
        pipe.close()
    _note_embeddings(model)
    return float(loss), {n: p.main_grad.clone() for n, p in model.named_parameters()}


def test_pipe_recompute_bit_identical_with_dropout():
    """Same property through the single-process Pipe's Checkpoint/Recompute."""
    cfg = _cfg(dropout=0.2)
    m, mb = 4, 2
    loss0, g0 = _pipe_grads("never", cfg, m, mb)
    for mode in ("except_last", "always"):
        loss, g = _pipe_grads(mode, cfg, m, mb)
        assert loss == loss0, mode
        for n in g0:
            _assert_same_grad(g[n], g0[n], n, mode)


# ------------------------------------------------------------------ stream-race checker
def test_check_pipe_and_engine_on_gpu():
    """mipipe.debug: the scheduled step (copy / compute streams overlapping) equals
    the serialised one on our bf16 kernels with dropout 0.2 -- for the Pipe and
    the engine."""
    from mipipe.debug import check_engine, check_pipe

    cfg = _cfg(dropout=0.2)
    m, mb = 4, 2
    inputs, targets = _data(cfg, m, mb)
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Sequential(*build_lm_blocks(cfg, dtype=torch.bfloat16)).to(DEV)).train()
    FlatAdam(model.parameters(), lr=1e-3)
    pipe = Pipe(model, chunks=m, checkpoint="except_last")
    t = torch.cat(targets).to(DEV)
    try:
        torch.manual_seed(3)
        rep = check_pipe(pipe, torch.cat(inputs).to(DEV), loss_fn=lambda y: _loss_fn(cfg)(y, t))
    finally:
        pipe.close()
    assert rep.ok, rep.worst()
    assert len(rep.max_rel) > 10

    torch.manual_seed(0)
    full = torch.nn.Sequential(*build_lm_blocks(cfg)).train().to(DEV, torch.bfloat16)
    FlatAdam(full.parameters(), lr=1e-3)
    eng = PipelineEngine(full, chunks=m, checkpoint="always", act_shape=(mb, cfg.seq_len), act_dtype=torch.bfloat16,
                         loss_fn=_loss_fn(cfg), device=DEV)
    torch.manual_seed(4)
    rep = check_engine(eng, [x.to(DEV) for x in inputs], [y.to(DEV) for y in targets])
    assert rep.ok, rep.worst()
    assert "loss" in rep.max_rel and not eng.sync_debug


# ------------------------------------------------------------------ engine over RCCL
@pytest.mark.multigpu
@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("checkpoint,virtual,split,skips", ENGINE_CASES)
def test_engine_nccl_matches_single_rank(world, checkpoint, virtual, split, skips):
    """One rank per GPU over RCCL (isend/irecv on per-direction communicators)
    vs the single-rank engine; the same cases run over gloo on CPU in
    tests/test_engine.py::test_engine_cases_gloo_emulation."""
    if _ngpu() < world:
        pytest.skip(f"needs {world} GPUs")
    run_engine_case("nccl", world, checkpoint, virtual, split, skips)


# ------------------------------------------------------------------ engine over IPC links, ranks sharing cuda:0
@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("checkpoint,virtual,split,skips", ENGINE_CASES)
def test_engine_ipc_links_share_gpu(world, checkpoint, virtual, split, skips):
    """2 / 4 pipeline ranks on ONE MI355X, transport='ipc': every activation and
    gradient moves through device memory -- the sender's DMA copy into the
    receiver's exported slot ring, which the receiver reads in place; both
    sides order each other on the GPU through flag words (stream write /
    wait-value), no host wait, no host staging, no RCCL.  Against the
    single-rank engine (bf16 kernels)."""
    run_engine_case("ipc_gpu", world, checkpoint, virtual, split, skips)


@pytest.mark.parametrize("world,virtual", [(2, 1), (4, 2)])
def test_engine_ipc_links_dropout_recompute_bit_identical(world, virtual):
    """Dropout 0.2 on every rank (embedding, attention, GEMM epilogues): the
    multi-rank 'except_last' / 'always' gradients are BIT-identical to 'never'
    on every rank -- recompute replays each rank's own Philox stream."""
    run_dropout_recompute_case("ipc_gpu", world, virtual)


@pytest.mark.parametrize("world,virtual", [(2, 1), (4, 2)])
def test_engine_ipc_links_slot_reuse_over_steps(world, virtual):
    """Three steps: every slot, its flag words and its sequence counters are
    reused step after step (a slot read in place is released at the end of
    its step and refilled in the next) -- the last step still equals the
    single-rank engine."""
    run_engine_case("ipc_gpu", world, "except_last", virtual, virtual > 1, False, steps=3)



# ------------------------------------------------------------------ transport 'auto' (the bench's default at PP > 1)
@pytest.mark.parametrize("world,virtual", [(2, 1), (4, 2)])
def test_engine_auto_transport_self_tested_ipc(world, virtual):
    """transport='auto': the IPC links pass their self-test (every word of a
    whole-slot message per link and direction checked) and carry the step;
    ranks sharing one GPU copy on the producer's stream ('ipc-inline')."""
    run_engine_case("auto_gpu", world, "except_last", virtual, virtual > 1, False)


@pytest.mark.parametrize("world,virtual", [(2, 1), (4, 2)])
def test_engine_auto_transport_sdma_engine(world, virtual):
    """The cross-GPU engine of transport='auto' -- copies on each link's own copy
    stream (SDMA), ordered after the producer by an event and before the
    consumer by the flag wait -- self-tested and then carrying two steps, on
    ranks sharing one GPU (the only way to run it on a one-GPU box)."""
    run_engine_case("auto_sdma_gpu", world, "except_last", virtual, virtual > 1, False, steps=2)
