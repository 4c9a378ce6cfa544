"""Cross-stage @skippable skips through the multi-process engine (BASELINE config #5).

The LM with U-Net-style long residuals (``mipipe.models.long_skip``) split over
2-4 gloo ranks (and looping chunks, so some skips stay on one rank): loss and
every gradient must equal the unpartitioned model's."""
import dataclasses
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mipipe import ops
from mipipe.models import CONFIGS, TargetSequential, build_lm_blocks, lm_pipeline_units
from mipipe.models.long_skip import insert_long_skips, unet_pairs
from mipipe.models.transformer import merge_units
from mipipe.parallel import PipelineEngine, plan_stages
from mipipe.parallel.skips import routes_from_declarations
from mipipe.parallel.stage import stage_input_shape

PAIRS = [(0, 3), (1, 2)]


def _cfg():
    return dataclasses.replace(CONFIGS["tiny"], dropout=0.0, num_layers=4, d_model=32, nhead=4,
                               dim_feedforward=64, vocab=50, seq_len=8)


def _loss_fn(cfg):
    return lambda y, t: ops.cross_entropy(y.reshape(-1, cfg.vocab), t.reshape(-1))


def _data(cfg, m, mb):
    g = torch.Generator().manual_seed(7)
    tok = torch.randint(0, cfg.vocab, (m, mb, cfg.seq_len + 1), generator=g)
    return [tok[i, :, :-1] for i in range(m)], [tok[i, :, 1:].contiguous() for i in range(m)]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _reference(cfg, m, mb):
    torch.manual_seed(0)
    full = torch.nn.Sequential(*build_lm_blocks(cfg))
    model = TargetSequential(*merge_units(insert_long_skips(lm_pipeline_units(list(full.children())), PAIRS))).train()
    inputs, targets = _data(cfg, m, mb)
    total = 0.0
    for x, t in zip(inputs, targets):
        loss = _loss_fn(cfg)(model(x), t) / m
        loss.backward()
        total += float(loss.detach()) * m
    return {n: p.grad.clone() for n, p in full.named_parameters()}, total / m


def test_long_skips_change_the_model():
    cfg = _cfg()
    torch.manual_seed(0)
    full = torch.nn.Sequential(*build_lm_blocks(cfg)).eval()
    plain = TargetSequential(*merge_units(lm_pipeline_units(list(full.children())))).eval()
    skip = TargetSequential(*merge_units(insert_long_skips(lm_pipeline_units(list(full.children())), PAIRS))).eval()
    x, _ = _data(cfg, 1, 2)
    assert not torch.allclose(plain(x[0]), skip(x[0]))
    assert unet_pairs(12) == [(0, 11), (1, 10), (2, 9), (3, 8), (4, 7), (5, 6)]


def test_routes_from_declarations():
    decl = [(0, 3, "stash", "a:skip"), (2, 1, "pop", "a:skip"), (1, 0, "stash", "b:skip"), (1, 4, "pop", "b:skip")]
    routes = routes_from_declarations(decl)
    assert set(routes) == {"a:skip"}  # b is popped in the stage that stashed it
    assert (routes["a:skip"].stash_vstage, routes["a:skip"].pop_vstage) == (0, 2)
    with pytest.raises(TypeError, match="not stashed"):
        routes_from_declarations([(1, 0, "pop", "x")])
    with pytest.raises(TypeError, match="never popped"):
        routes_from_declarations([(0, 0, "stash", "x")])


def _worker(rank, world, port, checkpoint, virtual, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cfg = _cfg()
        m, mb = 4, 2
        torch.manual_seed(0)
        full = torch.nn.Sequential(*build_lm_blocks(cfg))
        names = {id(p): n for n, p in full.named_parameters()}
        units = lm_pipeline_units(list(full.children()))
        plan = plan_stages(cfg, world, virtual)
        chunks = []
        for s in plan.vstages(rank):
            sl = plan.slice(s)
            chunks.append(TargetSequential(*merge_units(insert_long_skips([units[i] for i in sl], PAIRS,
                                                                          start=sl.start))).train())
        eng = PipelineEngine(chunks, chunks=m, checkpoint=checkpoint,
                             act_shape=[stage_input_shape(cfg, plan, s, mb) for s in plan.vstages(rank)],
                             act_dtype=torch.float32, loss_fn=_loss_fn(cfg) if rank == world - 1 else None,
                             device=torch.device("cpu"),
                             # a stage may start inside a layer (packed input): name the skips' shape
                             skip_shapes={"skip": ((mb, cfg.seq_len, cfg.d_model), torch.float32)})
        inputs, targets = _data(cfg, m, mb)
        st = eng.step(inputs if rank == 0 else None, targets)
        grads = {names[id(p)]: p.grad.numpy().copy() for c in chunks for p in c.parameters() if p.grad is not None}
        cross = sorted((r.stash_vstage, r.pop_vstage) for r in eng.skip_routes.values())
        q.put((rank, None if st.loss is None else float(st.loss), grads, cross))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,virtual,checkpoint", [(2, 1, "never"), (2, 1, "always"), (2, 2, "except_last"),
                                                      (3, 1, "except_last"), (4, 1, "never")])
def test_engine_cross_stage_skips_gloo(world, virtual, checkpoint):
    cfg = _cfg()
    m, mb = 4, 2
    ref, ref_loss = _reference(cfg, m, mb)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, checkpoint, virtual, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    seen = set()
    crosses = set()
    for rank, loss, grads, cross in results:
        crosses.update(cross)
        if loss is not None:
            assert abs(loss - ref_loss) < 1e-5
        for name, g in grads.items():
            assert torch.allclose(torch.from_numpy(g), ref[name], atol=1e-5), name
            seen.add(name)
    assert seen == set(ref)
    assert crosses, "the split must put at least one skip across stages"


def _gpu_cfg():
    return dataclasses.replace(CONFIGS["tiny"], dropout=0.0, num_layers=4, d_model=256, nhead=4,
                               dim_feedforward=512, vocab=512, seq_len=64)


def _gpu_worker(rank, world, port, q):
    from mipipe.optim import FlatAdam

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cfg, dev, m, mb = _gpu_cfg(), torch.device("cuda", 0), 4, 2
        torch.manual_seed(0)
        full = torch.nn.Sequential(*build_lm_blocks(cfg))
        names = {id(p): n for n, p in full.named_parameters()}
        units = lm_pipeline_units(list(full.children()))
        plan = plan_stages(cfg, world, 1)
        sl = plan.slice(rank)
        stage = TargetSequential(*merge_units(insert_long_skips([units[i] for i in sl], PAIRS, start=sl.start)))
        stage = stage.train().to(dev, torch.bfloat16)
        opt = FlatAdam(stage.parameters(), lr=1e-3)
        eng = PipelineEngine(stage, chunks=m, checkpoint="except_last",
                             act_shape=stage_input_shape(cfg, plan, rank, mb), act_dtype=torch.bfloat16,
                             loss_fn=_loss_fn(cfg) if rank == world - 1 else None, device=dev,
                             skip_shapes={"skip": ((mb, cfg.seq_len, cfg.d_model), torch.bfloat16)})
        inputs, targets = _data(cfg, m, mb)
        opt.zero_grad()
        st = eng.step([x.to(dev) for x in inputs] if rank == 0 else None, [t.to(dev) for t in targets])
        opt.fold_grads()
        grads = {names[id(p)]: p.main_grad.float().cpu().numpy().copy() for p in stage.parameters()}
        q.put((rank, None if st.loss is None else float(st.loss), grads, len(eng.skip_routes)))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_engine_skips_two_ranks_share_gpu():
    """The long-residual LM on the HIP kernels, split over two ranks on one
    MI355X (host-staged boundaries and skips) vs the one-rank engine."""
    from mipipe.optim import FlatAdam

    cfg, dev, m, mb = _gpu_cfg(), torch.device("cuda", 0), 4, 2
    torch.manual_seed(0)
    full = torch.nn.Sequential(*build_lm_blocks(cfg))
    model = TargetSequential(*merge_units(insert_long_skips(lm_pipeline_units(list(full.children())), PAIRS)))
    model = model.train().to(dev, torch.bfloat16)
    names = {id(p): n for n, p in full.named_parameters()}
    opt = FlatAdam(model.parameters(), lr=1e-3)
    eng = PipelineEngine(model, chunks=m, checkpoint="never", act_shape=(mb, cfg.seq_len), act_dtype=torch.bfloat16,
                         loss_fn=_loss_fn(cfg), device=dev)
    inputs, targets = _data(cfg, m, mb)
    opt.zero_grad()
    ref_loss = float(eng.step([x.to(dev) for x in inputs], [t.to(dev) for t in targets]).loss)
    opt.fold_grads()
    ref = {names[id(p)]: p.main_grad.float().cpu() for p in model.parameters()}

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_gpu_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    results = [q.get(timeout=300) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    seen = set()
    assert sum(r[3] for r in results) > 0, "no skip crossed the two stages"
    for rank, loss, grads, _ in results:
        if loss is not None:
            assert abs(loss - ref_loss) < 2e-3 * abs(ref_loss)
        for name, g in grads.items():
            g = torch.from_numpy(g)
            scale = ref[name].abs().max().item() + 1e-6
            assert (g - ref[name]).abs().max().item() < 2e-2 * scale, name
            seen.add(name)
    assert seen == set(ref)
