"""Data parallelism: pipeline replicas with bucketed gradient
all-reduce (mipipe.parallel.data_parallel), and the reference's documented
interop -- ``Pipe`` wrapped in DDP with ``checkpoint='never'``
(/root/reference/pipe.py:290-293).  CPU, gloo, spawned ranks."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from helpers.engine_cases import _data, _grads, _loss_fn, _port, case_cfg


def _mode_setup(mode):
    """(config, dtype, device) of a case: ``cpu`` fp32, or ``gpu`` -- both ranks on
    cuda:0 in bf16 with HIP-kernel-sized shapes (deferred weight gradients, so
    the buckets go out from inside the flush) over gloo (RCCL refuses two ranks
    on one GPU)."""
    if mode == "gpu":
        return case_cfg("nccl"), torch.bfloat16, torch.device("cuda", 0)
    return case_cfg("gloo"), torch.float32, torch.device("cpu")


def _build(cfg, pp, stage):
    from mipipe.models import TargetSequential, build_lm_blocks, lm_pipeline_units
    from mipipe.models.transformer import merge_units
    from mipipe.parallel import plan_stages

    torch.manual_seed(0)
    full = torch.nn.Sequential(*build_lm_blocks(cfg))
    names = {id(p): n for n, p in full.named_parameters()}
    units = lm_pipeline_units(list(full.children()))
    plan = plan_stages(cfg, pp, 1, split_decoder=False)
    chunk = TargetSequential(*merge_units([units[i] for i in plan.slice(stage)])).train()
    return chunk, names, plan


def _reference(mode, m_total, mb):
    """Single-rank engine over ALL replicas' micro-batches."""
    from mipipe.optim import FlatAdam
    from mipipe.parallel import PipelineEngine

    cfg, dtype, dev = _mode_setup(mode)
    model, names, _ = _build(cfg, 1, 0)
    model = model.to(dev, dtype)
    opt = FlatAdam(model.parameters(), lr=1e-3)
    eng = PipelineEngine(model, chunks=m_total, act_shape=(mb, cfg.seq_len), act_dtype=dtype,
                         loss_fn=_loss_fn(cfg), device=dev)
    inputs, targets = _data(cfg, m_total, mb)
    opt.zero_grad()
    loss = float(eng.step([x.to(dev) for x in inputs], [t.to(dev) for t in targets]).loss)
    opt.fold_grads()
    return loss, _grads(model.parameters(), names), float(opt.grad_sumsq())


def _dp_worker(rank, world, port, pp, dp, m, mb, mode, q, transport="rccl"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mipipe.optim import FlatAdam
        from mipipe.parallel import PipelineEngine
        from mipipe.parallel.data_parallel import DataParallelGrads, make_pp_dp_groups
        from mipipe.parallel.stage import stage_input_shape

        cfg, dtype, dev = _mode_setup(mode)
        if dev.type == "cuda":
            torch.cuda.set_device(dev)
        stage_guess = rank % pp
        _, _, plan0 = _build(cfg, pp, stage_guess)
        recv = max(torch.Size(stage_input_shape(cfg, plan0, stage_guess, mb)).numel(), 1) * torch.empty(
            (), dtype=dtype).element_size()
        groups = make_pp_dp_groups(pp, dp, transport=transport,
                                   ipc_options={"device": dev, "recv_bytes": recv} if transport == "ipc" else None)
        if transport == "ipc" and pp > 1:
            assert type(groups.channels).__name__ == "IpcChannels"
        chunk, names, plan = _build(cfg, pp, groups.stage)
        chunk = chunk.to(dev, dtype)
        opt = FlatAdam(chunk.parameters(), lr=1e-3)
        dpg = DataParallelGrads(opt, groups.dp_group, bucket_mb=0.05)  # several buckets
        eng = PipelineEngine(chunk, chunks=m, act_shape=stage_input_shape(cfg, plan, groups.stage, mb),
                             act_dtype=dtype, loss_fn=_loss_fn(cfg) if groups.stage == pp - 1 else None,
                             device=dev, group=groups.channels, grad_divisor=dp)
        inputs, targets = _data(cfg, m * dp, mb)
        d = groups.replica
        mine_in = [x.to(dev) for x in inputs[d * m:(d + 1) * m]]
        mine_t = [t.to(dev) for t in targets[d * m:(d + 1) * m]]
        opt.zero_grad()
        dpg.begin()
        st = eng.step(mine_in if groups.stage == 0 else None, mine_t)
        early = sum(1 for _, w in dpg._works)  # reductions issued inside the weight-gradient flush
        dpg.finish()
        sq = opt.grad_sumsq()
        dist.all_reduce(sq, group=groups.pipeline_group)
        loss = None if st.loss is None else float(st.loss)
        q.put((rank, groups.replica, loss, _grads(chunk.parameters(), names), float(sq), len(dpg.buckets), early))
        # early issue: buckets whose parameters are all final go out at flush_begin,
        # the rest when their last weight gradient is done -- same sums either way
        params = list(chunk.parameters())
        w = params[-1]
        before = [b.clone() for b in dpg.buckets]
        dpg.begin()
        dpg.flush_begin([w])
        pending = [not x for x in dpg._issued]
        assert sum(pending) == 1 and pending[dpg._bucket_of[id(w)]]
        dpg.wgrad_done(w)
        assert all(dpg._issued)
        dpg.finish()
        for b0, b1 in zip(before, dpg.buckets):
            torch.testing.assert_close(b1, b0 * dp)
    finally:
        dist.destroy_process_group()


def _run_dp(pp, dp, mode, transport="rccl"):
    m, mb = 4, 2
    ref_loss, ref, ref_sq = _reference(mode, m * dp, mb)
    world = pp * dp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_dp_worker, args=(r, world, port, pp, dp, m, mb, mode, q, transport))
             for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    losses = {}
    seen = set()
    gpu = mode == "gpu"
    for rank, replica, loss, grads, sq, nb, early in results:
        assert nb >= 2
        if gpu:
            assert early >= 1  # some buckets went out while weight-gradient GEMMs were still queued
        if loss is not None:
            losses[replica] = loss
        for name, g in grads.items():
            r = torch.from_numpy(ref[name])
            g = torch.from_numpy(g)
            tol = 2e-2 if gpu else 1e-4
            assert (g - r).abs().max().item() <= tol * (r.abs().max().item() + 1e-6), name
            seen.add(name)
        assert abs(sq - ref_sq) / ref_sq < (1e-2 if gpu else 1e-4)
    assert seen == set(ref)
    assert len(losses) == dp
    assert abs(sum(losses.values()) / dp - ref_loss) < (2e-3 if gpu else 1e-5) * abs(ref_loss)


@pytest.mark.parametrize("pp,dp", [(2, 2), (1, 2)])
def test_engine_data_parallel_matches_single_rank(pp, dp):
    """pp x dp ranks (gloo): every gradient, the loss and the global gradient
    norm equal the single-rank engine on the union of the replicas' batches."""
    _run_dp(pp, dp, "cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("pp,dp", [(1, 2), (2, 2)])
def test_engine_data_parallel_share_gpu(pp, dp):
    """The same on one MI355X (all ranks on cuda:0, bf16 HIP kernels, gloo):
    buckets are issued from inside the deferred weight-gradient flush."""
    _run_dp(pp, dp, "gpu")


def test_engine_pp2_dp2_ipc_links_host():
    """pp2 x dp2 with the pipelines' activations on IPC links (host mode)."""
    _run_dp(2, 2, "cpu", transport="ipc")


@pytest.mark.gpu
def test_engine_pp2_dp2_ipc_links_share_gpu():
    """pp2 x dp2, four ranks on cuda:0: stage boundaries over device-memory IPC
    links (DMA copies into the peer's slots), gradients all-reduced over gloo."""
    _run_dp(2, 2, "gpu", transport="ipc")


def _ddp_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import mipipe

        torch.manual_seed(0)
        seq = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 4))
        pipe = mipipe.Pipe(seq, chunks=2, checkpoint="never", return_rref=False)
        ddp = torch.nn.parallel.DistributedDataParallel(pipe)
        g = torch.Generator().manual_seed(3)
        x = torch.randn(8, 8, generator=g)
        mine = x[rank * 4:(rank + 1) * 4]
        ddp(mine).pow(2).mean().backward()
        q.put((rank, [p.grad.numpy().copy() for p in seq.parameters()]))
    finally:
        dist.destroy_process_group()


def test_pipe_wrapped_in_ddp_checkpoint_never():
    """The reference's DDP interop: DDP(Pipe(..., checkpoint='never')) averages
    the replicas' gradients -- equal to one process on the whole batch."""
    torch.manual_seed(0)
    seq = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 4))
    g = torch.Generator().manual_seed(3)
    x = torch.randn(8, 8, generator=g)
    seq(x[:4]).pow(2).mean().backward()
    seq(x[4:]).pow(2).mean().backward()
    ref = [p.grad / 2 for p in seq.parameters()]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_ddp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    results = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, grads in results:
        for a, b in zip(grads, ref):
            torch.testing.assert_close(torch.from_numpy(a), b, rtol=1e-5, atol=1e-6)


def test_listener_unhooked_on_abort_and_finish():
    """begin() hooks the weight-gradient flush; finish() and abort() unhook it
    (a failed step must not leave a stale listener behind)."""
    import importlib

    lin = importlib.import_module("mipipe.ops.linear")

    class _Opt:
        groups = []

        def fold_grads(self):
            pass

    from mipipe.parallel.data_parallel import DataParallelGrads

    dpg = DataParallelGrads.__new__(DataParallelGrads)
    dpg.opt, dpg.group, dpg.world, dpg.average = _Opt(), None, 1, False
    dpg.buckets, dpg._members, dpg._bucket_of = [], [], {}
    dpg._left, dpg._works, dpg._issued, dpg._active = [], [], [], False
    dpg.begin()
    assert dpg in lin._WGRAD_LISTENERS
    dpg.abort()
    assert dpg not in lin._WGRAD_LISTENERS
    dpg.begin()
    dpg.finish()
    assert dpg not in lin._WGRAD_LISTENERS
    with pytest.raises(RuntimeError):
        dpg.finish()
