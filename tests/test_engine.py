"""Multi-process pipeline engine (mipipe.parallel) on CPU with gloo, world_size 2.

The distributed path the benchmark runs over RCCL is exercised here rank-for-
rank over gloo: each rank owns a slice of the same LM; losses and gradients must
match the unpartitioned model (dropout 0 for exact comparison)."""
import copy
import dataclasses
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mipipe import ops
from mipipe.models import CONFIGS, TargetSequential, build_lm_blocks, lm_pipeline_units
from mipipe.optim import FlatAdam
from mipipe.parallel import PipelineEngine, plan_stages, schedule_actions
from mipipe.models.transformer import merge_units, pipeline_units
from mipipe.parallel.stage import block_costs, stage_input_shape

from helpers.engine_cases import ENGINE_CASES, run_engine_case


def _pairs(acts):
    return [(k, i) for k, c, i in acts]


def test_schedule_actions():
    assert _pairs(schedule_actions("gpipe", 3, 2, 0)) == [("F", 0), ("F", 1), ("F", 2), ("B", 2), ("B", 1), ("B", 0)]
    a = _pairs(schedule_actions("1f1b", 4, 2, 0))
    assert a == [("F", 0), ("F", 1), ("B", 0), ("F", 2), ("B", 1), ("F", 3), ("B", 2), ("B", 3)]
    last = _pairs(schedule_actions("1f1b", 4, 2, 1))
    assert last == [("F", 0), ("B", 0), ("F", 1), ("B", 1), ("F", 2), ("B", 2), ("F", 3), ("B", 3)]
    for kind in ("gpipe", "1f1b"):
        for j in range(3):
            acts = _pairs(schedule_actions(kind, 5, 3, j))
            assert sorted(acts) == sorted([("F", i) for i in range(5)] + [("B", i) for i in range(5)])
    # looping: breadth-first over chunks, backward in exact reverse
    lp = schedule_actions("gpipe", 2, 2, 1, virtual=2)
    assert lp == [("F", 0, 0), ("F", 0, 1), ("F", 1, 0), ("F", 1, 1),
                  ("B", 1, 1), ("B", 1, 0), ("B", 0, 1), ("B", 0, 0)]
    with pytest.raises(ValueError):
        schedule_actions("1f1b", 2, 2, 0, virtual=2)


def test_simulated_bubble_matches_gpipe_formula():
    from mipipe.parallel.stage import simulate_step

    for n, m in ((2, 4), (4, 16), (8, 32)):
        t, busy = simulate_step([1.0] * n, n, 1, m)
        bubble = 1 - sum(busy) / len(busy) / t
        assert abs(bubble - (n - 1) / (m + n - 1)) < 1e-9
        # looping with v chunks: fill/drain shrink by v
        v = 2
        t, busy = simulate_step([0.5] * (n * v), n, v, m)
        bubble = 1 - sum(busy) / len(busy) / t
        assert abs(bubble - (n - 1) / (v * m + n - 1)) < 1e-9


def test_looping_plans():
    from mipipe.parallel.stage import choose_virtual

    cfg = CONFIGS["enc12_d4096"]
    p = plan_stages(cfg, 4, 2)
    assert len(p.balance) == 8 and p.virtual == 2 and p.ranks == 4
    assert p.vstages(1) == [1, 5]
    assert sum(p.balance) == len(block_costs(cfg))
    v, plan = choose_virtual(cfg, 2, 8, micro_batch=64)
    assert v >= 2 and plan.virtual == v  # looping wins at PP=2
    v1, _ = choose_virtual(cfg, 1, 4)
    assert v1 == 1


def test_plan_stages_balance():
    cfg = CONFIGS["enc12_d4096"]
    for n in (1, 2, 4, 8):
        plan = plan_stages(cfg, n)
        assert sum(plan.balance) == len(block_costs(cfg)) and len(plan.balance) == n
        assert plan.imbalance() < 1.25
    # 8 stages: split between attention and MLP halves keeps imbalance low
    assert plan_stages(cfg, 8).imbalance() < 1.13


def _tiny(dropout=0.0):
    return dataclasses.replace(CONFIGS["tiny"], dropout=dropout, num_layers=2, d_model=32, nhead=4,
                               dim_feedforward=64, vocab=50, seq_len=8)


def _loss_fn(cfg):
    return lambda y, t: ops.cross_entropy(y.reshape(-1, cfg.vocab), t.reshape(-1))


def _data(cfg, m, mb):
    g = torch.Generator().manual_seed(7)
    tok = torch.randint(0, cfg.vocab, (m, mb, cfg.seq_len + 1), generator=g)
    return [tok[i, :, :-1] for i in range(m)], [tok[i, :, 1:].contiguous() for i in range(m)]


def _reference(cfg, m, mb):
    torch.manual_seed(0)
    model = torch.nn.Sequential(*build_lm_blocks(cfg)).train()
    inputs, targets = _data(cfg, m, mb)
    total = 0.0
    for x, t in zip(inputs, targets):
        loss = _loss_fn(cfg)(model(x), t) / m
        loss.backward()
        total += float(loss.detach()) * m
    return model, total / m


@pytest.mark.parametrize("checkpoint", ["never", "except_last", "always"])
def test_engine_single_rank_matches_reference(checkpoint):
    cfg = _tiny()
    m, mb = 3, 2
    ref, ref_loss = _reference(cfg, m, mb)
    torch.manual_seed(0)
    model = torch.nn.Sequential(*build_lm_blocks(cfg)).train()
    eng = PipelineEngine(model, chunks=m, checkpoint=checkpoint, act_shape=(mb, cfg.seq_len, cfg.d_model),
                         act_dtype=torch.float32, loss_fn=_loss_fn(cfg), device=torch.device("cpu"))
    inputs, targets = _data(cfg, m, mb)
    st = eng.step(inputs, targets)
    assert abs(float(st.loss) - ref_loss) < 1e-5
    for (n, p), q in zip(model.named_parameters(), ref.parameters()):
        assert torch.allclose(p.grad, q.grad, atol=1e-5), n


def test_engine_dropout_recompute_consistent():
    """With dropout, checkpoint='always' must reproduce 'never' exactly (RNG replay)."""
    cfg = _tiny(dropout=0.3)
    m, mb = 2, 2
    grads = {}
    for mode in ("never", "always"):
        torch.manual_seed(0)
        model = torch.nn.Sequential(*build_lm_blocks(cfg)).train()
        eng = PipelineEngine(model, chunks=m, checkpoint=mode, act_shape=(mb, cfg.seq_len, cfg.d_model),
                             act_dtype=torch.float32, loss_fn=_loss_fn(cfg), device=torch.device("cpu"))
        inputs, targets = _data(cfg, m, mb)
        torch.manual_seed(99)
        eng.step(inputs, targets)
        grads[mode] = [p.grad.clone() for p in model.parameters()]
    for a, b in zip(grads["never"], grads["always"]):
        assert torch.allclose(a, b, atol=1e-6)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _gpu_cfg():
    # HIP-kernel-sized: head dim 64, S % 64 == 0, every GEMM dim a multiple of 8.
    return dataclasses.replace(CONFIGS["tiny"], dropout=0.0, num_layers=2, d_model=256, nhead=4,
                               dim_feedforward=512, vocab=512, seq_len=64)


def _split_cfg():
    return dataclasses.replace(_tiny(), vocab=1000)


def test_vocab_split_decoder_matches_full_cpu():
    """DecoderHead + DecoderTail == Decoder + cross-entropy (loss and every gradient)."""
    from mipipe.models import Decoder, split_decoder

    torch.manual_seed(0)
    dec = Decoder(1000, 32)
    head, tail = split_decoder(dec)
    assert head.va == 512 and tail.vb == 488
    x = torch.randn(3, 8, 32, requires_grad=True)
    t = torch.randint(0, 1000, (3, 8))
    t[0, 0] = -100  # ignored
    ref = torch.nn.functional.cross_entropy(dec(x).reshape(-1, 1000), t.reshape(-1), ignore_index=-100)
    ref.backward()
    x2 = x.detach().clone().requires_grad_()
    loss = tail(head(x2, t), t)
    loss.backward()
    assert abs(loss.item() - ref.item()) < 1e-5
    assert torch.allclose(x2.grad, x.grad, atol=1e-6)
    assert torch.allclose(head.weight.grad, dec.weight.grad[:512], atol=1e-6)
    assert torch.allclose(tail.weight.grad[:488], dec.weight.grad[512:1000], atol=1e-6)
    assert torch.allclose(tail.bias.grad[:488], dec.bias.grad[512:1000], atol=1e-6)
    assert tail.weight.grad[488:].abs().max() == 0


def _worker(rank, world, port, checkpoint, q, gpu=False, virtual=1, split=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cfg = _gpu_cfg() if gpu else (_split_cfg() if split else _tiny())
        device = torch.device("cuda", 0) if gpu else torch.device("cpu")
        dtype = torch.bfloat16 if gpu else torch.float32
        m, mb = 4, 2
        torch.manual_seed(0)
        full = torch.nn.Sequential(*build_lm_blocks(cfg))
        names = {id(p): n for n, p in full.named_parameters()}
        units = lm_pipeline_units(list(full.children()), split_decoder=split)
        if split:
            for tag, u in (("dec_head", units[-2]), ("dec_tail", units[-1])):
                names[id(u.weight)], names[id(u.bias)] = f"{tag}.weight", f"{tag}.bias"
        plan = plan_stages(cfg, world, virtual, split_decoder=split)
        chunks = [TargetSequential(*merge_units([units[i] for i in plan.slice(s)])).train().to(device, dtype)
                  for s in plan.vstages(rank)]
        stage = torch.nn.ModuleList(chunks)
        opt = FlatAdam(stage.parameters(), lr=1e-3, max_grad_norm=0.5)
        eng = PipelineEngine(chunks, chunks=m, checkpoint=checkpoint,
                             act_shape=[stage_input_shape(cfg, plan, s, mb) for s in plan.vstages(rank)],
                             act_dtype=dtype, loss_fn=_loss_fn(cfg) if rank == world - 1 else None,
                             device=device)
        inputs, targets = _data(cfg, m, mb)
        inputs = [x.to(device) for x in inputs]
        targets = [t.to(device) for t in targets]
        opt.zero_grad()
        st = eng.step(inputs if rank == 0 else None, targets)
        opt.fold_grads()
        # numpy: pickled by value (a torch tensor would be shared by fd, which
        # dies with this process)
        grads = {names[id(p)]: p.main_grad.float().cpu().numpy().copy() for p in stage.parameters()}
        sq = opt.grad_sumsq().cpu()
        dist.all_reduce(sq)
        q.put((rank, None if st.loss is None else float(st.loss), grads, float(sq)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("checkpoint,world,virtual,split", [("never", 2, 1, False), ("except_last", 2, 1, False),
                                                            ("never", 2, 2, False), ("always", 2, 3, False),
                                                            ("except_last", 3, 2, False), ("never", 2, 1, True),
                                                            ("except_last", 2, 2, True), ("always", 3, 2, True)])
def test_engine_multi_rank_gloo(checkpoint, world, virtual, split):
    cfg = _split_cfg() if split else _tiny()
    m, mb = 4, 2
    ref, ref_loss = _reference(cfg, m, mb)
    ref_params = dict(ref.named_parameters())
    if split:  # the vocabulary-split head / tail gradients are row blocks of the decoder's
        dec_name = [n for n in ref_params if n.endswith(".weight")][-1].rsplit(".", 1)[0]
        dw, db = ref_params[dec_name + ".weight"].grad, ref_params[dec_name + ".bias"].grad
        va, v = 512, cfg.vocab
        pad = lambda t: torch.cat([t, torch.zeros((512 - (v - va),) + t.shape[1:])])  # noqa: E731
        ref_params = {n: p for n, p in ref_params.items() if not n.startswith(dec_name + ".")}
        for name, g in (("dec_head.weight", dw[:va]), ("dec_head.bias", db[:va]),
                        ("dec_tail.weight", pad(dw[va:v])), ("dec_tail.bias", pad(db[va:v]))):
            ref_params[name] = torch.nn.Parameter(torch.zeros_like(g))
            ref_params[name].grad = g
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, checkpoint, q, False, virtual, split))
             for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    total_sq = 0.0
    seen = set()
    for rank, loss, grads, sq in results:
        if loss is not None:
            assert abs(loss - ref_loss) < 1e-5
        for name, g in grads.items():
            assert torch.allclose(torch.from_numpy(g), ref_params[name].grad, atol=1e-5), name
            seen.add(name)
        total_sq = sq
    assert seen == set(ref_params)
    ref_sq = sum(float(p.grad.double().pow(2).sum()) for p in ref.parameters())
    assert abs(total_sq - ref_sq) / ref_sq < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("checkpoint,virtual,split", [("never", 1, False), ("always", 1, False),
                                                      ("except_last", 2, False), ("never", 2, True)])
def test_engine_two_ranks_share_gpu(checkpoint, virtual, split):
    """Two pipeline ranks on one MI355X (gloo, host-staged boundaries): the HIP
    kernels of both stages and the multi-rank schedule against the single-rank
    engine on the whole model (same bf16 kernels, same initial weights)."""
    cfg = _gpu_cfg()
    m, mb = 4, 2
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    full = torch.nn.Sequential(*build_lm_blocks(cfg)).train().to(dev, torch.bfloat16)
    opt = FlatAdam(full.parameters(), lr=1e-3, max_grad_norm=0.5)
    eng = PipelineEngine(full, chunks=m, checkpoint="never", act_shape=(mb, cfg.seq_len), act_dtype=torch.bfloat16,
                         loss_fn=_loss_fn(cfg), device=dev)
    inputs, targets = _data(cfg, m, mb)
    opt.zero_grad()
    st = eng.step([x.to(dev) for x in inputs], [t.to(dev) for t in targets])
    ref_loss = float(st.loss)
    ref_sq = float(opt.grad_sumsq())
    ref = {n: p.main_grad.float().cpu() for n, p in full.named_parameters()}

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, checkpoint, q, True, virtual, split)) for r in range(2)]
    for p in procs:
        p.start()
    results = [q.get(timeout=300) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    if split:
        dec_name = [n for n in ref if n.endswith(".weight")][-1].rsplit(".", 1)[0]
        dw, db = ref.pop(dec_name + ".weight"), ref.pop(dec_name + ".bias")
        va, v = 256, cfg.vocab  # split_point(512)
        ref.update({"dec_head.weight": dw[:va], "dec_head.bias": db[:va],
                    "dec_tail.weight": dw[va:], "dec_tail.bias": db[va:]})
    seen = set()
    for rank, loss, grads, sq in results:
        if loss is not None:
            assert abs(loss - ref_loss) < 2e-3 * abs(ref_loss)
        for name, g in grads.items():
            g = torch.from_numpy(g)
            scale = ref[name].abs().max().item() + 1e-6
            assert (g - ref[name]).abs().max().item() < 2e-2 * scale, name
            seen.add(name)
        assert abs(sq - ref_sq) / ref_sq < 1e-2
    assert seen == set(ref)


@pytest.mark.gpu
def test_engine_deferred_wgrad_same_gradients():
    """defer_wgrad (weight GEMMs after the last backward, K-segmented) gives the
    gradients of the immediate path."""
    cfg = _gpu_cfg()
    m, mb = 4, 2
    dev = torch.device("cuda", 0)
    inputs, targets = _data(cfg, m, mb)
    grads = {}
    for defer in (False, True):
        torch.manual_seed(0)
        full = torch.nn.Sequential(*build_lm_blocks(cfg)).train().to(dev, torch.bfloat16)
        opt = FlatAdam(full.parameters(), lr=1e-3)
        eng = PipelineEngine(full, chunks=m, checkpoint="except_last", act_shape=(mb, cfg.seq_len),
                             act_dtype=torch.bfloat16, loss_fn=_loss_fn(cfg), device=dev, defer_wgrad=defer)
        opt.zero_grad()
        eng.step([x.to(dev) for x in inputs], [t.to(dev) for t in targets])
        opt.fold_grads()
        grads[defer] = {n: p.main_grad.clone() for n, p in full.named_parameters()}
    for n, g in grads[False].items():
        scale = g.abs().max().item() + 1e-6
        assert (grads[True][n] - g).abs().max().item() < 1e-2 * scale, n


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("checkpoint,virtual,split,skips", ENGINE_CASES)
def test_engine_cases_gloo_emulation(world, checkpoint, virtual, split, skips):
    """The cases tests/test_gpu_pipeline.py runs over RCCL on 2 / 4 GPUs, here
    rank-for-rank over gloo on CPU (fp32, exact comparison)."""
    run_engine_case("cpu", world, checkpoint, virtual, split, skips)


def test_check_hw_queues_warns_below_minimum(monkeypatch):
    """RCCL ranks want a hardware queue per stream (profiles/hw_queue_sharing.txt):
    below MIN_HW_QUEUES the engine's transport warns; bench.py raises the value
    before HIP initialises."""
    import warnings

    from mipipe.parallel.p2p import MIN_HW_QUEUES, check_hw_queues

    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "4")
    with pytest.warns(RuntimeWarning, match="GPU_MAX_HW_QUEUES=4"):
        assert not check_hw_queues()
    monkeypatch.delenv("GPU_MAX_HW_QUEUES")
    with pytest.warns(RuntimeWarning):
        assert not check_hw_queues()  # HIP's default is 4
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", str(MIN_HW_QUEUES))
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        assert check_hw_queues()
    src = open(os.path.join(os.path.dirname(__file__), "..", "bench.py")).read()
    assert src.index("GPU_MAX_HW_QUEUES") < src.index("import torch")


def test_planner_unloads_busiest_rank():
    """The PP=8 enc12 plan: the post-pass moves one unit off the vocabulary-tail
    rank (measured 321 -> 287 ms per step, profiles/pp8_ranks_mb64.txt) while the
    simulated step stays within 0.2 % of the refined one."""
    from mipipe.parallel.stage import _unload_busiest, choose_virtual, simulate_step

    cfg = CONFIGS["enc12_d4096"]
    bwd = 2.0 + 31 / 32
    v, plan = choose_virtual(cfg, 8, 32, bwd_ratio=bwd, micro_batch=64)
    assert v == 2 and plan.split_decoder
    assert plan.balance[6:8] == [4, 4]
    assert plan.imbalance() < 1.03

    def sim(p):
        return simulate_step([p.stage_cost(g) for g in range(16)], 8, 2, 32, bwd, deferred_w=1.0 / bwd)[0]

    # from the split the simulation alone prefers, the post-pass reaches a less loaded busiest rank
    import dataclasses as dc

    before = dc.replace(plan, balance=plan.balance[:6] + [3, 5] + plan.balance[8:])
    after = _unload_busiest(before, plan.costs, 32, bwd, sim(before))
    peak = lambda p: max(p.rank_cost(r) for r in range(8))  # noqa: E731
    assert peak(after) < peak(before)
    assert sim(after) <= sim(before) * 1.002


# ------------------------------------------------------------------ IPC transport (host mode)
@pytest.mark.parametrize("world,case", [(2, c) for c in ENGINE_CASES] + [(4, ENGINE_CASES[1]), (4, ENGINE_CASES[3])])
def test_engine_cases_ipc_links_host(world, case):
    """transport='ipc' (mipipe.parallel.ipc.IpcChannels): activations and
    gradients through the native IPC links' slot rings and sequence counters
    -- here their host mode (shared memory, memcpy), the same protocol the
    device mode runs on a GPU -- against the single-rank engine, exactly."""
    run_engine_case("ipc_cpu", world, *case)


def test_engine_ipc_dropout_recompute_bit_identical_host():
    """Dropout 0.2 on both ranks: 'except_last' / 'always' == 'never' bit for bit
    (each rank recomputes with the RNG state it saved at its forward)."""
    from helpers.engine_cases import run_dropout_recompute_case

    run_dropout_recompute_case("ipc_cpu", 2)


@pytest.mark.parametrize("virtual,split", [(1, False), (2, True)])
def test_engine_ipc_links_host_slot_reuse_over_steps(virtual, split):
    """Three steps: 2-slot host rings wrap within a step (plain chain), or the
    slots are reused step after step (looping placement)."""
    run_engine_case("ipc_cpu", 2, "except_last", virtual, split, False, steps=3)


def test_planner_boundary_terms_and_wide_candidates():
    """choose_virtual tries v beyond 3 and prices every
    stage-boundary message and chunk action: with the boundary terms at zero a
    deep GPT-2-XL loop simulates faster than v = 2; charged for its extra
    boundaries (26 MB per message at micro-batch 8 x 1024) it does not."""
    from mipipe.parallel.stage import boundary_terms, choose_virtual, plan_stages, simulate_step

    cfg = CONFIGS["gpt2_xl"]
    tr, la = boundary_terms(cfg, 8)
    assert tr > 0 and la > 0
    p2, p4 = plan_stages(cfg, 8, 2, 8, False, 3.0), plan_stages(cfg, 8, 4, 8, True, 3.0)

    def sim(p, v, t=0.0, lch=0.0):
        return simulate_step([p.stage_cost(g) for g in range(8 * v)], 8, v, 8, 3.0, deferred_w=1 / 3.0, transfer=t,
                             launch=lch)[0]

    assert sim(p4, 4) < sim(p2, 2)                    # free boundaries: the deep loop wins
    assert sim(p4, 4, tr, la) > sim(p2, 2, tr, la)    # priced boundaries: it does not
    # the planner considers v up to units / stages (capped at 8)
    v, _ = choose_virtual(CONFIGS["enc12_d4096"], 2, 8, micro_batch=64)
    assert v > 3

