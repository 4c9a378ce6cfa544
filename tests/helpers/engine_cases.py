"""Multi-rank engine cases shared by the RCCL (one rank per GPU) and the gloo
(CPU) tests: each rank builds its slice of a 4-layer LM, runs one engine step
and reports its gradients; the caller compares them with the single-rank
engine on the whole model."""
import dataclasses
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mipipe import ops
from mipipe.models import CONFIGS, TargetSequential, build_lm_blocks, lm_pipeline_units
from mipipe.models.long_skip import insert_long_skips
from mipipe.models.transformer import merge_units
from mipipe.optim import FlatAdam
from mipipe.parallel import PipelineEngine, plan_stages
from mipipe.parallel.p2p import MIN_HW_QUEUES
from mipipe.parallel.stage import stage_input_shape

# (checkpoint, virtual chunks per rank, vocabulary-split head, cross-stage skips)
ENGINE_CASES = [
    ("never", 1, False, False),
    ("except_last", 1, False, False),
    ("always", 1, False, False),
    ("except_last", 2, True, False),  # looping placement + split head: the PP=8 plan shape
    ("never", 1, False, True),        # @skippable long residuals across ranks (BASELINE config #5)
]
SKIP_PAIRS = [(0, 3), (1, 2)]


# Modes: "cpu" (gloo, fp32), "nccl" (RCCL, one rank per GPU), "ipc_cpu" (gloo for
# collectives, activations over shared-memory IPC links), "ipc_gpu" (every rank
# on cuda:0, activations over device-memory IPC links -- mipipe.parallel.ipc).
GPU_MODES = ("nccl", "ipc_gpu", "auto_gpu", "auto_sdma_gpu")


def case_cfg(mode):
    base = CONFIGS["tiny"]
    if mode in GPU_MODES:  # HIP-kernel-sized shapes
        return dataclasses.replace(base, dropout=0.0, num_layers=4, d_model=256, nhead=4, dim_feedforward=512,
                                   vocab=512, seq_len=64)
    return dataclasses.replace(base, dropout=0.0, num_layers=4, d_model=32, nhead=4, dim_feedforward=64,
                               vocab=1000, seq_len=8)


def _setting(mode):
    if mode in GPU_MODES:
        return torch.bfloat16, 8, 2
    return torch.float32, 8, 2


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


def _device(mode, rank):
    if mode == "nccl":
        return torch.device("cuda", rank)
    return torch.device("cuda", 0) if mode in ("ipc_gpu", "auto_gpu", "auto_sdma_gpu") else torch.device("cpu")


def _grads(params, names):
    out = {}
    for p in params:
        g = p.main_grad if hasattr(p, "main_grad") else p.grad
        out[names[id(p)]] = g.float().cpu().numpy().copy()
    return out


def _transport_options(mode, steps, virtual):
    opts = {}
    if (mode.startswith("ipc") or mode.startswith("auto")) and steps > 1 and virtual == 1:
        opts["slots"] = 2
    if mode == "auto_sdma_gpu":  # the cross-GPU engine (copies on the links' copy streams), on one GPU
        opts["engine"] = "sdma"
    return opts or None


def worker(rank, world, port, mode, checkpoint, virtual, split, skips, q, dropout=0.0, seed=0, steps=1):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = _device(mode, rank)
    if mode == "nccl":
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    else:
        if dev.type == "cuda":
            torch.cuda.set_device(dev)
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cfg = dataclasses.replace(case_cfg(mode), dropout=dropout)
        dtype, m, mb = _setting(mode)
        torch.manual_seed(0)
        full = torch.nn.Sequential(*build_lm_blocks(cfg))
        names = {id(p): n for n, p in full.named_parameters()}
        units = lm_pipeline_units(list(full.children()), split_decoder=split)
        if split:
            for tag, u in (("dec_head", units[-2]), ("dec_tail", units[-1])):
                names[id(u.weight)], names[id(u.bias)] = f"{tag}.weight", f"{tag}.bias"
        plan = plan_stages(cfg, world, virtual, split_decoder=split)
        chunks = []
        for s in plan.vstages(rank):
            sl = plan.slice(s)
            us = [units[i] for i in sl]
            if skips:
                us = insert_long_skips(us, SKIP_PAIRS, start=sl.start)
            chunks.append(TargetSequential(*merge_units(us)).train().to(dev, dtype))
        stage = torch.nn.ModuleList(chunks)
        opt = FlatAdam(stage.parameters(), lr=1e-3, max_grad_norm=0.5)
        eng = PipelineEngine(chunks, chunks=m, checkpoint=checkpoint,
                             act_shape=[stage_input_shape(cfg, plan, s, mb) for s in plan.vstages(rank)],
                             act_dtype=dtype, loss_fn=_loss_fn(cfg) if rank == world - 1 else None,
                             device=dev, watchdog=120.0,
                             skip_shapes={"skip": ((mb, cfg.seq_len, cfg.d_model), dtype)},
                             transport=("ipc" if mode.startswith("ipc") else
                                        "auto" if mode.startswith("auto") else "rccl"),
                             # several steps of a plain chain: a 2-slot ring is reused many times over
                             # (a looping placement keeps one slot per message of the step)
                             transport_options=_transport_options(mode, steps, virtual))
        if mode.startswith("ipc") or mode.startswith("auto"):
            assert type(eng.chan).__name__ == "IpcChannels"
        if mode.startswith("auto"):  # the self-test passed: no fallback
            assert eng.transport == ("ipc-sdma" if mode == "auto_sdma_gpu" else "ipc-inline"), eng.transport
            assert eng.transport_note is None
        inputs, targets = _data(cfg, m, mb)
        for _ in range(steps):  # no optimizer step: every step computes the same gradients
            torch.manual_seed(1000 + seed * 97 + rank)  # dropout streams: per rank, same in every mode
            opt.zero_grad()
            st = eng.step([x.to(dev) for x in inputs] if rank == 0 else None, [t.to(dev) for t in targets])
        opt.fold_grads()
        sq = opt.grad_sumsq()
        dist.all_reduce(sq)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        q.put((rank, None if st.loss is None else float(st.loss), _grads(stage.parameters(), names), float(sq),
               len(eng.skip_routes)))
        q.close()
        q.join_thread()  # delivered before any teardown
    finally:
        dist.destroy_process_group()


def single_rank_reference(mode, checkpoint, split, skips):
    cfg = case_cfg(mode)
    dtype, m, mb = _setting(mode)
    dev = torch.device("cuda", 0) if mode in GPU_MODES else torch.device("cpu")
    torch.manual_seed(0)
    full = torch.nn.Sequential(*build_lm_blocks(cfg))
    names = {id(p): n for n, p in full.named_parameters()}
    units = lm_pipeline_units(list(full.children()))
    if skips:
        units = insert_long_skips(units, SKIP_PAIRS)
    model = TargetSequential(*merge_units(units)).train().to(dev, dtype)
    opt = FlatAdam(model.parameters(), lr=1e-3)
    eng = PipelineEngine(model, chunks=m, checkpoint=checkpoint, act_shape=(mb, cfg.seq_len),
                         act_dtype=dtype, loss_fn=_loss_fn(cfg), device=dev)
    inputs, targets = _data(cfg, m, mb)
    opt.zero_grad()
    loss = float(eng.step([x.to(dev) for x in inputs], [t.to(dev) for t in targets]).loss)
    opt.fold_grads()
    sq = float(opt.grad_sumsq())
    ref = {k: torch.from_numpy(v) for k, v in _grads(model.parameters(), names).items()}
    if split:
        dec = [n for n in ref if n.endswith(".weight")][-1].rsplit(".", 1)[0]
        dw, db = ref.pop(dec + ".weight"), ref.pop(dec + ".bias")
        from mipipe.models.vocab_split import split_point

        va, v = split_point(cfg.vocab), cfg.vocab
        pad_to = max(va, v - va)

        def pad(t):
            extra = pad_to - t.shape[0]
            return torch.cat([t, torch.zeros((extra,) + t.shape[1:])]) if extra > 0 else t

        ref.update({"dec_head.weight": pad(dw[:va]), "dec_head.bias": pad(db[:va]),
                    "dec_tail.weight": pad(dw[va:v]), "dec_tail.bias": pad(db[va:v])})
    return loss, ref, sq


def spawn_ranks(mode, world, checkpoint, virtual, split, skips, dropout=0.0, seed=0, steps=1):
    """Runs one engine step on ``world`` spawned ranks; returns their results."""
    if mode in GPU_MODES:
        # the ranks initialise HIP after spawn: give every stream its own
        # hardware queue (mipipe.parallel.p2p.check_hw_queues)
        os.environ["GPU_MAX_HW_QUEUES"] = str(MIN_HW_QUEUES)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=worker, args=(r, world, port, mode, checkpoint, virtual, split, skips, q, dropout,
                                              seed, steps))
             for r in range(world)]
    for p in procs:
        p.start()
    import queue as _queue
    import time as _time

    results = []
    deadline = _time.time() + 300
    try:
        while len(results) < world:
            try:
                results.append(q.get(timeout=1.0))
            except _queue.Empty:
                dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
                if dead or _time.time() > deadline:
                    raise AssertionError(f"rank(s) failed (exit codes {dead}) or timed out; "
                                         f"{len(results)}/{world} results")
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.exitcode is None:
                p.kill()
    for p in procs:
        assert p.exitcode == 0
    return sorted(results, key=lambda r: r[0])


def run_dropout_recompute_case(mode, world, virtual=1):
    """Dropout 0.2 on every rank: 'except_last' and 'always' recompute with the
    RNG state each rank saved at its forward, so their gradients are
    BIT-identical to 'never' on every rank (and a different seed changes them)."""
    base = spawn_ranks(mode, world, "never", virtual, False, False, dropout=0.2)
    other = spawn_ranks(mode, world, "never", virtual, False, False, dropout=0.2, seed=1)
    assert any(not (base[r][2][n] == other[r][2][n]).all() for r in range(world) for n in base[r][2])
    for ck in ("except_last", "always"):
        res = spawn_ranks(mode, world, ck, virtual, False, False, dropout=0.2)
        for (rank, loss, grads, sq, _), (_, loss0, grads0, sq0, _) in zip(res, base):
            assert loss == loss0, (ck, rank)
            for name, g in grads.items():
                assert (g == grads0[name]).all(), (ck, rank, name)


def run_engine_case(mode, world, checkpoint, virtual, split, skips, steps=1):
    """Spawns ``world`` ranks and checks loss, every gradient and the global
    gradient norm against the single-rank engine (after ``steps`` steps)."""
    ref_loss, ref, ref_sq = single_rank_reference(mode, checkpoint, split, skips)
    results = spawn_ranks(mode, world, checkpoint, virtual, split, skips, steps=steps)
    rel = 2e-2 if mode in GPU_MODES else 1e-4
    seen = set()
    for rank, loss, grads, sq, nskips in results:
        if loss is not None:
            assert abs(loss - ref_loss) < (2e-3 if mode in GPU_MODES else 1e-5) * abs(ref_loss)
        for name, g in grads.items():
            g = torch.from_numpy(g)
            r = ref[name]
            if g.shape != r.shape:  # a padded split-head block: compare the real rows
                r = r[: g.shape[0]] if r.shape[0] > g.shape[0] else r
                g = g[: r.shape[0]]
            scale = r.abs().max().item() + 1e-6
            assert (g - r).abs().max().item() <= rel * scale, name
            seen.add(name)
        assert abs(sq - ref_sq) / ref_sq < (1e-2 if mode in GPU_MODES else 1e-4)
        if skips:
            assert nskips > 0, "no skip crossed a stage boundary"
    assert seen == set(ref)
