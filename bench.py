#!/usr/bin/env python3
"""mipipe headline benchmark: pipeline-parallel LM training throughput on MI355X.

Metric (BASELINE.json): tokens/sec for the 12-layer Transformer (d_model 4096,
nhead 16) at PP = 1/2/4/8, plus the pipeline bubble.  One process per GPU,
pipeline stages connected by self-tested device-memory IPC links (DMA copies
into the receiver's slots; RCCL send/recv as the common fall-back), GPipe
schedule, chunks = 4 x PP
(BASELINE configs #2/#3: PP=2 chunks=8, PP=8 chunks=32), fixed micro-batch, so
per-GPU work is constant as PP grows ("weak" scaling).

Model = the reference driver's LM (/root/reference/main.py): embedding x sqrt(E)
+ sinusoidal positions -> 12 x post-norm TransformerEncoderLayer (ReLU,
dim_feedforward = d_model, dropout 0.2) -> Linear decoder over the WikiText-2
vocabulary (28,782) -> cross-entropy; Adam with clip_grad_norm(0.5).  Random
init, synthetic tokens (no dataset access).  bf16 compute, fp32 master weights
and gradient accumulation.

    python bench.py                                  # 1 GPU
    torchrun --nproc-per-node 8 bench.py --gpus 8    # PP = 8
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import sys
import time

# Before HIP initialises: enough hardware queues that the compute stream and
# every RCCL communicator stream get one each.  At HIP's default of 4, streams
# share in-order queues, and a pre-posted RCCL receive (a spinning kernel)
# holds back the compute kernels queued behind it -- serialising the pipeline,
# or deadlocking a looping one (profiles/hw_queue_sharing.txt).
if int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 16:
    os.environ["GPU_MAX_HW_QUEUES"] = "16"

import torch
import torch.distributed as dist

# the reference's derived throughput on ITS config (main.py: fp32,
# 16 x TransformerEncoderLayer(2048, 32, 2048), V 28,782, batch 32 x 128,
# chunks 4, 2 GPUs).  vs_baseline is only reported for that same config
# (--config ref_main --dtype fp32 --chunks 4 --micro-batch 8); any other
# model / precision is a different workload and gets vs_baseline = null.
REF_TOKENS_PER_S = {"never": 3500.0, "except_last": 2850.0}
REF_PEAK_MB = {"never": [6361.6, 7954.0], "except_last": [5051.8, 6254.1]}


def matches_reference(cfg, args, m, mb) -> bool:
    return (cfg.name == "ref_main" and args.dtype == "fp32" and m == 4 and m * mb == 32
            and cfg.seq_len == 128 and args.checkpoint in REF_TOKENS_PER_S)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="enc12_d4096")
    ap.add_argument("--micro-batch", type=int, default=None,
                    help="sequences per micro-batch (default 128 for enc12_d4096, 8 for ref_main (the reference's) "
                         "and gpt2_xl)")
    ap.add_argument("--seq-len", type=int, default=None)
    ap.add_argument("--num-layers", type=int, default=None, help="override the model's layer count (tests)")
    ap.add_argument("--act-dropout", type=float, default=None,
                    help="override the dropout between the MLP's activation and its second linear (default: the "
                         "config's -- enc12 / ref_main: = dropout, as torch's TransformerEncoderLayer; gpt2_xl: 0, "
                         "as GPT-2's MLP)")
    ap.add_argument("--chunks", type=int, default=None, help="micro-batches per step (default 4 x PP)")
    ap.add_argument("--checkpoint", default="auto", choices=["auto", "never", "except_last", "always"],
                    help="auto = the BASELINE.json config for this model and PP: enc12 'except_last' at PP=8 "
                         "(config #3), else 'never' (config #2); gpt2_xl 'always' (config #4)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--lr", type=float, default=1e-4)
    ap.add_argument("--clip", type=float, default=0.5)
    ap.add_argument("--no-bubble", action="store_true", help="skip the extra instrumented step")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu = gloo + fp32 plumbing check of the multi-rank path (tests only)")
    ap.add_argument("--plan", default="auto", choices=["auto", "analytic", "measured"],
                    help="stage-plan unit costs: analytic FLOPs, or measured (mipipe.parallel.calibrate: layer / head / "
                         "tail stages timed in the engine on this GPU, all-reduced over the ranks; cached).  auto = "
                         "measured on GPUs at PP > 1")
    ap.add_argument("--plan-objective", default="makespan", choices=["makespan", "balance"],
                    help="stage plan: shortest simulated step (may load ranks unevenly to shorten fill / drain) "
                         "or the most even per-rank work")
    ap.add_argument("--plan-select", default="auto", choices=["auto", "emulate", "model"],
                    help="final pick of the stage plan: emulate = the few best plans of the cost model are each run "
                         "on every rank alone (loop-back engine, a few steps) and the fastest by measured walls "
                         "wins, after single units were moved off each candidate's slowest measured rank "
                         "(mipipe.parallel.calibrate.select_plan_by_emulation; profiles/plan_table_r5.txt, "
                         "plan_refine_r6.txt); "
                         "model = the cost model's choice.  auto = emulate with measured costs on GPUs at PP > 1")
    ap.add_argument("--split-decoder", default="auto", choices=["auto", "on", "off"],
                    help="cut the LM head along the vocabulary into two pipeline units")
    ap.add_argument("--chunks-per-rank", dest="virtual", default="auto",
                    help="model chunks per rank (looping placement); 'auto' = shortest simulated step")
    ap.add_argument("--impl", default="engine", choices=["engine", "pipe"],
                    help="engine = one process per GPU (default; what torchrun launches); "
                         "pipe = the single-process mipipe.Pipe driving --gpus devices with peer copies")
    ap.add_argument("--watchdog", type=float, default=300.0,
                    help="seconds without pipeline progress before a rank reports its pending transfers and "
                         "exits (0 = off)")
    ap.add_argument("--dp", type=int, default=1,
                    help="data-parallel replicas of the pipeline (world = PP x DP; gradients averaged by bucketed "
                         "RCCL all-reduces overlapped with the deferred weight gradients). Default 1: PP = world")
    ap.add_argument("--transport", default="auto", choices=["auto", "rccl", "ipc"],
                    help="stage-boundary transport of the engine: auto (default) = self-tested device-memory IPC "
                         "links (payload and completion flag both DMA copies on the links' copy streams: no kernel "
                         "there; the consumer's own stream waits for the flag; profiles/ipc_cu_free_r6.txt), every "
                         "rank falling back to RCCL together if a link fails its set-up or self-test; rccl = "
                         "send/recv of the process group "
                         "(each receive a resident kernel on CUs); ipc = the IPC links without the self-test "
                         "(mipipe.parallel.ipc)")
    ap.add_argument("--shared-gpu", action="store_true",
                    help="every rank on cuda:0 (gloo for the small collectives, --transport ipc for the stage "
                         "boundaries): a one-GPU rehearsal of the multi-rank step for timelines "
                         "(tools/profile_ranks.py); NOT a throughput number for n_gpus ranks")
    ap.add_argument("--pipe-balance", default=None,
                    help="--impl pipe: transformer LAYERS per partition, e.g. 8,8 (the reference's main.py: "
                         "embedding + layers 0-7 | layers 8-15 + decoder); with --gpus 1 every partition sits on "
                         "cuda:0 and each boundary is a native device-to-device copy on the copy streams "
                         "(Pipe(balance=..., copy_same_device=True)), else partition j on cuda:j")
    ap.add_argument("--pipe-stage-streams", default="dedicated", choices=["shared", "dedicated"],
                    help="--impl pipe with several partitions on one GPU: compute them all on the device's stream "
                         "(shared, the reference's one stream per device) or each later one on its own stream")
    ap.add_argument("--pipe-boundary", default="copy", choices=["copy", "inplace"],
                    help="--impl pipe, several partitions on ONE GPU: a native device-to-device copy on the copy "
                         "streams at each boundary (copy, the multi-GPU path) or the tensor handed over in place "
                         "(inplace: what the reference's Copy does on one device -- .to(same device) is a no-op)")
    ap.add_argument("--pipe-copy-streams", type=int, default=1,
                    help="--impl pipe: copy streams per partition (default 1; 0 = the reference's one per micro-batch)")
    ap.add_argument("--opt-overlap", default="off", choices=["on", "off"],
                    help="on = the Adam step runs on a side stream in forward-order chunks and the next step's "
                         "forward waits per module (FlatAdam(overlap_modules=...)): the memory-bound update fills "
                         "CUs the GEMMs leave idle")
    ap.add_argument("--skips", default="none", choices=["none", "unet"],
                    help="unet = @skippable long residuals layer i -> layer L-1-i across stages "
                         "(BASELINE config #5; stash rank -> pop rank over their own xGMI link)")
    return ap.parse_args()


def main() -> int:
    t_main = time.perf_counter()
    startup = {}  # start-up breakdown (s), reported in the JSON
    args = parse()
    if os.environ.get("MIPIPE_BENCH_PROGRESS", "0") != "0":
        import faulthandler

        # a rehearsal that stops printing shows where every thread is, every 60 s
        faulthandler.dump_traceback_later(60, repeat=True, file=sys.stderr)
    if args.impl == "pipe":
        return run_pipe(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE", file=sys.stderr)
    on_gpu = args.device == "cuda"
    if args.shared_gpu:
        args.transport = "ipc"  # RCCL refuses two ranks on one GPU
    if on_gpu:
        local = 0 if args.shared_gpu else local
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
        if world > 1:
            if args.shared_gpu:
                dist.init_process_group("gloo")
            else:
                dist.init_process_group("nccl", device_id=device)
    else:
        device = torch.device("cpu")
        args.dtype = "fp32"
        if world > 1:
            dist.init_process_group("gloo")

    def sync():
        if on_gpu:
            torch.cuda.synchronize()

    import mipipe  # noqa: F401
    from mipipe import ops
    from mipipe.models import CONFIGS
    from mipipe.optim import FlatAdam
    from mipipe.parallel import PipelineEngine, plan_stages
    from mipipe.parallel.stage import build_stage, choose_virtual, simulate_step, stage_input_shape

    cfg = _config(args)
    S, E, V = cfg.seq_len, cfg.d_model, cfg.vocab
    dp = args.dp
    if dp < 1 or world % dp:
        raise SystemExit(f"--dp {dp} does not divide the world size {world}")
    if dp > 1 and args.skips != "none":
        raise SystemExit("--skips with --dp > 1 is not supported")
    pp = world // dp
    replica, prank = divmod(rank, pp)  # stage prank of pipeline replica `replica`
    if cfg.name == "gpt2_xl":
        # BASELINE config #4: GPT-2-XL PP=8 chunks=8, checkpoint='always'
        m = args.chunks or (8 if pp == 8 else 4 * pp)
        auto_ckpt = "always"
    else:
        # configs #2 / #3: chunks = 4 x PP; the full-node PP=8 run uses 'except_last'
        m = args.chunks or 4 * pp
        auto_ckpt = "except_last" if pp == 8 else "never"
    if args.checkpoint == "auto":
        args.checkpoint = auto_ckpt
    mb = args.micro_batch or _default_micro_batch(cfg, pp)
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32

    splits = {"auto": (False, True), "on": (True,), "off": (False,)}[args.split_decoder]
    # backward / forward cost: 2, plus the recomputed forward of checkpointed micro-batches
    recompute = {"never": 0.0, "except_last": (m - 1) / m, "always": 1.0}[args.checkpoint]
    bwd_ratio = 2.0 + recompute
    # measured by default on GPUs at PP > 1 (not in the one-GPU rehearsal: its ranks would time each other)
    plan_mode = args.plan if args.plan != "auto" else ("measured" if on_gpu and pp > 1 and not args.shared_gpu
                                                       else "analytic")
    cost_fn = None
    unit_ms = None
    plan_report = None
    startup["process_init"] = time.perf_counter() - t_main  # torch import, process group
    if plan_mode == "measured" and pp > 1:
        from mipipe.parallel.calibrate import CalibrationError, calibrated_costs, engine_unit_costs

        t_ = time.perf_counter()
        try:
            unit_ms = calibrated_costs(cfg, mb, m, args.checkpoint, device=device, dtype=dtype)
            cost_fn = lambda split: engine_unit_costs(cfg, unit_ms, split)  # noqa: E731
        except CalibrationError as exc:  # raised on every rank alike: all fall back together
            print(f"warning: {exc}; planning with analytic costs", file=sys.stderr)
        startup["calibration"] = time.perf_counter() - t_
    if args.virtual == "auto":
        virtual, plan = choose_virtual(cfg, pp, m, split_options=splits, bwd_ratio=bwd_ratio, micro_batch=mb,
                                       cost_fn=cost_fn, objective=args.plan_objective)
    else:
        virtual = int(args.virtual)
        split = splits[-1] and pp > 1
        plan = plan_stages(cfg, pp, virtual, m, split_decoder=split, bwd_ratio=bwd_ratio,
                           costs=cost_fn(split) if cost_fn is not None else None, objective=args.plan_objective)
    select = args.plan_select
    if select == "auto":
        select = "emulate" if (cost_fn is not None and args.virtual == "auto" and args.skips == "none"
                               and args.plan_objective == "makespan") else "model"
    if select == "emulate" and pp > 1:
        if cost_fn is None:
            raise SystemExit("--plan-select emulate needs measured costs (--plan measured, on GPUs)")
        from mipipe.parallel.calibrate import select_plan_by_emulation
        from mipipe.parallel.stage import candidate_plans

        t_ = time.perf_counter()
        cands = candidate_plans(cfg, pp, m, bwd_ratio, mb, cost_fn, split_options=splits)
        if len(cands) > 1:
            # ranks sharing one GPU measure each other's time slices: walls of a refinement move (two ranks
            # emulating) are not comparable with the all-rank ones, so --shared-gpu skips the refinement
            plan, plan_report = select_plan_by_emulation(cfg, cands, prank, m, mb, args.checkpoint, unit_ms,
                                                         device=device, dtype=dtype, replica=replica,
                                                         refine_rounds=0 if args.shared_gpu else 6)
            virtual = plan.virtual
        else:
            plan, virtual = cands[0], cands[0].virtual
            plan_report = {"method": "one candidate within 6 % of the model's best: no emulation needed",
                           "candidates": [{"v": plan.virtual, "split_decoder": plan.split_decoder,
                                           "balance": list(plan.balance)}], "chosen": 0}
        startup["plan_emulation"] = time.perf_counter() - t_
    from mipipe.parallel.watchdog import Watchdog

    wd = Watchdog(args.watchdog) if args.watchdog > 0 else None
    act_shapes = [stage_input_shape(cfg, plan, vs, mb) for vs in plan.vstages(prank)]
    # The stage transport first, before the stages take their memory: link set-up maps peer memory, and it is
    # kept out of the way of the big allocations (profiles/ipc_import_stall_r5.txt).
    early_chan = None
    if world > 1 and dp == 1 and args.skips == "none":
        from mipipe.parallel.engine import make_transport

        item = torch.empty((), dtype=dtype).element_size()
        t_ = time.perf_counter()
        early_chan, _, _ = make_transport(list(range(world)), device=device, chunks=m, virtual=virtual,
                                          recv_bytes=max(torch.Size(s_).numel() for s_ in act_shapes) * item,
                                          transport=args.transport, watchdog=wd)
        startup["transport"] = time.perf_counter() - t_
        if getattr(early_chan, "setup_s", None) is not None:  # IPC links: set-up / self-test split
            startup["transport_link_setup"] = early_chan.setup_s
            startup["transport_self_test"] = early_chan.selftest_s
    t_ = time.perf_counter()
    torch.manual_seed(1234 + prank)  # same initial weights in every data-parallel replica
    # Build only this rank's chunks (analytic plan; nothing else is instantiated).
    from mipipe.models.long_skip import unet_pairs

    skip_pairs = unet_pairs(cfg.num_layers) if args.skips == "unet" else []
    stages = [build_stage(cfg, plan, vs, device=device, dtype=dtype, skips=skip_pairs).train()
              for vs in plan.vstages(prank)]
    params = [p for st_ in stages for p in st_.parameters()]
    n_params_local = sum(p.numel() for p in params)

    opt = FlatAdam(params, lr=args.lr, max_grad_norm=args.clip,
                   overlap_modules=stages if args.opt_overlap == "on" else None)

    is_last = prank == pp - 1
    groups = dpg = None
    if dp > 1:
        from mipipe.parallel.data_parallel import DataParallelGrads, make_pp_dp_groups

        ipc_opts = None
        if args.transport == "ipc":
            item = torch.empty((), dtype=dtype).element_size()
            ipc_opts = {"device": device, "slots": m * virtual,
                        "recv_bytes": max(torch.Size(s_).numel() for s_ in act_shapes) * item}
        groups = make_pp_dp_groups(pp, dp, wrap=virtual > 1, transport="ipc" if args.transport == "ipc" else "rccl",
                                   ipc_options=ipc_opts)
        dpg = DataParallelGrads(opt, groups.dp_group)

    def loss_fn(y, t):
        return ops.cross_entropy(y.reshape(-1, V), t.reshape(-1))

    engine = PipelineEngine(stages, chunks=m, checkpoint=args.checkpoint, act_shape=act_shapes,
                            act_dtype=dtype, loss_fn=loss_fn if is_last else None, device=device,
                            skip_shapes={"skip": ((mb, S, E), dtype)}, watchdog=wd,
                            group=groups.channels if groups is not None else early_chan,
                            grad_divisor=dp, transport=args.transport)
    startup["stages_and_engine"] = time.perf_counter() - t_
    # explicit recompute (issued before each gradient wait, as the engine does)
    from mipipe.pipeline import checkpoint_stop_for
    sim_t, sim_busy = simulate_step([plan.stage_cost(g) * 3.0 / (1.0 + bwd_ratio) for g in range(pp * virtual)],
                                    pp, virtual, m, 2.0, deferred_w=0.5,
                                    checkpoint_stop=checkpoint_stop_for(args.checkpoint, m))

    g = torch.Generator(device="cpu").manual_seed(replica)  # each data-parallel replica its own shard
    tokens = torch.randint(0, V, (m, mb, S + 1), generator=g)
    inputs = [tokens[i, :, :S].to(device) for i in range(m)] if prank == 0 else None
    # every rank gets the targets: the vocabulary-split decoder's head stage needs them too
    targets = [tokens[i, :, 1:].contiguous().to(device) for i in range(m)]

    progress = os.environ.get("MIPIPE_BENCH_PROGRESS", "0") != "0" and rank == 0
    t_start = time.perf_counter()

    def mark(label):
        if wd is not None:
            wd.progress(label)
        if progress:  # a heartbeat for long rehearsals (host issue time, not GPU time)
            print(f"[bench {time.perf_counter() - t_start:8.1f} s] {label}", file=sys.stderr, flush=True)

    def train_step():
        opt.zero_grad()
        if dpg is not None:
            dpg.begin()
        try:
            st = engine.step(inputs, targets)
        except BaseException:
            if dpg is not None:
                dpg.abort()  # unhook the gradient buckets from the weight-gradient flush
            raise
        if dpg is not None:
            mark("data-parallel gradient all-reduce")
            dpg.finish()
        mark("grad-norm all-reduce")
        sq = opt.grad_sumsq()
        if pp > 1:
            dist.all_reduce(sq, group=groups.pipeline_group if groups is not None else None)
        opt.step(sq)
        return st

    armed = wd.watch("bench start") if wd is not None else contextlib.nullcontext()
    armed.__enter__()
    t_ = time.perf_counter()
    for k in range(args.warmup):
        mark(f"warmup step {k}")
        st = train_step()
    mark("synchronize after warmup")
    sync()
    if world > 1:
        dist.barrier()
    sync()
    startup["warmup_steps"] = time.perf_counter() - t_
    startup["total_before_timed_steps"] = time.perf_counter() - t_main
    tele = _telemetry(device) if on_gpu else None
    t0 = time.perf_counter()
    for k in range(args.steps):
        mark(f"timed step {k}")
        st = train_step()
    mark("synchronize after the timed steps")
    sync()
    if world > 1:
        dist.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    tele = tele.stop() if tele is not None else None
    ms = elapsed / max(args.steps, 1) * 1e3
    ms_t = torch.tensor([ms], device=device)
    if world > 1:
        dist.all_reduce(ms_t, op=dist.ReduceOp.MAX)
    ms = float(ms_t.item())
    peaks = _allgather([torch.cuda.max_memory_allocated(device) / 2**30 if on_gpu else 0.0], device, world)

    loss_val = None
    if is_last and st.loss is not None:
        loss_val = float(st.loss.item())

    # Bubble: one extra instrumented step, per-stage GPU busy time vs step time.
    bubble = None
    stage_busy = None
    if not args.no_bubble and on_gpu:
        mark("instrumented step")
        engine.measure = True
        sync()
        if world > 1:
            dist.barrier()
        st = train_step()
        sync()
        busy = torch.tensor([st.busy_ms, st.step_ms], device=device)
        if world > 1:
            gathered = [torch.zeros_like(busy) for _ in range(world)]
            dist.all_gather(gathered, busy)
        else:
            gathered = [busy]
        engine.measure = False
        step_ms = max(float(x[1]) for x in gathered)
        busys = [float(x[0]) for x in gathered]
        stage_busy = [round(b, 3) for b in busys]
        bubble = 100.0 * (1.0 - (sum(busys) / len(busys)) / step_ms) if step_ms > 0 else None

    if world > 1:
        lt = torch.tensor([loss_val if loss_val is not None else 0.0], device=device)
        dist.broadcast(lt, src=world - 1)
        loss_val = float(lt.item())

    comm = _comm_report(engine, device, world, local, on_gpu)
    # what the stage boundaries actually ran on ('auto' resolves in the engine; one rank: none)
    transport_used = getattr(engine, "transport", None) or "none (one stage)"
    teles = [tele]
    if world > 1:
        teles = [None] * world
        dist.all_gather_object(teles, tele)
    armed.__exit__(None, None, None)
    if wd is not None:
        wd.close()
    stop_n = checkpoint_stop_for(args.checkpoint, m)
    tokens_per_step = m * mb * S * dp
    value = tokens_per_step / (ms / 1e3)
    total_params = sum(int(x) for x in _allsum([n_params_local], device, world)) // dp  # one replica
    ref_match = matches_reference(cfg, args, m, mb)
    if rank == 0:
        out = {
            "metric": ("tokens/sec for 12-layer Transformer at PP=N (pipeline-parallel training)"
                       if cfg.name == "enc12_d4096" else f"tokens/sec for {cfg.name} at PP=N (pipeline-parallel training)"),
            "value": round(value, 1),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": _scaling_label(cfg, args, pp, m, mb),
            "vs_baseline": round(value / REF_TOKENS_PER_S[args.checkpoint], 2) if ref_match else None,
            "dtype": args.dtype,
            "data": "synthetic (random tokens, random-init weights)",
            "config": {
                "model": f"{cfg.name}: {cfg.num_layers}x {'causal decoder' if cfg.causal else 'TransformerEncoder'}Layer(d_model={E}, nhead={cfg.nhead}, "
                         f"dim_feedforward={cfg.dim_feedforward}, dropout={cfg.dropout}"
                         f"{'' if cfg.act_dropout is None else f' (after the activation: {cfg.act_dropout})'}, "
                         f"{cfg.activation}, "
                         f"{'pre' if cfg.norm_first else 'post'}-norm) + embedding/decoder V={V}",
                "params": total_params,
                "global_batch": m * mb * dp,
                "tokens_per_gpu_per_step": m * mb * dp * S // max(1, world),
                "micro_batch_note": ("enc12 default: 128 sequences at every N (chunks 4 x N), so every N carries "
                                     "the same tokens per GPU per step (weak scaling); N = 8 also runs config #3's "
                                     "'except_last' (see work_note and like_for_like)"
                                     if cfg.name == "enc12_d4096" and not args.micro_batch else None),
                "seq_len": S,
                "micro_batch": mb,
                "chunks": m,
                "checkpoint": args.checkpoint,
                "schedule": "gpipe" if virtual == 1 else f"gpipe-looping(v={virtual})",
                "virtual_chunks_per_rank": virtual,
                "vocab_split_decoder": plan.split_decoder,
                "skips": args.skips if not skip_pairs else f"{args.skips}: {len(skip_pairs)} long residuals, "
                                                           f"{len(engine.skip_routes)} cross-stage",
                "parallelism": f"pp{pp}" + (f"dp{dp}" if dp > 1 else ""),
                "impl": ("engine (one process per GPU, RCCL send/recv)" if transport_used == "rccl" else
                         "engine (one process per GPU, device-memory IPC links: DMA into the receiver's slots)"
                         if transport_used.startswith("ipc") else "engine (one process per GPU)"),
                "transport": transport_used,
                "transport_note": getattr(engine, "transport_note", None),
                "optimizer": "FlatAdam, " + ("overlapped with the next forward (side stream, forward-order chunks)"
                                             if opt._overlap is not None else "serial at the end of the step"),
                "shared_gpu": bool(args.shared_gpu),
                "balance": plan.balance,
                "stage_imbalance": round(plan.imbalance(), 3),
                "plan_costs": "measured (engine-context unit costs)" if cost_fn is not None else "analytic FLOPs",
                "plan_selection": plan_report,
            },
            "like_for_like": _like_for_like(cfg, args, pp, mb, unit_ms) if pp > 1 else None,
            "startup_s": {k: round(v, 3) for k, v in startup.items()},
            "bubble_pct": None if bubble is None else round(bubble, 2),
            "work_note": (f"checkpoint={args.checkpoint!r} re-runs the forward of {stop_n} of {m} micro-batches: "
                          f"~{1.0 + stop_n / m / 3.0:.2f}x the per-GPU compute of a 'never' step (the PP=1 "
                          f"default), which bounds weak-scaling efficiency against it")
            if stop_n else None,
            "bubble_theory_pct": round(100.0 * (pp - 1) / (virtual * m + pp - 1), 2),
            "bubble_gpipe_v1_pct": round(100.0 * (pp - 1) / (m + pp - 1), 2),
            "stage_busy_ms": stage_busy,
            "bubble_sim_pct": round(100.0 * (1 - sum(sim_busy) / len(sim_busy) / sim_t), 2),
            "loss": loss_val,
            "peak_hbm_gib_per_gpu": [round(x, 2) for x in peaks] if on_gpu else None,
            "baseline_note": _baseline_note(ref_match, args.checkpoint),
            "comm": comm,
            "telemetry": teles[0] if world == 1 else teles,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


def _telemetry(device):
    """GPU clock / power / temperature over the timed region (mipipe.utils.telemetry;
    firmware counters read on a side thread, no GPU work)."""
    from mipipe.utils.telemetry import GpuTelemetry

    return GpuTelemetry(device.index if device.index is not None else 0).start()


def _comm_report(engine, device, world, local, on_gpu):
    """What the job's communicators actually are, for a multi-GPU run to be
    checked against its own JSON: the default group's backend and size, the
    RCCL version, and per rank its device (index, PCI bus, UUID) and every
    pipeline channel it owns as its communicator reports it (backend,
    ``get_world_size``, whether the warm-up exchanged over it).  Collective."""
    me = {"rank": dist.get_rank() if world > 1 else 0, "local_rank": local, "device": str(device)}
    if on_gpu:
        props = torch.cuda.get_device_properties(device)
        me.update(device_index=device.index, pci_bus_id=int(getattr(props, "pci_bus_id", -1)),
                  uuid=str(getattr(props, "uuid", "")))
    chan = getattr(engine, "chan", None)
    if chan is not None and hasattr(chan, "comm_info"):
        me["channels"] = chan.comm_info()
        me["warmup_s"] = None if getattr(chan, "warmup_s", None) is None else round(chan.warmup_s, 3)
    else:
        me["channels"] = []
    ranks = [me]
    if world > 1:
        ranks = [None] * world
        dist.all_gather_object(ranks, me)
    rccl = None
    try:
        import torch.cuda.nccl as _nccl

        rccl = ".".join(str(x) for x in _nccl.version())
    except Exception:
        pass
    links = {c["dir"] for r in ranks for c in r["channels"]}
    warmed = {c["dir"] for r in ranks for c in r["channels"] if c["warmed"]}
    return {
        "backend": str(dist.get_backend()) if world > 1 else None,
        "world_size": dist.get_world_size() if world > 1 else 1,
        "rccl_version": rccl,
        "hip_version": torch.version.hip,
        "pipeline_links": len(links),
        "pipeline_links_warmed": len(warmed),
        "distinct_devices": len({(r.get("pci_bus_id"), r.get("uuid")) for r in ranks}) if on_gpu else None,
        "per_rank": ranks,
    }


def run_pipe(args) -> int:
    """``--impl pipe``: the single-process :class:`mipipe.Pipe` (the reference's
    execution model, ``/root/reference/pipeline.py:100-117``) over ``--gpus``
    devices of this process -- worker thread per device, per-(stage, chunk)
    copy streams, native peer copies.  Same model, data, optimizer and timing
    contract as the engine path; the pipeline is the GPipe clock schedule with
    one partition per device."""
    if int(os.environ.get("WORLD_SIZE", "1")) != 1:
        raise SystemExit("--impl pipe is one process driving every GPU: run it without torchrun")
    if args.dp != 1:
        raise SystemExit("--dp applies to the engine (--impl engine); a Pipe is one pipeline")
    import mipipe
    from mipipe import ops
    from mipipe.optim import FlatAdam
    from mipipe.parallel.stage import build_stage, plan_stages

    on_gpu = args.device == "cuda"
    n = args.gpus
    if on_gpu and torch.cuda.device_count() < n:
        raise SystemExit(f"--impl pipe --gpus {n}: only {torch.cuda.device_count()} GPU(s) visible")
    devices = [torch.device("cuda", d) for d in range(n)] if on_gpu else [torch.device("cpu")] * n
    if not on_gpu:
        args.dtype = "fp32"
    cfg = _config(args)
    S, V = cfg.seq_len, cfg.vocab
    m = args.chunks or (8 if (cfg.name == "gpt2_xl" and n == 8) else 4 * n)
    if args.checkpoint == "auto":
        args.checkpoint = "always" if cfg.name == "gpt2_xl" else ("except_last" if n == 8 else "never")
    mb = args.micro_batch or _default_micro_batch(cfg)
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    torch.manual_seed(1234)
    if args.pipe_balance:
        # the reference's partitioning (main.py:139-171): whole layers per partition, the
        # embedding with the first, the decoder (and a final norm) with the last
        from mipipe.models import build_lm_blocks

        layers = [int(v) for v in args.pipe_balance.split(",")]
        if sum(layers) != cfg.num_layers or min(layers) < 0:
            raise SystemExit(f"--pipe-balance {args.pipe_balance}: must sum to the {cfg.num_layers} layers")
        if n > 1 and len(layers) != n:
            raise SystemExit(f"--pipe-balance has {len(layers)} partitions for --gpus {n}")
        balance = [2 * L for L in layers]  # an attention and an MLP block per layer
        balance[0] += 1
        balance[-1] += 2 if cfg.norm_first else 1
        blocks = build_lm_blocks(cfg, device=devices[0], dtype=dtype)
        first = 0
        for j, size in enumerate(balance):
            for b in blocks[first:first + size]:
                b.to(devices[j if n > 1 else 0]).train()
            first += size
        params = [p for b in blocks for p in b.parameters()]
        opt = FlatAdam(params, lr=args.lr, max_grad_norm=args.clip, defer_wgrad=True)
        pipe = mipipe.Pipe(torch.nn.Sequential(*blocks), chunks=m, checkpoint=args.checkpoint, balance=balance,
                           copy_same_device=(n == 1 and len(balance) > 1 and args.pipe_boundary == "copy"),
                           stage_streams=args.pipe_stage_streams,
                           copy_streams=args.pipe_copy_streams if args.pipe_copy_streams != 0 else None)
        plan = None
    else:
        plan = plan_stages(cfg, n, 1, m, split_decoder=False)
        stages = [build_stage(cfg, plan, s, device=devices[s], dtype=dtype).train() for s in range(n)]
        params = [p for st_ in stages for p in st_.parameters()]
        # weight gradients deferred to one K-segmented GEMM per weight after the backward, as the engine does
        opt = FlatAdam(params, lr=args.lr, max_grad_norm=args.clip, defer_wgrad=True)
        pipe = mipipe.Pipe(torch.nn.Sequential(*stages), chunks=m, checkpoint=args.checkpoint)
    devices_used = list(dict.fromkeys(pipe.devices))

    g = torch.Generator(device="cpu").manual_seed(0)
    tokens = torch.randint(0, V, (m * mb, S + 1), generator=g)
    x = tokens[:, :S].contiguous().to(devices[0])
    t = tokens[:, 1:].contiguous().to(devices[-1])

    t = t.to(devices_used[-1])

    def sync():
        for d in dict.fromkeys(devices):
            if d.type == "cuda":
                torch.cuda.synchronize(d)

    def train_step():
        opt.zero_grad()
        out = pipe(x).local_value()
        loss = ops.cross_entropy(out.reshape(-1, V), t.reshape(-1))
        loss.backward()
        opt.step(opt.grad_sumsq())
        return loss

    for _ in range(args.warmup):
        loss = train_step()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = train_step()
    sync()
    ms = (time.perf_counter() - t0) / max(args.steps, 1) * 1e3
    value = m * mb * S / (ms / 1e3)
    ref_match = matches_reference(cfg, args, m, mb)
    peaks = [torch.cuda.max_memory_allocated(d) / 2**30 for d in devices_used] if on_gpu else None
    out = {
        "metric": ("tokens/sec for 12-layer Transformer at PP=N (pipeline-parallel training)"
                   if cfg.name == "enc12_d4096" else f"tokens/sec for {cfg.name} at PP=N (pipeline-parallel training)"),
        "value": round(value, 1), "unit": "tokens/s", "n_gpus": n, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": round(value / REF_TOKENS_PER_S[args.checkpoint], 2) if ref_match else None,
        "dtype": args.dtype, "data": "synthetic (random tokens, random-init weights)",
        "config": {
            "model": f"{cfg.name}: {cfg.num_layers} layers d_model={cfg.d_model} nhead={cfg.nhead} "
                     f"dim_feedforward={cfg.dim_feedforward} V={V}",
            "params": sum(p.numel() for p in params), "global_batch": m * mb, "seq_len": S, "micro_batch": mb,
            "chunks": m, "checkpoint": args.checkpoint, "schedule": "gpipe", "parallelism": f"pp{n}",
            "impl": "pipe (single process, worker thread per GPU, peer copies on copy streams)" + (
                f"; {len(pipe.partitions)} partitions on one GPU, device-to-device copies on the copy streams"
                if pipe.copy_same_device else ""),
            "balance": plan.balance if plan is not None else [len(p_) for p_ in pipe.partitions],
            "partitions": len(pipe.partitions),
        },
        "bubble_gpipe_v1_pct": round(100.0 * (n - 1) / (m + n - 1), 2),
        "loss": float(loss.item()),
        "peak_hbm_gib_per_gpu": [round(p, 2) for p in peaks] if peaks else None,
        "baseline_note": _baseline_note(ref_match, args.checkpoint),
    }
    print(json.dumps(out), flush=True)
    pipe.close()
    return 0


def _config(args):
    import dataclasses

    from mipipe.models import CONFIGS

    cfg = dataclasses.replace(CONFIGS[args.config])
    if args.seq_len:
        cfg.seq_len = args.seq_len
    if args.num_layers:
        cfg.num_layers = args.num_layers
    if getattr(args, "act_dropout", None) is not None:
        cfg.act_dropout = args.act_dropout
    return cfg


def _scaling_label(cfg, args, pp: int, m: int, mb: int) -> str:
    """``weak`` when the tokens per GPU per step are what the same flags give at
    N = 1 (default chunks 4 x PP, the same micro-batch at every N), ``strong``
    when the whole job's tokens are (an explicit --chunks, or GPT-2-XL's fixed
    config #4 chunks at PP = 8)."""
    m1 = args.chunks or 4
    n1 = m1 * (args.micro_batch or _default_micro_batch(cfg, 1))  # sequences per step at N = 1 (= per GPU)
    per_gpu, total = m * mb / pp, m * mb * args.dp
    if abs(per_gpu - n1) < 1e-9:
        return "weak"
    if abs(total - n1) < 1e-9:
        return "strong"
    # neither fixed (GPT-2-XL's config #4: chunks 8 at PP = 8): the closer one
    return "weak" if abs(per_gpu / n1 - 1) <= abs(total / n1 - 1) else "strong"


def _like_for_like(cfg, args, pp: int, mb: int, unit_ms):
    """The PP = 1 rate at THIS run's micro-batch and checkpoint mode, for reading
    an N > 1 value against N = 1 without mixing in a different micro-batch or
    recompute share: one GPU running every unit of the model per micro-batch,
    priced by the engine-context unit costs this run calibrated on its own GPUs
    (mipipe.parallel.calibrate: recompute, weight-gradient flush, optimizer and
    host issue included).  None where no costs were measured (analytic plan,
    --shared-gpu rehearsals, CPU)."""
    out = {"micro_batch": mb, "checkpoint": args.checkpoint, "pp1_tokens_per_s": None,
           "source": "no measured unit costs in this run (analytic plan)"}
    if unit_ms:
        from mipipe.parallel.calibrate import engine_unit_costs

        ms = sum(engine_unit_costs(cfg, unit_ms, False))  # one micro-batch through the whole model, one GPU
        if ms > 0:
            out["pp1_tokens_per_s"] = round(mb * cfg.seq_len / (ms / 1e3), 1)
            out["source"] = ("engine-context unit costs calibrated in this run (ms per micro-batch, summed over "
                             "the whole model): an estimate of the N = 1 rate at this micro-batch and checkpoint "
                             "mode, not a separate N = 1 run")
    return out


def _default_micro_batch(cfg, pp: int = 1) -> int:
    # ref_main: the reference's own micro-batch (batch 32 / chunks 4 = 8 sequences).
    # enc12_d4096: 128 x 128 = 16,384 tokens per GEMM, sized for 288 GB of HBM (89 GiB peak at
    # PP=1): +3.5 % for 64 over 32 (round 2), then +2.2 % for 128 over 64 at the power cap (the
    # optimizer, grad-norm and per-launch costs amortised over twice the tokens; same box,
    # interleaved: profiles/microbatch_sizing.txt).  The same 128 at every N, the full-node PP=8
    # run included (config #3, 'except_last', chunks 32), so the scaling curve is weak scaling --
    # the same tokens per GPU per step at every N -- although 64 predicts
    # 868k job tok/s there against 817k for 128 (profiles/plan_table_r5.txt; --micro-batch 64).
    # gpt2_xl: 18 x 1024 tokens -- the 1600-wide GEMM outputs (attention out-proj, fc2 and
    # the dgrads into the residual stream) are 7 256-wide tile columns, so M = 18,432 makes
    # 504 tiles = 98 % of two rounds of the 256 CUs (8 x 1024: 224 tiles, 88 % of one):
    # PP=1 54.6k (mb 8) -> 58.3k (mb 9) -> 59.8k tok/s (mb 18), 208 GiB peak with
    # checkpoint='always' (profiles/microbatch_sizing.txt).
    return {"gpt2_xl": 18, "tiny": 8, "ref_main": 8}.get(cfg.name, 128)


def _baseline_note(ref_match: bool, checkpoint: str) -> str:
    if ref_match:
        return (f"vs_baseline = value / the reference's derived {REF_TOKENS_PER_S[checkpoint]:.0f} tokens/s on the SAME "
                f"config (BASELINE.md: fp32, 16x d2048, batch 32x128, chunks 4, checkpoint={checkpoint!r}; the "
                f"reference used 2 GPUs, profiled); reference peak allocated per GPU "
                f"{REF_PEAK_MB[checkpoint]} MB")
    return ("vs_baseline = null: the reference published only its own config (BASELINE.md: fp32, 16x d2048, "
            "chunks 4, ~3.5k tokens/s on 2 GPUs); this run is a different model/precision. The like-for-like "
            "number is `bench.py --config ref_main --dtype fp32`")


def _allgather(vals, device, world):
    t = torch.tensor(vals, dtype=torch.float64, device=device)
    if world == 1:
        return [float(x) for x in t.tolist()]
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [float(x) for o in out for x in o.tolist()]


def _allsum(vals, device, world):
    t = torch.tensor(vals, dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t)
    return t.tolist()


if __name__ == "__main__":
    sys.exit(main())
