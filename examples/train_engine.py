#!/usr/bin/env python3
"""LM training with the multi-process pipeline engine: PP x DP ranks, save / resume.

The scale-out counterpart of ``examples/train_lm.py`` (which drives the
single-process ``mipipe.Pipe``, as the reference's ``main.py`` does): one
process per GPU, launched by torchrun; ``--pp`` pipeline stages connected by
RCCL send/recv, ``--dp`` replicas of that pipeline averaging their gradients
(``mipipe.parallel.data_parallel``); FlatAdam with ``clip_grad_norm`` over the
pipeline; per-rank training-state files (``mipipe.utils.checkpoint_io``).

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/train_engine.py \\
        --config enc12_d4096 --pp 4 --dp 2 --steps 100 --save-dir /ckpt
    torchrun ... examples/train_engine.py ... --resume-dir /ckpt --steps 200
    # CPU plumbing check (gloo, fp32):
    torchrun --nproc-per-node 2 --master-addr 127.0.0.1 examples/train_engine.py --device cpu --config tiny

Data: a local text file (``--train-file``: basic_english tokens, batchified as
``main.py:92-113``) or a synthetic Zipf stream (no network).  Each step takes
the next ``seq_len + 1`` rows of the batchified stream; replica ``d`` trains on
its slice of the batch columns, micro-batches are consecutive column groups.
"""
from __future__ import annotations

import argparse
import dataclasses
import os
import sys
import time

# before HIP initialises (see bench.py / profiles/hw_queue_sharing.txt)
if int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 16:
    os.environ["GPU_MAX_HW_QUEUES"] = "16"

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from mipipe import ops  # noqa: E402
from mipipe.models import CONFIGS  # noqa: E402
from mipipe.optim import FlatAdam  # noqa: E402
from mipipe.parallel import PipelineEngine  # noqa: E402
from mipipe.parallel.data_parallel import DataParallelGrads, make_pp_dp_groups  # noqa: E402
from mipipe.parallel.stage import build_stage, plan_stages, stage_input_shape  # noqa: E402
from mipipe.utils import data as D  # noqa: E402
from mipipe.utils.checkpoint_io import load_training_state, rank_path, save_training_state  # noqa: E402


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="tiny", choices=sorted(CONFIGS))
    ap.add_argument("--layers", type=int, default=None)
    ap.add_argument("--pp", type=int, default=None, help="pipeline stages (default: world / dp)")
    ap.add_argument("--dp", type=int, default=1, help="data-parallel replicas of the pipeline")
    ap.add_argument("--chunks", type=int, default=4, help="micro-batches per step and replica")
    ap.add_argument("--micro-batch", type=int, default=2, help="sequences per micro-batch")
    ap.add_argument("--checkpoint", default="except_last", choices=["never", "except_last", "always"])
    ap.add_argument("--steps", type=int, default=8, help="train until this global step")
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--clip", type=float, default=0.5)
    ap.add_argument("--train-file", default=None)
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"])
    ap.add_argument("--save-dir", default=None, help="write one training-state file per pipeline rank at the end")
    ap.add_argument("--resume-dir", default=None, help="continue from --save-dir files (same pp and model)")
    ap.add_argument("--seed", type=int, default=0)
    return ap.parse_args(argv)


def main(argv=None) -> int:
    args = parse(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    on_gpu = args.device == "cuda"
    if on_gpu:
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
        dist.init_process_group("nccl", device_id=device)
    else:
        device = torch.device("cpu")
        dist.init_process_group("gloo")
    dtype = torch.bfloat16 if on_gpu else torch.float32
    dp = args.dp
    pp = args.pp or world // dp
    groups = make_pp_dp_groups(pp, dp)
    cfg = CONFIGS[args.config]
    if args.layers:
        cfg = dataclasses.replace(cfg, num_layers=args.layers)

    # ---- data: every rank builds the same stream and takes its replica's columns
    m, mb, S = args.chunks, args.micro_batch, cfg.seq_len
    cols = dp * m * mb
    if args.train_file:
        vocab = D.build_vocab(map(D.basic_english, D.read_lines(args.train_file)))
        ids = D.data_process(D.read_lines(args.train_file), vocab)
        cfg = dataclasses.replace(cfg, vocab=len(vocab))
    else:
        # a fixed-size stream (not sized by --steps: a resumed run must see the same tokens), wrapped around
        ids = D.synthetic_corpus(cols * (S + 1) * 64 + 1, min(cfg.vocab, 28782), seed=args.seed)
    stream = D.batchify(ids, cols)  # [rows, cols]
    rows_per_step = S + 1

    def batch(step: int):
        i = (step * rows_per_step) % max(1, stream.size(0) - rows_per_step)
        win = stream[i: i + S + 1].t().contiguous()  # [cols, S + 1], batch-first
        mine = win[groups.replica * m * mb:(groups.replica + 1) * m * mb]
        xs = [mine[j * mb:(j + 1) * mb, :S].to(device) for j in range(m)]
        ts = [mine[j * mb:(j + 1) * mb, 1:].contiguous().to(device) for j in range(m)]
        return xs, ts

    # ---- this rank's stage (same initial weights in every replica)
    plan = plan_stages(cfg, pp, 1, m)
    torch.manual_seed(1234 + groups.stage)
    stage = build_stage(cfg, plan, groups.stage, device=device, dtype=dtype).train()
    opt = FlatAdam(stage.parameters(), lr=args.lr, max_grad_norm=args.clip)
    dpg = DataParallelGrads(opt, groups.dp_group) if dp > 1 else None
    last = groups.stage == pp - 1
    engine = PipelineEngine(stage, chunks=m, checkpoint=args.checkpoint,
                            act_shape=stage_input_shape(cfg, plan, groups.stage, mb), act_dtype=dtype,
                            loss_fn=(lambda y, t: ops.cross_entropy(y.reshape(-1, cfg.vocab), t.reshape(-1)))
                            if last else None,
                            device=device, group=groups.channels, grad_divisor=dp)
    start = 0
    if args.resume_dir:
        meta = load_training_state(rank_path(args.resume_dir, groups.stage), stage.named_parameters(), opt)
        start = int(meta["step"])
    reporter = rank == world - 1  # last stage of the last replica
    t0 = time.perf_counter()
    for step in range(start, args.steps):
        xs, ts = batch(step)
        opt.zero_grad()
        if dpg is not None:
            dpg.begin()
        try:
            st = engine.step(xs if groups.stage == 0 else None, ts)
        except BaseException:
            if dpg is not None:
                dpg.abort()  # unhook the gradient buckets from the weight-gradient flush
            raise
        if dpg is not None:
            dpg.finish()
        sq = opt.grad_sumsq()
        if pp > 1:
            dist.all_reduce(sq, group=groups.pipeline_group)
        opt.step(sq)
        if reporter and st.loss is not None:
            print(f"| step {step:4d} | loss {float(st.loss):7.4f} | grad-norm {float(sq.sqrt()):8.4f} |", flush=True)
    if on_gpu:
        torch.cuda.synchronize()
    if reporter:
        done = max(0, args.steps - start)
        dt = time.perf_counter() - t0
        print(f"{done} steps in {dt:.2f}s, {done * dp * m * mb * S / max(dt, 1e-9):.0f} tokens/s", flush=True)
    if args.save_dir and groups.replica == 0:  # replicas hold identical state
        save_training_state(rank_path(args.save_dir, groups.stage), stage.named_parameters(), opt,
                            step=args.steps, extra={"config": args.config, "pp": pp})
    dist.barrier()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
