#!/usr/bin/env python3
"""Language-model training with ``mipipe.Pipe`` -- the reference driver, MI355X-native.

Mirrors ``/root/reference/main.py``: Encoder -> N x
TransformerEncoderLayer -> Decoder split evenly over the visible GPUs,
``Pipe(chunks=4, checkpoint=argv)``, cross-entropy, Adam + ``clip_grad_norm(0.5)``,
StepLR(gamma 0.95), optional ``torch.profiler`` (wait1/warmup1/active2) and
memory snapshot.  Differences, all deliberate:

* the blocks are mipipe's (HIP kernels for GEMM/attention/LN/dropout on GPU);
* ``--flat-adam`` (default on GPU) uses the fused flat-buffer Adam whose clip
  coefficient never leaves the device; ``--torch-adam`` uses ``torch.optim.Adam``
  + ``clip_grad_norm_`` exactly like the reference;
* data is a local text file (``--train-file``) tokenised with the
  basic_english tokenizer, or a synthetic WikiText-2-sized stream (no network);
* with a single GPU every partition lives on ``cuda:0`` (still a real pipeline:
  separate copy streams, clock-cycle schedule); on CPU it runs the same code.

    python examples/train_lm.py never --config tiny --batches 4
    python examples/train_lm.py except_last --config ref_main --profile-dir /tmp/prof
"""
from __future__ import annotations

import argparse
import math
import os
import sys
import time

import torch
from torch import nn

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import mipipe  # noqa: E402
from mipipe.models import CONFIGS, build_lm_blocks  # noqa: E402
from mipipe.ops import cross_entropy  # noqa: E402
from mipipe.optim import FlatAdam  # noqa: E402
from mipipe.utils import data as D  # noqa: E402
from mipipe.utils import profiling as P  # noqa: E402


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("checkpoint", nargs="?", default="except_last", choices=["never", "except_last", "always"])
    ap.add_argument("--config", default="ref_main", choices=sorted(CONFIGS))
    ap.add_argument("--layers", type=int, default=None, help="override number of layers")
    ap.add_argument("--chunks", type=int, default=4)
    ap.add_argument("--partitions", type=int, default=None, help="pipeline stages (default: #GPUs, 2 on CPU)")
    ap.add_argument("--batch-size", type=int, default=20)
    ap.add_argument("--bptt", type=int, default=None)
    ap.add_argument("--batches", type=int, default=8)
    ap.add_argument("--lr", type=float, default=1e-3, help="main.py uses 5.0 (diverges with Adam)")
    ap.add_argument("--clip", type=float, default=0.5)
    ap.add_argument("--dtype", default=None, choices=["fp32", "bf16"])
    ap.add_argument("--train-file", default=None)
    ap.add_argument("--torch-adam", action="store_true")
    ap.add_argument("--profile-dir", default=None)
    ap.add_argument("--memory-snapshot", default=None)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--save", default=None, help="write the training state (weights, optimizer, RNG) here at the end")
    ap.add_argument("--resume", default=None, help="continue from a --save file (same model and partition)")
    return ap.parse_args(argv)


def build_pipe(cfg, nparts: int, devices, dtype, chunks: int, checkpoint: str) -> mipipe.Pipe:
    """Even layer split as main.py:139-158 (encoder on the first, decoder on the last)."""
    blocks = build_lm_blocks(cfg, dtype=dtype)
    enc, body, tail = blocks[0], blocks[1:-1], blocks[-1]
    per = (len(body) + nparts - 1) // nparts
    stages = []
    for s in range(nparts):
        part = body[s * per:(s + 1) * per]
        if s == 0:
            part = [enc] + part
        if s == nparts - 1:
            part = part + [tail]
        stages.append(nn.Sequential(*part).to(devices[s]))
    return mipipe.Pipe(nn.Sequential(*stages), chunks=chunks, checkpoint=checkpoint)


def main(argv=None) -> int:
    args = parse(argv)
    torch.manual_seed(args.seed)
    cfg = CONFIGS[args.config]
    if args.layers is not None:
        from dataclasses import replace

        cfg = replace(cfg, num_layers=args.layers)
    bptt = args.bptt or cfg.seq_len
    on_gpu = torch.cuda.is_available()
    ngpu = torch.cuda.device_count() if on_gpu else 0
    nparts = args.partitions or (ngpu if ngpu > 1 else 2)
    devices = [torch.device("cuda", i % ngpu) for i in range(nparts)] if on_gpu else [torch.device("cpu")] * nparts
    dtype = {"fp32": torch.float32, "bf16": torch.bfloat16}[args.dtype or ("bf16" if on_gpu else "fp32")]

    # ---- data (main.py:76-113) ----
    if args.train_file:
        vocab = D.build_vocab(map(D.basic_english, D.read_lines(args.train_file)))
        ids = D.data_process(D.read_lines(args.train_file), vocab)
        from dataclasses import replace

        cfg = replace(cfg, vocab=len(vocab))
    else:
        ids = D.synthetic_corpus(args.batch_size * bptt * (args.batches + 1) + 1, cfg.vocab, seed=args.seed)
    train_data = D.batchify(ids, args.batch_size)

    model = build_pipe(cfg, nparts, devices, dtype, args.chunks, args.checkpoint)
    total = sum(p.numel() for p in model.parameters())
    print(f"Total parameters in model: {total:,}")

    if args.torch_adam or not on_gpu:
        opt = torch.optim.Adam(model.parameters(), lr=args.lr)
        flat = None
    else:
        flat = FlatAdam(model.parameters(), lr=args.lr, max_grad_norm=args.clip, defer_wgrad=True)
        opt = None
    lr = args.lr
    out_dev = devices[-1]
    start = 0
    if args.resume:
        from mipipe.utils.checkpoint_io import load_training_state

        meta = load_training_state(args.resume, model.named_parameters(), flat if flat is not None else opt)
        start = int(meta["step"])
        lr = flat.lr if flat is not None else opt.param_groups[0]["lr"]
        print(f"resumed from {args.resume} at batch {start}")

    def step(data, targets):
        nonlocal lr
        if flat is not None:
            flat.zero_grad()
        else:
            opt.zero_grad()
        output = model(data).local_value()
        loss = cross_entropy(output.reshape(-1, output.size(-1)), targets.to(out_dev))
        loss.backward()
        if flat is not None:
            flat.step()
        else:
            torch.nn.utils.clip_grad_norm_(model.parameters(), args.clip)
            opt.step()
        return loss

    if args.memory_snapshot and on_gpu:
        P.record_memory_history(True)
    P.reset_peak_memory(set(devices))
    prof = P.torch_profiler(os.path.join(args.profile_dir, args.checkpoint)) if args.profile_dir else None
    if prof is not None:
        prof.__enter__()
    model.train()
    t0 = time.time()
    total_loss, ntok, nbatches = 0.0, 0, 0
    try:
        for batch, (data, targets) in enumerate(D.iter_batches(train_data, bptt, args.batches)):
            if batch < start:
                continue
            if prof is not None:
                prof.step()
            data = data.to(devices[0])
            loss = step(data, targets)
            lv = loss.item()
            total_loss += lv
            nbatches += 1
            ntok += data.numel()
            print(f"| batch {batch:3d} | lr {lr:.3g} | loss {lv:6.3f} | ppl {math.exp(min(lv, 20)):9.2f}")
    finally:
        if prof is not None:
            prof.__exit__(None, None, None)
    if on_gpu:
        torch.cuda.synchronize()
    elapsed = time.time() - t0
    # StepLR(step_size=1, gamma=0.95) per epoch, as main.py:184.
    lr *= 0.95
    if flat is not None:
        flat.lr = lr
    else:
        for g in opt.param_groups:
            g["lr"] = lr
    print(f"tokens/s {ntok / elapsed:.1f} over {elapsed:.2f}s; mean loss {total_loss / max(1, nbatches):.3f}")
    for d, r in P.memory_report(set(devices)).items():
        print(f"{d}: peak allocated {r['peak_allocated_mb']:.0f} MB, peak reserved {r['peak_reserved_mb']:.0f} MB")
    if args.memory_snapshot and on_gpu:
        P.dump_memory_snapshot(args.memory_snapshot)
        P.record_memory_history(False)
    if args.save:
        from mipipe.utils.checkpoint_io import save_training_state

        save_training_state(args.save, model.named_parameters(), flat if flat is not None else opt,
                            step=batch + 1, extra={"config": args.config, "checkpoint": args.checkpoint})
        print(f"saved the training state to {args.save}")
    model.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
