"""Stage-transport timeline of a multi-partition Pipe on ONE MI355X.

``run``: a ``Pipe`` with P partitions of enc12_d4096 layers (bf16, our kernels)
all on cuda:0 (``balance=``), real device-to-device boundary copies on the copy
streams (``copy_same_device=True``, the native ``peer_copy`` path), a few
training steps.  Meant to run under rocprofv3::

    rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/pipe_trace -o run -- \\
        python tools/pipe_overlap_trace.py run 4 8

``analyze``: reads the rocpd database rocprofv3 writes and reports, for the
last step: per-stream busy time, how much of the boundary-copy time ran while
compute kernels were running on OTHER streams, and pairwise stage overlap
(time two stage streams were busy at once)::

    python tools/pipe_overlap_trace.py analyze gpurun_out/pipe_trace/<host>/<pid>_results.db
"""
from __future__ import annotations

import sqlite3
import sys
from collections import defaultdict
from typing import Dict, List, Tuple

Interval = Tuple[int, int]


def _union(iv: List[Interval]) -> List[Interval]:
    out: List[Interval] = []
    for a, b in sorted(iv):
        if out and a <= out[-1][1]:
            out[-1] = (out[-1][0], max(out[-1][1], b))
        else:
            out.append((a, b))
    return out


def _total(iv: List[Interval]) -> int:
    return sum(b - a for a, b in iv)


def _intersect(x: List[Interval], y: List[Interval]) -> int:
    i = j = tot = 0
    while i < len(x) and j < len(y):
        a, b = max(x[i][0], y[j][0]), min(x[i][1], y[j][1])
        if a < b:
            tot += b - a
        if x[i][1] < y[j][1]:
            i += 1
        else:
            j += 1
    return tot


def _cols(con, table: str) -> List[str]:
    return [r[1] for r in con.execute(f"pragma table_info({table})")]


def _pick(cols: List[str], *names: str) -> str:
    for n in names:
        if n in cols:
            return n
    raise KeyError(f"none of {names} in {cols}")


def analyze(db: str, window_ns: int = 0) -> None:
    con = sqlite3.connect(db)
    tables = [r[0] for r in con.execute("select name from sqlite_master where type in ('table', 'view')")]
    kc = _cols(con, "kernels")
    name_c = _pick(kc, "name", "kernel_name")
    sid_c = _pick(kc, "stream_id", "queue_id")
    kern = con.execute(f"select {name_c}, {sid_c}, start, end from kernels").fetchall()
    copies: List[Tuple[str, int, int, int]] = []
    if "memory_copies" in tables:
        mc = _cols(con, "memory_copies")
        msid = _pick(mc, "stream_id", "queue_id")
        mname = next((c for c in ("name", "direction", "kind") if c in mc), None)
        sel = f"{mname}, " if mname else "'copy', "
        copies = [(str(n), s, a, b) for n, s, a, b in
                  con.execute(f"select {sel}{msid}, start, end from memory_copies").fetchall()]
    # blit copies (our kernel or HIP's own copy kernels) are copies too
    is_copy = lambda n: ("blit16" in n) or ("copyBuffer" in n) or ("__amd_rocclr_copy" in n)
    copies += [(n, s, a, b) for n, s, a, b in kern if is_copy(n)]
    compute = [(n, s, a, b) for n, s, a, b in kern if not is_copy(n) and "sleep" not in n]
    if not compute:
        print("no compute kernels in", db)
        return
    end = max(b for _, _, _, b in compute)
    start = end - window_ns if window_ns else min(a for _, _, a, _ in compute)
    compute = [c for c in compute if c[2] >= start]
    copies = [c for c in copies if c[2] >= start]
    by_stream: Dict[int, List[Interval]] = defaultdict(list)
    for _, s, a, b in compute:
        by_stream[s].append((a, b))
    busy = {s: _union(iv) for s, iv in by_stream.items()}
    span = end - start
    print(f"# window {span / 1e6:.2f} ms, {len(compute)} compute kernels, {len(copies)} copies")
    print(f"{'stream':>8} {'kernels':>8} {'busy ms':>9} {'busy %':>7}")
    for s in sorted(busy, key=lambda s: -_total(busy[s])):
        print(f"{s:>8} {len(by_stream[s]):>8} {_total(busy[s]) / 1e6:9.2f} {100 * _total(busy[s]) / span:6.1f}%")
    any_compute = _union([iv for ivs in busy.values() for iv in ivs])
    print(f"device busy (any stream): {_total(any_compute) / 1e6:.2f} ms "
          f"({100 * _total(any_compute) / span:.1f}% of the window)")
    top = sorted(busy, key=lambda s: -_total(busy[s]))[:8]
    print("pairwise overlap (ms of both streams busy at once):")
    for i, s in enumerate(top):
        for t in top[i + 1:]:
            ov = _intersect(busy[s], busy[t])
            if ov:
                print(f"  stream {s} & {t}: {ov / 1e6:.2f} ms")
    if copies:
        tot = ov_tot = 0
        for _, s, a, b in copies:
            others = _union([iv for t, ivs in busy.items() if t != s for iv in ivs])
            tot += b - a
            ov_tot += _intersect([(a, b)], others)
        print(f"boundary copies: {len(copies)}, {tot / 1e6:.3f} ms total, "
              f"{100 * ov_tot / max(tot, 1):.1f}% of it overlapped by compute on other streams")
        names = defaultdict(int)
        for n, _, _, _ in copies:
            names[n[:60]] += 1
        print("copy kinds:", dict(names))


def run(parts: int, chunks: int, steps: int = 3) -> None:
    import dataclasses
    import os
    import time

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch

    from mipipe import Pipe, ops
    from mipipe.models import CONFIGS, build_lm_blocks
    from mipipe.optim import FlatAdam

    dev = torch.device("cuda", 0)
    cfg = dataclasses.replace(CONFIGS["enc12_d4096"], num_layers=parts)
    torch.manual_seed(0)
    blocks = build_lm_blocks(cfg, dtype=torch.bfloat16)  # encoder, 2 blocks per layer, decoder
    n = len(blocks)
    base, extra = divmod(n, parts)
    balance = [base + (1 if k < extra else 0) for k in range(parts)]
    model = torch.nn.Sequential(*blocks).to(dev).train()
    opt = FlatAdam(model.parameters(), lr=1e-4)
    pipe = Pipe(model, chunks=chunks, checkpoint="except_last", balance=balance, copy_same_device=True,
                stage_streams="dedicated",
                return_rref=False)
    mb = 8
    tok = torch.randint(0, cfg.vocab, (chunks * mb, cfg.seq_len + 1))
    x, t = tok[:, :-1].to(dev), tok[:, 1:].contiguous().to(dev)
    for s in range(steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        opt.zero_grad()
        loss = ops.cross_entropy(pipe(x).reshape(-1, cfg.vocab), t.reshape(-1))
        loss.backward()
        opt.step()
        torch.cuda.synchronize()
        print(f"step {s}: {1e3 * (time.perf_counter() - t0):.1f} ms loss {float(loss):.3f} "
              f"partitions {len(pipe.partitions)} balance {balance}", flush=True)
    pipe.close()


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(int(sys.argv[2]) if len(sys.argv) > 2 else 4, int(sys.argv[3]) if len(sys.argv) > 3 else 8)
    else:
        analyze(sys.argv[2], int(float(sys.argv[3]) * 1e6) if len(sys.argv) > 3 else 0)
