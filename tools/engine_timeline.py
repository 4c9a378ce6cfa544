"""Per-rank pipeline timeline from rocprofv3 databases of a PipelineEngine run.

Record (one database per process; the engine labels every action with roctx,
see ``PipelineEngine.step``)::

    rocprofv3 --kernel-trace --marker-trace -d gpurun_out/tl -o rank -- python bench.py --steps 2 --warmup 1
    torchrun ... (each rank under rocprofv3 the same way)

Report::

    python tools/engine_timeline.py gpurun_out/tl/**/*_results.db [--step -1]

For the chosen ``engine step`` range (default: the last one of each rank) the
window runs from the earliest step start (host clock, shared by every process
of a node) to the last kernel end of the step on any rank.  Per rank:

* ``busy``     -- union of the rank's kernel intervals in the window (GPU time),
  EXCLUDING the runtime's stream-operation kernels: on this ROCm a
  ``hipStreamWaitValue64`` is dispatched as ``__amd_rocclr_streamOpsWait``, a
  kernel that spins on a CU until the flag flips, and a
  ``hipStreamWriteValue64`` as ``__amd_rocclr_streamOpsWrite`` -- counting the
  spin as work understated the bubble;
* ``spin``     -- union of those stream-op kernels (ms) and their counts
  (``waits/writes`` per step), reported separately, with the runtime's copy
  kernels (``copy k.``, ``__amd_rocclr_copyBuffer*``: a copy the runtime ran
  on the CUs) and, with a memory-copy trace, the copies the DMA engines ran
  (``DMA cp.``);
* ``lead``     -- window start -> the rank's first kernel (fill: waiting for
  upstream activations);
* ``tail``     -- the rank's last kernel -> window end (drain);
* ``bubble``   -- 1 - busy / window;
* host-side time in each action kind (``F``, ``B``, ``recompute``, ``wait
  recv act``, ``wait recv grad``, ``wgrad flush``, ``wait sends``): where the
  rank's launch thread spent the step.

The mean bubble over ranks is the measured counterpart of the
``bubble_sim_pct`` / ``bubble_theory_pct`` bench.py prints.
"""
from __future__ import annotations

import argparse
import glob
import json
import re
import sqlite3
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


def _clip(iv: List[Interval], lo: int, hi: int) -> List[Interval]:
    return [(max(a, lo), min(b, hi)) for a, b in iv if b > lo and a < hi]


def _total(iv: List[Interval]) -> int:
    return sum(b - a for a, b in iv)


_KIND = re.compile(r"^(F|B|recompute|wait recv act|wait recv grad|post recvs|wgrad flush|wait sends)")


def load(db: str):
    """(label, start, end) of the roctx ranges and (start, end) of the kernels.
    rocpd keeps a roctx range's text in ``extdata`` ({"message": ...}); the
    ``name`` column is the API (``roctxThreadRangeA``)."""
    con = sqlite3.connect(db)
    regions = []
    for name, ext, a, b in con.execute("select name, extdata, start, end from regions"):
        try:
            label = json.loads(ext or "{}").get("message") or name
        except ValueError:
            label = name
        regions.append((label, a, b))
    kernels = con.execute("select start, end, name from kernels order by start").fetchall()
    try:  # recorded with --memory-copy-trace (tools/profile_ranks.py --copy-trace)
        copies = con.execute("select start, end, size from memory_copies order by start").fetchall()
    except sqlite3.Error:
        copies = []
    return regions, kernels, copies


_STREAM_OP = "__amd_rocclr_streamOps"
_COPY_KERNEL = "__amd_rocclr_copy"


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("dbs", nargs="+")
    ap.add_argument("--step", type=int, default=-1, help="which 'engine step' range of each rank (default last)")
    ap.add_argument("--end-kernel", default="sumsq_partial",
                    help="a step's GPU work ends where the first kernel whose name contains this starts (the "
                         "optimizer's grad-norm pass after PipelineEngine.step; '' = up to the next step's start "
                         "or the last kernel)")
    args = ap.parse_args()
    paths = sorted({p for pat in args.dbs for p in glob.glob(pat, recursive=True)})
    ranks = []
    for p in paths:
        regions, kernels, dma = load(p)
        steps = sorted((a, b) for n, a, b in regions if n == "engine step")
        if not steps:
            print(f"{p}: no 'engine step' ranges (run with --marker-trace)")
            continue
        s0, s1 = steps[args.step]
        nxt = [a for a, _ in steps if a > s0]
        limit = nxt[0] if nxt else max(b for _, b, _ in kernels)
        if args.end_kernel:
            # the GPU runs behind the host: a step's kernels end where the work queued
            # after it (the optimizer) begins, not at the next step's host start
            ends = [a for a, _, n in kernels if a >= s0 and args.end_kernel in n]
            if ends:
                limit = ends[0]
        # kernels of this step: started after the step began, before the limit
        ks = [(a, b) for a, b, n in kernels if s0 <= a < limit and _STREAM_OP not in n]
        ops = [(a, b, n) for a, b, n in kernels if s0 <= a < limit and _STREAM_OP in n]
        copies = sum(1 for a, _, n in kernels if s0 <= a < limit and _COPY_KERNEL in n)
        dmas = [(a, b, z) for a, b, z in dma if s0 <= a < limit]
        acts = [(n, a, b) for n, a, b in regions if s0 <= a and b <= s1 and n != "engine step"]
        ranks.append((p, s0, s1, ks, acts, ops, copies, dmas))
    if not ranks:
        return
    w0 = min(r[1] for r in ranks)
    w1 = max(max((b for _, b in r[3]), default=r[2]) for r in ranks)
    span = w1 - w0
    print(f"# window {span / 1e6:.3f} ms over {len(ranks)} rank(s)")
    print(f"{'rank db':<40} {'busy ms':>8} {'lead ms':>8} {'tail ms':>8} {'bubble':>7} {'spin ms':>8} "
          f"{'waits/writes':>12} {'copy k.':>7} {'DMA cp.':>7}   host ms per action kind")
    bubbles = []
    for p, s0, s1, ks, acts, ops, copies, dmas in ranks:
        busy = _union(_clip(ks, w0, w1))
        b = _total(busy)
        lead = (busy[0][0] - w0) if busy else span
        tail = (w1 - busy[-1][1]) if busy else span
        bub = 1 - b / span if span else 0.0
        bubbles.append(bub)
        kinds: Dict[str, int] = defaultdict(int)
        for n, a, e in acts:
            m = _KIND.match(n)
            if m:
                kinds[m.group(1)] += e - a
        host = ", ".join(f"{k} {v / 1e6:.2f}" for k, v in sorted(kinds.items(), key=lambda kv: -kv[1]))
        name = p if len(p) <= 40 else "..." + p[-37:]
        spin = _total(_union(_clip([(a, e) for a, e, _ in ops], w0, w1)))
        nw = sum(1 for _, _, n in ops if "Wait" in n)
        nwr = len(ops) - nw
        print(f"{name:<40} {b / 1e6:8.2f} {lead / 1e6:8.2f} {tail / 1e6:8.2f} {100 * bub:6.1f}% {spin / 1e6:8.2f} "
              f"{f'{nw}/{nwr}':>12} {copies:7d} {len(dmas):7d}   {host}")
    print(f"mean bubble {100 * sum(bubbles) / len(bubbles):.2f}% (stream-op spin kernels excluded from busy)")
    if len(ranks) > 1:
        # ranks sharing one GPU (--shared-gpu): how full the device was
        dev = _union([iv for r in ranks for iv in _clip(r[3], w0, w1)])
        print(f"union of every rank's kernels: {_total(dev) / 1e6:.2f} ms = {100 * _total(dev) / span:.1f}% of the "
              f"window (the device's busy share when the ranks share one GPU)")


if __name__ == "__main__":
    main()
