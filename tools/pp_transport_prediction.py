#!/usr/bin/env python3
"""PP=8 job predictions WITH the stage transport's measured cost (VERDICT r4
item 1: every earlier PP=2/4/8 prediction assumed transfers free).

Inputs, all measured on MI355X and committed:
* per-rank GPU work of every rank of the PP=8 plans (profiles/pp8_ranks_r3.txt:
  each rank emulated through the real engine over a loopback channel);
* the cost of an RCCL receive kernel resident beside the compute
  (profiles/cu_hold_r5.txt: +33.9 % enc12, +19.6 % GPT-2-XL step time for ONE
  resident block, no more for 16);
* the IPC link's one-GPU latencies (profiles/ipc_stream_ordered.txt and
  profiles/ipc_vs_gloo_one_gpu.txt: ~150 us of cross-stream event latency for
  the copy-stream engines).

Unknown on a one-GPU box: the xGMI copy bandwidth between two MI355X.  The hop
latency of a message is priced as 150 us + bytes / BW for BW = 50 and 100 GB/s
(SDMA copy over one link), and each transport's step is simulated with
mipipe.parallel.stage.simulate_step -- the dependency of stage j+1's micro-batch
i on stage j's output arrives one hop later; the DMA engines take no compute
from either rank, so only the fill / drain see the hops.

    python tools/pp_transport_prediction.py > profiles/pp8_transport_prediction_r5.txt
"""
from __future__ import annotations

import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mipipe.parallel.stage import simulate_step  # noqa: E402
from mipipe.pipeline import checkpoint_stop_for  # noqa: E402

CASES = [
    # name, section header in pp8_ranks_r3.txt, chunks, micro-batch tokens, d_model, checkpoint, v, cu-hold cost, PP=1 tok/s
    ("enc12 except_last (config #3)", "## enc12_d4096, PP=8, chunks 32, micro-batch 64 x 128, except_last",
     32, 64 * 128, 4096, "except_last", 2, 0.339, 147.5e3),
    ("GPT-2-XL always (config #4)", "## GPT-2-XL, PP=8, chunks 8, micro-batch 18 x 1024, always",
     8, 18 * 1024, 1600, "always", 2, 0.196, 64.5e3),
]


def rank_walls(text: str, header: str):
    sec = text.split(header, 1)[1].split("\n## ", 1)[0]
    return [float(x) for x in re.findall(r"^wall ([\d.]+) ms/step", sec, re.M)]


def main() -> int:
    text = open(os.path.join(ROOT, "profiles", "pp8_ranks_r3.txt")).read()
    print("# PP=8 predictions with the stage transport priced in (tools/pp_transport_prediction.py).")
    print("# Per-rank work: profiles/pp8_ranks_r3.txt (every rank of the bench's PP=8 plan, emulated on one MI355X).")
    print("# Stage costs per virtual stage = rank wall / v (the ranks are balanced to within a few %); backward = 2x")
    print("# forward with the recompute modelled explicitly; weight gradients deferred (1/3 of the backward).")
    print("# RCCL: every rank's compute x (1 + the measured one-block cost, profiles/cu_hold_r5.txt), hop 0.1 ms.")
    print("# IPC (auto): compute unchanged (copies on the DMA engines, waits in the command processor), hop = 0.15 ms")
    print("# event latency + message / xGMI copy bandwidth (not measurable on a one-GPU box: 50 and 100 GB/s shown).")
    for name, header, m, tokens, d, ckpt, v, hold, pp1 in CASES:
        walls = rank_walls(text, header)
        if len(walls) != 8:
            print(f"# {name}: could not read 8 rank walls ({len(walls)})")
            continue
        msg_bytes = tokens * d * 2
        stop = checkpoint_stop_for(ckpt, m)
        # per-rank wall = its vstages' work; simulate_step wants forward + 2 x forward per vstage (no recompute)
        rec = stop / m  # recomputed forwards per micro-batch, as a fraction of one forward
        per_v = []
        for c in range(v):
            for r in range(8):
                # one micro-batch of one virtual stage, the recompute stripped (simulate_step adds it back)
                per_v.append(walls[r] / v / m / (3.0 + rec) * 3.0)
        job_tokens = m * tokens

        def sim(scale: float, hop_ms: float) -> float:
            t, _ = simulate_step([c * scale for c in per_v], 8, v, m, 2.0, deferred_w=1.0 / 3.0,
                                 checkpoint_stop=stop, transfer=hop_ms)
            return t

        free = sim(1.0, 0.0)
        print(f"\n## {name}: chunks {m}, v={v}, message {msg_bytes / 2**20:.0f} MiB, rank walls "
              f"{min(walls):.0f}-{max(walls):.0f} ms")
        print(f"   {'transport':34s} {'step ms':>8s} {'job tok/s':>10s} {'vs 8 x PP=1':>11s}")
        rows = [("transfers free (earlier tables)", 1.0, 0.0),
                ("RCCL (resident receive kernels)", 1.0 + hold, 0.1)]
        for bw in (100.0, 50.0):
            hop = 0.15 + msg_bytes / (bw * 1e9) * 1e3
            rows.append((f"IPC sdma, {bw:.0f} GB/s (hop {hop:.2f} ms)", 1.0, hop))
        for label, scale, hop in rows:
            t = sim(scale, hop) if (scale, hop) != (1.0, 0.0) else free
            tps = job_tokens / (t / 1e3)
            print(f"   {label:34s} {t:8.1f} {tps:10.0f} {tps / (8 * pp1):10.2f}x")
    return 0


if __name__ == "__main__":
    sys.exit(main())
