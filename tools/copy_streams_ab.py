"""Pipe copy-stream layouts on one MI355X: the reference's one copy stream per (partition, micro-batch)
(``copy_streams=None``, /root/reference/pipe.py:417-429) against a pool of k streams per partition.

All partitions sit on cuda:0 (a one-GPU box, ``balance=``), so the boundary copies are same-device native
copies on the copy streams (``copy_same_device=True``); what differs between the arms is only how many HIP streams the copies and their waits are spread
over, which a process maps onto its GPU_MAX_HW_QUEUES (4) hardware queues.  Arms alternate, medians of the
step times are reported.

    python tools/copy_streams_ab.py [partitions] [chunks] [layers]
"""
import dataclasses
import statistics
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from mipipe import Pipe, ops  # noqa: E402
from mipipe.models import CONFIGS, build_lm_blocks  # noqa: E402
from mipipe.optim import FlatAdam  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 4
M = int(sys.argv[2]) if len(sys.argv) > 2 else 16
L = int(sys.argv[3]) if len(sys.argv) > 3 else 4
MB = 8
DEV = torch.device("cuda", 0)

cfg = dataclasses.replace(CONFIGS["enc12_d4096"], num_layers=L)
torch.manual_seed(0)
blocks = build_lm_blocks(cfg, dtype=torch.bfloat16)
per = (len(blocks) + P - 1) // P
parts = [torch.nn.Sequential(*blocks[i * per:(i + 1) * per]).to(DEV) for i in range(P) if blocks[i * per:(i + 1) * per]]
model = torch.nn.Sequential(*parts).train()
opt = FlatAdam(model.parameters(), lr=1e-4)
tok = torch.randint(0, cfg.vocab, (M * MB, cfg.seq_len + 1))
x, t = tok[:, :-1].to(DEV), tok[:, 1:].contiguous().to(DEV)


def step(pipe):
    opt.zero_grad()
    out = pipe(x).local_value()
    loss = ops.cross_entropy(out.reshape(-1, cfg.vocab), t.reshape(-1))
    loss.backward()
    opt.step()


arms = {"per (partition, micro-batch)": None, "pool k=1": 1, "pool k=2": 2, "pool k=4": 4}
# balance=[1]*P: one partition per part even though they share cuda:0 (without it the
# reference's split rule merges same-device children into ONE partition: no boundaries)
pipes = {name: Pipe(model, chunks=M, checkpoint="never", copy_streams=k, balance=[1] * len(parts), stage_streams="dedicated",
                    copy_same_device=True) for name, k in arms.items()}
assert all(len(p.partitions) == len(parts) for p in pipes.values())
times = {name: [] for name in arms}
for _ in range(2):  # warm-up
    for pipe in pipes.values():
        step(pipe)
torch.cuda.synchronize()
for _ in range(6):
    for name, pipe in pipes.items():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        step(pipe)
        torch.cuda.synchronize()
        times[name].append((time.perf_counter() - t0) * 1e3)
print(f"Pipe on cuda:0: {len(parts)} partitions, chunks {M}, {L}x enc12_d4096 layers, micro-batch {MB}x{cfg.seq_len}, bf16")
for name, ts in times.items():
    n = len({id(st) for st in pipes[name].pipeline.copy_streams[0]}) if pipes[name].pipeline.copy_streams else 0
    print(f"  copy streams {name:30s} ({n:2d} per partition): step {statistics.median(ts):8.2f} ms "
          f"(min {min(ts):.2f})")
for pipe in pipes.values():
    pipe.close()
