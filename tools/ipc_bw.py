"""Stage-boundary transport between two PROCESSES: 1-64 MiB messages.

Two ranks (spawned, gloo for bootstrap) exchange bf16 tensors through the
engine's channel classes, ping-pong, and report the one-way time per message
(median of the round trips / 2) and the bandwidth it implies:

* ``ipc``   -- :class:`mipipe.parallel.ipc.IpcChannels` (device-memory slots,
  sender DMA copy, interprocess-event completion);
* ``ipc-blit`` -- the same links with the blit-kernel copy engine;
* ``gloo``  -- :class:`mipipe.parallel.p2p.Channels` over gloo (host staging:
  D2H, TCP loopback, H2D) -- what multi-rank-on-one-GPU used before;
* ``rccl``  -- the same Channels over RCCL, when the two ranks have GPUs of
  their own (``--peer``: rank r on cuda:r; needs >= 2 GPUs).

    python tools/ipc_bw.py [--peer] [--iters 20]

On a one-GPU box both ranks share cuda:0 (``ipc`` / ``gloo``).
"""
from __future__ import annotations

import argparse
import os
import socket
import statistics
import sys
import time

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

SIZES_MIB = [1, 2, 4, 8, 16, 32, 64]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _channels(kind, dev, max_bytes):
    from mipipe.parallel.ipc import IpcChannels
    from mipipe.parallel.p2p import Channels

    if kind.startswith("ipc"):
        return IpcChannels([0, 1], device=dev, recv_bytes=max_bytes, slots=4,
                           engine="blit" if kind == "ipc-blit" else "sdma")
    ch = Channels([0, 1])
    ch.warmup(dev)
    return ch


def _worker(rank, ports, kinds, peer, iters, q):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    dev = torch.device("cuda", rank if peer else 0)
    torch.cuda.set_device(dev)
    out = {}
    for kind, port in zip(kinds, ports):
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        backend = "nccl" if kind == "rccl" else "gloo"
        if backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=2, device_id=dev)
        else:
            dist.init_process_group("gloo", rank=rank, world_size=2)
        try:
            max_bytes = SIZES_MIB[-1] << 20
            ch = _channels(kind, dev, max_bytes)
            for mib in SIZES_MIB:
                n = (mib << 20) // 2
                buf = torch.full((n,), float(rank), dtype=torch.bfloat16, device=dev)
                rx = torch.empty_like(buf)
                times = []
                for it in range(iters + 3):
                    torch.cuda.synchronize()
                    dist.barrier()
                    t0 = time.perf_counter()
                    if rank == 0:
                        ch.send_act(buf).wait()
                        ch.recv_grad(rx).wait()
                    else:
                        ch.recv_act(rx).wait()
                        ch.send_grad(rx).wait()
                    torch.cuda.synchronize()
                    if it >= 3:
                        times.append(time.perf_counter() - t0)
                if rank == 0:
                    assert float(rx[-1]) == 0.0  # rank 1 returned rank 0's payload
                    one_way = statistics.median(times) / 2
                    out[(kind, mib)] = (one_way * 1e6, (mib << 20) / one_way / 1e9)
            if hasattr(ch, "close"):
                ch.close()
        finally:
            dist.destroy_process_group()
    q.put(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--peer", action="store_true", help="rank r on cuda:r (>= 2 GPUs); adds rccl")
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    kinds = ["ipc", "ipc-blit", "gloo"] + (["rccl"] if args.peer else [])
    os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ports = [_port() for _ in kinds]
    procs = [ctx.Process(target=_worker, args=(r, ports, kinds, args.peer, args.iters, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        res.update(q.get(timeout=600))
    for p in procs:
        p.join(timeout=60)
    where = "rank r on cuda:r" if args.peer else "both ranks on cuda:0"
    print(f"# two processes, {where}; one-way time per message (median of {args.iters} ping-pongs / 2), "
          f"us and GB/s")
    print(f"{'MiB':>5} " + " ".join(f"{k + ' us':>12} {k + ' GB/s':>12}" for k in kinds))
    for mib in SIZES_MIB:
        cells = []
        for k in kinds:
            us, gbs = res.get((k, mib), (float("nan"), float("nan")))
            cells.append(f"{us:12.1f} {gbs:12.1f}")
        print(f"{mib:5d} " + " ".join(cells))


if __name__ == "__main__":
    main()
