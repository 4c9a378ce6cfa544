"""Stage-boundary transport between two PROCESSES: 1-64 MiB messages.

Two ranks (spawned, gloo for bootstrap) exchange bf16 tensors through the
engine's channel classes, ping-pong, and report the one-way time per message
(median of the round trips / 2) and the bandwidth it implies:

* ``ipc``   -- :class:`mipipe.parallel.ipc.IpcChannels` (device-memory slots,
  sender DMA copy, GPU-side flags), timed like the others: one ping-pong per
  host iteration with a device sync and a barrier around it;
* ``ipc-stream`` -- the same links driven the way the engine drives them: the
  ping-pongs queued back to back with zero-copy receives and no host wait,
  timed on the GPU (events) -- the transport's own one-way latency.  Both
  ranks queue the whole loop behind a GPU sleep first, so the timed part runs
  at the GPU's pace, not at Python's enqueue rate;
* ``ipc-stream-blit`` -- ``ipc-stream`` with the blit-kernel copy engine;
* ``ipc-stream-inline`` -- ``ipc-stream`` with the copy (blit) on the producer's
  stream itself: no cross-stream dependency per message;
* ``ipc-blit`` -- the ``ipc`` arm with the blit-kernel copy engine;
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
        return IpcChannels([0, 1], device=dev, recv_bytes=max_bytes, slots=4, timeout=30.0,
                           engine="inline" if kind.endswith("inline") else ("blit" if kind.endswith("blit")
                                                                            else "sdma"))
    ch = Channels([0, 1])
    ch.warmup(dev)
    return ch


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def _worker(rank, ports, kinds, peer, iters, q, cpu=False):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    dev = torch.device("cpu") if cpu else torch.device("cuda", rank if peer else 0)
    if dev.type == "cuda":
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
                print(f"[rank {rank}] {kind} {mib} MiB", flush=True)
                n = (mib << 20) // 2
                buf = torch.full((n,), float(rank), dtype=torch.bfloat16, device=dev)
                rx = torch.empty_like(buf)
                if kind.startswith("ipc-stream"):
                    # back-to-back ping-pongs, zero-copy receives, no host wait; GPU-timed.
                    # The loop is queued behind a sleep so it runs at the GPU's pace.
                    n_it = max(iters, 50)  # ~13 queue packets per iteration: stays within the HW queue
                    _sync(dev)
                    dist.barrier()
                    from mipipe._native_loader import kernels
                    kernels().gpu_sleep(300_000)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    last = None
                    t_host = time.perf_counter()
                    for it in range(n_it):
                        if rank == 0:
                            ch.send_act(buf).wait()
                            last, w = ch.recv_grad_view(buf.shape, buf.dtype)
                            w.wait()
                        else:
                            t, w = ch.recv_act_view(buf.shape, buf.dtype)
                            w.wait()
                            ch.send_grad(t).wait()  # the reply reads the slot: release after its copy
                        if rank == 0:
                            rx.copy_(last)
                        ch.end_step()
                    e1.record()
                    t_host = time.perf_counter() - t_host
                    _sync(dev)
                    if t_host > 0.25:
                        print(f"[rank {rank}] {kind}: queueing took {t_host:.3f} s, longer than the sleep: "
                              "the time below is host-bound", flush=True)
                    elif mib == 1:
                        print(f"[rank {rank}] {kind}: host enqueue {t_host / n_it * 1e6:.1f} us per ping-pong "
                              "(all queued behind the sleep)", flush=True)
                    if rank == 0:
                        assert float(rx[-1]) == 0.0
                        one_way = e0.elapsed_time(e1) / 1e3 / n_it / 2
                        out[(kind, mib)] = (one_way * 1e6, (mib << 20) / one_way / 1e9)
                    continue
                times = []
                for it in range(iters + 3):
                    if mib == 1 and it < 8:
                        print(f"[rank {rank}] {kind} it {it}", flush=True)
                    _sync(dev)
                    dist.barrier()
                    t0 = time.perf_counter()
                    if rank == 0:
                        ch.send_act(buf).wait()
                        ch.recv_grad(rx).wait()
                    else:
                        ch.recv_act(rx).wait()
                        ch.send_grad(rx).wait()
                    _sync(dev)
                    if it >= 3:
                        times.append(time.perf_counter() - t0)
                if rank == 0:
                    assert float(rx[-1]) == 0.0  # rank 1 returned rank 0's payload
                    one_way = statistics.median(times) / 2
                    out[(kind, mib)] = (one_way * 1e6, (mib << 20) / one_way / 1e9)
            q.put(out)  # before any teardown
            q.close()
            q.join_thread()
            if hasattr(ch, "close"):
                ch.close()
        finally:
            dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--peer", action="store_true", help="rank r on cuda:r (>= 2 GPUs); adds rccl")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--cpu", action="store_true", help="host-mode links (protocol check, no GPU)")
    args = ap.parse_args()
    kinds = ["ipc-stream", "ipc-stream-blit", "ipc-stream-inline", "ipc", "ipc-blit", "gloo"] + (["rccl"] if args.peer else [])
    if args.cpu:
        kinds = ["ipc", "gloo"]
    os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
    ctx = mp.get_context("spawn")
    res = {}
    for kind in kinds:  # fresh processes per transport
        q = ctx.Queue()
        port = _port()
        procs = [ctx.Process(target=_worker, args=(r, [port], [kind], args.peer, args.iters, q, args.cpu))
                 for r in range(2)]
        for p in procs:
            p.start()
        try:
            for _ in range(2):
                res.update(q.get(timeout=120))
        except Exception as exc:  # noqa: BLE001 -- report the arm as missing, keep the others
            print(f"# {kind}: no result ({type(exc).__name__})", flush=True)
        for p in procs:
            p.join(timeout=10)
            if p.exitcode is None:
                p.kill()
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
