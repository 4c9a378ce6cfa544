"""Debug aid: two ranks on cuda:0 exchange a few messages over IpcChannels, then
tear the links down with a trace of every step (MIPIPE_IPC_DEBUG=1).

    MIPIPE_IPC_DEBUG=1 python tools/ipc_teardown_probe.py
"""
import faulthandler
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _worker(rank, port, q):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    faulthandler.dump_traceback_later(40, exit=True)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    from mipipe.parallel.ipc import IpcChannels

    ch = IpcChannels([0, 1], device=dev, recv_bytes=1 << 20, slots=2, timeout=20.0)
    x = torch.full((1 << 19,), float(rank + 1), dtype=torch.bfloat16, device=dev)
    for it in range(6):
        if rank == 0:
            ch.send_act(x).wait()
            ch.recv_grad(x).wait()
        else:
            ch.recv_act(x).wait()
            ch.send_grad(x).wait()
    torch.cuda.synchronize()
    print(f"[rank {rank}] exchanged, value {float(x[0])}; closing", flush=True)
    ch.close()
    print(f"[rank {rank}] closed; destroying the process group", flush=True)
    dist.destroy_process_group()
    print(f"[rank {rank}] done; putting", flush=True)
    faulthandler.dump_traceback_later(15, exit=False, repeat=True)
    q.put(rank)
    print(f"[rank {rank}] put returned", flush=True)
    q.close()
    q.join_thread()
    print(f"[rank {rank}] queue flushed", flush=True)


if __name__ == "__main__":
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = [q.get(timeout=90) for _ in range(2)]
    for p in ps:
        p.join(30)
    print("results", sorted(got))
