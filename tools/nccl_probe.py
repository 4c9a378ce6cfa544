"""Probe: can two ranks share one GPU under the nccl (RCCL) backend?  If so, run
the engine's Channels (per-direction groups, warm-up, isend/irecv) over RCCL."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    rank = int(os.environ["RANK"])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    from mipipe.parallel.p2p import Channels

    ch = Channels(list(range(dist.get_world_size())), wrap=True)
    ch.warmup(dev)
    x = torch.full((4, 8), float(rank), device=dev)
    buf = torch.empty(4, 8, device=dev)
    if rank == 0:
        w1 = ch.recv_act(buf)  # wrap link from the last rank
        w0 = ch.send_act(x)
        w0.wait()
        w1.wait()
    else:
        w1 = ch.recv_act(buf)
        w1.wait()
        w0 = ch.send_act(buf + 1)
        w0.wait()
    torch.cuda.synchronize()
    print(f"rank {rank}: received {buf[0, 0].item()}", flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
