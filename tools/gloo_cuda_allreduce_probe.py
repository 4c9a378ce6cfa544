"""Does all_reduce over a gloo group reduce CUDA tensors in place?  (bench.py --shared-gpu reduces the grad-norm
sum of squares, a CUDA scalar, over gloo.)

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 tools/gloo_cuda_allreduce_probe.py
"""
import os

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
dist.init_process_group("gloo")
t = torch.full((), float(rank + 1), device="cuda")
dist.all_reduce(t)
torch.cuda.synchronize()
w = dist.get_world_size()
print(f"rank {rank}: all_reduce(cuda scalar) = {t.item()} (expect {w * (w + 1) / 2})", flush=True)
dist.destroy_process_group()
