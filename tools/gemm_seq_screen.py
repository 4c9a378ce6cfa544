"""Which neighbour makes the GELU + pre-activation forward GEMM come out wrong now and then?
Runs sequences of forward GEMMs (the launches of tools/gemm_round_screen.py) many times and counts
runs whose GELU output differs from the first run of the same sequence:

  seq A: relu+dropout fwd (y1), GELU+aux fwd (y2)          -- the round screen's first two launches
  seq B: the same with a device synchronize between them
  seq C: GELU+aux alone
  seq D: plain bias fwd, then GELU+aux

    python tools/gemm_seq_screen.py [reps]
"""
import math
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from mipipe._native_loader import kernels  # noqa: E402

k = kernels()
DEV = "cuda"
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
torch.manual_seed(12)
T, K, N = 2048, 512, 9000
x = torch.randn(T, K, device=DEV).to(torch.bfloat16)
w = (torch.randn(N, K, device=DEV) / math.sqrt(K)).to(torch.bfloat16)
b = torch.randn(N, device=DEV).to(torch.bfloat16)


def gelu_aux():
    torch.manual_seed(78)
    return k.linear_fwd(x, w, b, 2, 0.0, True)[:2]


def relu_drop():
    torch.manual_seed(77)
    return k.linear_fwd(x, w, b, 1, 0.3, False)[0]


SEQS = {
    "A relu+drop -> gelu+aux": lambda: (relu_drop(), gelu_aux())[1],
    "B relu+drop, sync, gelu+aux": lambda: (relu_drop(), torch.cuda.synchronize(), gelu_aux())[2],
    "C gelu+aux alone": gelu_aux,
    "D bias fwd -> gelu+aux": lambda: (k.linear_fwd(x, w, b, 0, 0.0, False)[0], gelu_aux())[1],
}
for name, fn in SEQS.items():
    first = [t.clone() for t in fn()]
    bad = 0
    for _ in range(reps):
        got = fn()
        if not all(torch.equal(g, f) for g, f in zip(got, first)):
            bad += 1
    print(f"{name:30s}: {bad}/{reps} runs differ", flush=True)
