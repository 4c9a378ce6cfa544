"""Why the Adam step's time swings between profiles: the
same kernel on the same 1.44B-parameter buffers (the enc12 PP=1 stage: bf16
model + fp32 master / grad / moments, 30 B per parameter) timed in three chip
states, each with the amdsmi telemetry of its window:

  idle   -- after 3 s with nothing running, one update at a time
  burst  -- right after ~150 ms of back-to-back 8192x4096x4096 GEMMs (the state
            the step's optimizer runs in: after the weight-gradient flush)
  stream -- 20 updates back to back

    python tools/adam_power_probe.py
"""
import statistics
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from mipipe._native_loader import kernels  # noqa: E402
from mipipe.utils.telemetry import GpuTelemetry  # noqa: E402

k = kernels()
n = 1_444_860_160
dev = "cuda"
master = torch.randn(n, device=dev)
model = master.to(torch.bfloat16)
grad = torch.randn(n, device=dev) * 1e-3
m = torch.zeros(n, device=dev)
v = torch.zeros(n, device=dev)
sq = torch.ones(1, device=dev)
x = torch.randn(8192, 4096, device=dev).to(torch.bfloat16)
w = torch.randn(4096, 4096, device=dev).to(torch.bfloat16)


def adam():
    k.adam_step(master, model, grad, m, v, 1e-4, 0.9, 0.999, 1e-8, 0.0, 0.1, 0.001, sq, 0.5, False)


def timed(fn):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e)


def report(name, ts, tel):
    gb = 30.0 * n / 1e9
    med = statistics.median(ts)
    t = tel.stop()
    clk = t.get("gfxclk_mhz") or {}
    pw = t.get("socket_power_w") or {}
    uc = t.get("uclk_mhz") or {}
    print(f"{name:7s} median {med:6.2f} ms (min {min(ts):6.2f}, max {max(ts):6.2f}) = {gb / med:5.2f} TB/s | gfxclk "
          f"{clk.get('mean')} MHz, power {pw.get('mean')} W (max {pw.get('max')}), power-limited "
          f"{t.get('power_limited_pct')} %, uclk {uc.get('mean')} MHz", flush=True)


for _ in range(3):
    adam()
torch.cuda.synchronize()
for rep in range(2):
    ts = []
    tel = GpuTelemetry(0, period=0.02).start()
    for _ in range(5):
        time.sleep(3.0)
        ts.append(timed(adam))
    report("idle", ts, tel)

    ts = []
    tel = GpuTelemetry(0, period=0.02).start()
    for _ in range(5):
        time.sleep(1.0)
        for _ in range(800):  # ~150 ms of GEMMs at ~190 us each
            k.linear_fwd(x, w, None, 0, 0.0, False)
        ts.append(timed(adam))
    report("burst", ts, tel)

    tel = GpuTelemetry(0, period=0.02).start()
    ts = [timed(adam) for _ in range(20)]
    report("stream", ts, tel)
