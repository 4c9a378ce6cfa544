"""Does splitting one large DMA copy over several streams (SDMA engines) raise its bandwidth?  The IPC links copy a
64-128 MiB boundary message with hipMemcpyDeviceToDeviceNoCU on ONE copy stream (~60 GB/s within a device,
profiles/nocu_copy_r5.txt).  Here: a 128 MiB device-to-device NoCU copy as 1, 2, 4, 8 equal parts on as many
streams, each part ordered after an event on the launching stream, all joined back -- the pattern a split send
would use.  Same device (the one-GPU box); the copy engines and queues are the ones a cross-GPU send uses."""
import statistics
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mipipe import _native_loader  # noqa: E402

k = _native_loader.kernels()
n = 128 << 20
src = torch.empty(n, dtype=torch.uint8, device="cuda")
dst = torch.empty_like(src)
main = torch.cuda.current_stream()
pool = [torch.cuda.Stream() for _ in range(8)]


def copy(parts: int) -> None:
    step = n // parts
    ev = torch.cuda.Event()
    ev.record(main)
    done = []
    for i in range(parts):
        s = pool[i]
        s.wait_event(ev)
        err = k.copy_nocu(dst[i * step:(i + 1) * step], src[i * step:(i + 1) * step], s.cuda_stream)
        assert not err, err
        e = torch.cuda.Event()
        e.record(s)
        done.append(e)
    for e in done:
        main.wait_event(e)


for parts in (1, 2, 4, 8, 1, 2, 4, 8):
    for _ in range(3):
        copy(parts)
    torch.cuda.synchronize()
    ts = []
    for _ in range(20):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(main)
        copy(parts)
        b.record(main)
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ms = statistics.median(ts)
    print(f"128 MiB NoCU copy in {parts} part(s) on {parts} stream(s): {ms * 1e3:8.1f} us  {n / ms / 1e6:6.1f} GB/s",
          flush=True)
