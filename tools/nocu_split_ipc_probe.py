"""The IPC links' case of tools/nocu_split_probe.py: the destination is ANOTHER process's allocation mapped through
CUDA/HIP IPC (torch.multiprocessing shares the tensor by an IPC handle), as a link's slot is -- same GPU.  A 128 MiB
hipMemcpyDeviceToDeviceNoCU copy as 1, 2, 4, 8 parts on as many streams."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

N = 128 << 20


def child(q_in, q_out):
    from mipipe import _native_loader

    k = _native_loader.kernels()
    dst = q_in.get()  # mapped from the parent by an IPC handle
    src = torch.empty(N, dtype=torch.uint8, device="cuda")
    main = torch.cuda.current_stream()
    pool = [torch.cuda.Stream() for _ in range(8)]

    def copy(parts):
        step = N // parts
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

    lines = []
    for parts in (1, 2, 4, 8, 1, 2, 4, 8):
        for _ in range(3):
            copy(parts)
        torch.cuda.synchronize()
        ts = []
        for _ in range(10):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(main)
            copy(parts)
            b.record(main)
            b.synchronize()
            ts.append(a.elapsed_time(b))
        ms = statistics.median(ts)
        lines.append(f"128 MiB NoCU copy into an IPC-mapped peer allocation, {parts} part(s) on {parts} stream(s): "
                     f"{ms * 1e3:8.1f} us  {N / ms / 1e6:6.1f} GB/s")
    del dst
    q_out.put(lines)


def main():
    ctx = mp.get_context("spawn")
    q_in, q_out = ctx.Queue(), ctx.Queue()
    dst = torch.empty(N, dtype=torch.uint8, device="cuda")
    p = ctx.Process(target=child, args=(q_in, q_out))
    p.start()
    q_in.put(dst)
    for line in q_out.get(timeout=120):
        print(line, flush=True)
    p.join(timeout=60)
    assert p.exitcode == 0


if __name__ == "__main__":
    main()
