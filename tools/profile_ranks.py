"""Per-rank rocprofv3 timelines of a multi-rank bench.py run, then the bubble report.

Each rank is started as its OWN child process under rocprofv3 (kernel + roctx
marker traces; no launcher re-exec): ``rocprofv3 ... -- python bench.py ...``
with RANK / WORLD_SIZE / LOCAL_RANK / MASTER_* set, exactly as torchrun would
set them.  Afterwards :mod:`tools.engine_timeline` reads every rank's database
and prints per-rank busy / lead / tail / bubble and where each rank's host
thread spent the step (the engine labels every action, ``PipelineEngine.step``).

    python tools/profile_ranks.py --nproc 2 --out gpurun_out/tl -- --shared-gpu --config enc12_d4096 \\
        --num-layers 4 --steps 2 --warmup 1

On a one-GPU box use ``--shared-gpu`` (all ranks on cuda:0 over IPC links); on
a node, one rank per GPU (the ranks' LOCAL_RANK picks the device).
"""
from __future__ import annotations

import argparse
import glob
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--nproc", type=int, required=True)
    ap.add_argument("--out", default="gpurun_out/profile_ranks")
    ap.add_argument("--no-profile", action="store_true", help="run the ranks without rocprofv3")
    ap.add_argument("--copy-trace", action="store_true",
                    help="also record the runtime's memory copies (--memory-copy-trace): which engine moved what")
    ap.add_argument("bench_args", nargs=argparse.REMAINDER)
    args = ap.parse_args()
    extra = [a for a in args.bench_args if a != "--"]
    port = _port()
    procs = []
    for r in range(args.nproc):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.nproc), LOCAL_WORLD_SIZE=str(
            args.nproc), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(args.nproc)] + extra
        if not args.no_profile:
            cmd = (["rocprofv3", "--kernel-trace", "--marker-trace"] + (["--memory-copy-trace"] if args.copy_trace
                                                                          else [])
                   + ["-d", os.path.join(args.out, f"rank{r}"), "-o", "rank", "--"] + cmd)
        procs.append(subprocess.Popen(cmd, env=env, cwd=ROOT))
    rc = 0
    for p in procs:
        rc = p.wait() or rc
    if rc:
        print(f"a rank failed (rc {rc})", file=sys.stderr)
        return rc
    if not args.no_profile:
        dbs = sorted(glob.glob(os.path.join(args.out, "rank*", "**", "*.db"), recursive=True))
        return subprocess.call([sys.executable, os.path.join(ROOT, "tools", "engine_timeline.py")] + dbs)
    return 0


if __name__ == "__main__":
    sys.exit(main())
