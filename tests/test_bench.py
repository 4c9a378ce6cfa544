"""bench.py contract: one JSON line with the driver's fields, single and multi-rank.

Runs the CPU plumbing mode (``--device cpu``: gloo + fp32, tiny model) so the
torchrun launch, barriers, max-over-ranks timing and the rank-0 JSON line are
exercised here; the GPU/RCCL numbers come from the MI355X runs."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REQUIRED = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config"}


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


@pytest.mark.parametrize("nproc,extra", [(1, []), (2, []), (2, ["--chunks-per-rank", "1", "--checkpoint", "always"]),
                                         (3, ["--skips", "unet", "--chunks-per-rank", "1"]),
                                         # the full-node plan shape: looping stages, split LM head, except_last
                                         (4, ["--split-decoder", "on", "--chunks-per-rank", "2",
                                              "--checkpoint", "except_last"]),
                                         (8, [])])
def test_bench_json_contract(nproc, extra):
    args = ["--gpus", str(nproc), "--steps", "2", "--warmup", "1", "--device", "cpu", "--config", "tiny",
            "--micro-batch", "2"] + extra
    if nproc == 1:
        cmd = [sys.executable, os.path.join(ROOT, "bench.py")] + args
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr", "127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "bench.py")] + args
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd="/tmp",
                         env={**os.environ, "CUDA_VISIBLE_DEVICES": ""})
    assert out.returncode == 0, out.stderr[-3000:]
    lines = _json_lines(out.stdout)
    assert len(lines) == 1, out.stdout  # rank 0 only, exactly one line
    rec = lines[0]
    assert REQUIRED <= set(rec)
    assert rec["n_gpus"] == nproc and rec["steps"] == 2 and rec["warmup"] == 1
    assert rec["value"] > 0 and rec["higher_is_better"] is True and rec["scaling"] == "weak"
    cfg = rec["config"]
    assert {"model", "global_batch", "seq_len", "parallelism"} <= set(cfg)
    assert cfg["parallelism"] == f"pp{nproc}"
    assert cfg["global_batch"] == cfg["chunks"] * cfg["micro_batch"]
    tokens = cfg["global_batch"] * cfg["seq_len"]
    assert abs(rec["value"] - tokens / (rec["ms_per_step"] / 1e3)) / rec["value"] < 0.01
    assert rec["loss"] is not None and rec["loss"] > 0
