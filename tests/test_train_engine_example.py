"""examples/train_engine.py (torchrun, gloo, CPU): PP x DP training runs, and a
run resumed from its per-rank training-state files continues with the losses
of the uninterrupted run, bit for bit."""
import os
import re
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(nproc, *args):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", f"--master-port={_port()}",
           os.path.join(ROOT, "examples", "train_engine.py"), "--device", "cpu", *args]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd="/tmp",
                         env={**os.environ, "CUDA_VISIBLE_DEVICES": ""})
    assert out.returncode == 0, out.stderr[-3000:]
    return {int(m.group(1)): (m.group(2), m.group(3))
            for m in re.finditer(r"\| step\s+(\d+) \| loss\s+(\S+) \| grad-norm\s+(\S+) \|", out.stdout)}


def test_resume_continues_bit_identically(tmp_path):
    full = _run(2, "--steps", "4")
    assert sorted(full) == [0, 1, 2, 3]
    first = _run(2, "--steps", "2", "--save-dir", str(tmp_path))
    assert sorted(os.listdir(tmp_path)) == ["rank00000.safetensors", "rank00001.safetensors"]
    rest = _run(2, "--steps", "4", "--resume-dir", str(tmp_path))
    assert sorted(rest) == [2, 3]
    assert {**first, **rest} == full


def test_pp_dp_training_runs():
    losses = _run(4, "--pp", "2", "--dp", "2", "--steps", "3")
    assert sorted(losses) == [0, 1, 2]
    assert float(losses[2][0]) < float(losses[0][0])
