"""Engine failure detection: the step watchdog.

Unit tests of :class:`mipipe.parallel.watchdog.Watchdog`, and an end-to-end
case over gloo with a deliberately missing send: both ranks must end with a
report naming the transfer that never completed instead of hanging."""
import os
import socket
import subprocess
import sys
import threading
import time

import pytest

from mipipe.parallel.watchdog import PendingWorks, Watchdog

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _W:
    def __init__(self, done):
        self.done = done

    def is_completed(self):
        return self.done


def test_pending_works_lists_unfinished_only():
    p = PendingWorks()
    p.add("recv a", _W(True))
    p.add("recv b", _W(False))
    p.add("odd", object())  # no is_completed: reported as unknown
    assert p.unfinished() == ["recv b", "odd (state unknown)"]
    p.clear()
    assert p.unfinished() == []


def test_watchdog_fires_only_when_armed_and_stalled():
    fired = []
    ev = threading.Event()

    def hook(text):
        fired.append(text)
        ev.set()

    wd = Watchdog(0.3, rank=5, on_timeout=hook, poll=0.05, describe=lambda: "engine state X")
    try:
        time.sleep(0.5)  # not armed: nothing happens
        assert not fired
        with wd.watch("phase A"):
            for k in range(6):  # steady progress keeps it quiet
                wd.progress(f"action {k}")
                time.sleep(0.1)
            assert not fired
            wd.pending.add("recv gradient: virtual stage 1 micro-batch 3 from rank 2", _W(False))
            wd.progress("backward virtual stage 1 micro-batch 3")
            assert ev.wait(3.0)
        (text,) = fired
        assert "rank 5" in text and "backward virtual stage 1 micro-batch 3" in text
        assert "recv gradient: virtual stage 1 micro-batch 3 from rank 2" in text
        assert "engine state X" in text
        assert wd.fired
    finally:
        wd.close()


def test_watchdog_rejects_bad_timeout():
    with pytest.raises(ValueError):
        Watchdog(0)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _launch(world, drop):
    port = _port()
    procs = []
    for r in range(world):
        env = {**os.environ, "RANK": str(r), "WORLD_SIZE": str(world), "LOCAL_RANK": str(r),
               "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "WD_TIMEOUT": "4",
               "WD_DROP": "1" if drop else "0", "CUDA_VISIBLE_DEVICES": ""}
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "helpers", "watchdog_worker.py")],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, cwd="/tmp"))
    outs = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=180)
        except subprocess.TimeoutExpired:
            p.kill()
            o, e = p.communicate()
        outs.append((p.returncode, o, e))
    return outs


def test_engine_watchdog_names_missing_send():
    outs = _launch(2, drop=True)
    (rc0, _, err0), (rc1, _, err1) = outs
    # Both ranks stall at about the same moment.  The first watchdog to fire
    # names its missing transfer, aborts its process group and exits 124; the
    # peer's watchdog either fires too (124) or the peer's pending receive
    # fails on the aborted connection first, and its error report lists the
    # same transfer as left in flight.  Either way each rank names its own.
    assert 124 in (rc0, rc1), (rc0, rc1, err0[-1500:], err1[-1500:])
    assert rc0 != 0 and rc1 != 0
    # rank 1 never gets micro-batch 3's activation
    assert "recv activation: virtual stage 1 micro-batch 3 from rank 0" in err1, err1[-2000:]
    assert ("[mipipe watchdog] rank 1" in err1) == (rc1 == 124)
    # rank 0 then never gets micro-batch 3's gradient
    assert "recv gradient: virtual stage 0 micro-batch 3 from rank 1" in err0, err0[-2000:]
    assert ("[mipipe watchdog] rank 0" in err0) == (rc0 == 124)


def test_engine_watchdog_quiet_on_healthy_step():
    outs = _launch(2, drop=False)
    for rc, out, err in outs:
        assert rc == 0, err[-2000:]
        assert "step finished" in out and "watchdog" not in err
