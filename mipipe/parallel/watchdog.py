"""Step watchdog for the multi-process pipeline.

The reference holds the first worker exception and re-raises it after the
clock tick drains (``/root/reference/pipeline.py:239-247,264-266``); it has no
cross-process failure story because it is one process.  With one process per
GPU a missing send on one rank leaves its peers waiting forever: with RCCL the
receive is a stream wait, so the host keeps issuing work and only blocks at the
next ``synchronize``; with gloo the host blocks in ``Work.wait``.  Neither says
which transfer never arrived.

:class:`Watchdog` is a daemon thread fed with progress marks (one per engine
action, per transfer posted / consumed).  When no mark arrives for ``timeout``
seconds while it is armed, it prints one report -- rank, the last action, and
every transfer of the current step that has not completed -- aborts the
process groups it was given (so RCCL kernels blocked on a peer are torn down)
and ends the process with ``exit_code``.  ``torchrun`` then stops the other
ranks.  No exec is involved: the process simply exits.
"""
from __future__ import annotations

import os
import sys
import threading
import time
from contextlib import contextmanager
from typing import Callable, Dict, Iterator, List, Optional, Tuple

import torch.distributed as dist

__all__ = ["Watchdog", "PendingWorks"]


class PendingWorks:
    """Labelled transfer handles of the current step, for the report."""

    def __init__(self) -> None:
        self._lock = threading.Lock()
        self._works: Dict[int, Tuple[str, object]] = {}
        self._next = 0

    def add(self, label: str, work):
        with self._lock:
            key = self._next
            self._next += 1
            self._works[key] = (label, work)
        return work

    def clear(self) -> None:
        with self._lock:
            self._works.clear()

    def unfinished(self) -> List[str]:
        with self._lock:
            items = list(self._works.values())
        out = []
        for label, work in items:
            done = None
            try:
                done = bool(work.is_completed())
            except Exception:  # a handle without is_completed: report it as unknown
                done = None
            if done is not True:
                out.append(f"{label}{'' if done is False else ' (state unknown)'}")
                continue
            # completed -- but a transfer whose peer went away completes with an error
            failed = False
            try:
                failed = not work.is_success()
            except Exception:
                try:
                    failed = work.exception() is not None
                except Exception:
                    failed = False
            if failed:
                out.append(f"{label} (failed)")
        return out

    def __len__(self) -> int:
        return len(self._works)


class Watchdog:
    """Kills a rank whose pipeline step stops making progress.

    Args:
        timeout: seconds without a :meth:`progress` mark (while armed) before firing.
        rank: rank printed in the report (default: ``dist.get_rank()`` when initialised).
        describe: optional callable adding state to the report.
        on_timeout: called with the report instead of the default abort + exit
            (tests use this to observe the report without dying).
        groups: process groups to abort before exiting (default: the world group).
        exit_code: process exit status on timeout.
    """

    def __init__(
        self,
        timeout: float,
        *,
        rank: Optional[int] = None,
        describe: Optional[Callable[[], str]] = None,
        on_timeout: Optional[Callable[[str], None]] = None,
        groups: Optional[List[object]] = None,
        exit_code: int = 124,
        poll: Optional[float] = None,
    ) -> None:
        if timeout <= 0:
            raise ValueError("watchdog timeout must be positive")
        self.timeout = float(timeout)
        self._rank = rank
        self.describe = describe
        self.on_timeout = on_timeout
        self.groups = groups
        self.exit_code = exit_code
        self.pending = PendingWorks()
        self._poll = poll if poll is not None else min(1.0, self.timeout / 4)
        self._cv = threading.Condition()
        self._armed = 0
        self._label = "idle"
        self._last = time.monotonic()
        self._fired = False
        self._stop = False
        self._thread = threading.Thread(target=self._run, name="mipipe-watchdog", daemon=True)
        self._thread.start()

    # ---------------------------------------------------------------- marks
    @property
    def rank(self) -> int:
        if self._rank is not None:
            return self._rank
        if dist.is_available() and dist.is_initialized():
            return dist.get_rank()
        return 0

    @property
    def fired(self) -> bool:
        return self._fired

    def progress(self, label: str) -> None:
        """Marks progress: the timer restarts and ``label`` becomes the last action."""
        with self._cv:
            self._label = label
            self._last = time.monotonic()

    @contextmanager
    def watch(self, label: str) -> Iterator["Watchdog"]:
        """Arms the watchdog for the block (nested blocks are counted)."""
        with self._cv:
            self._armed += 1
            self._label = label
            self._last = time.monotonic()
        try:
            yield self
        finally:
            with self._cv:
                self._armed -= 1
                self._last = time.monotonic()

    def close(self) -> None:
        with self._cv:
            self._stop = True
            self._cv.notify_all()
        self._thread.join(timeout=5)

    # ---------------------------------------------------------------- thread
    def report(self, stalled: float) -> str:
        lines = [f"[mipipe watchdog] rank {self.rank}: no pipeline progress for {stalled:.1f}s "
                 f"(timeout {self.timeout:.1f}s); last action: {self._label}"]
        unfinished = self.pending.unfinished()
        if unfinished:
            lines.append(f"[mipipe watchdog] rank {self.rank}: {len(unfinished)} transfer(s) of this step not "
                         f"completed:")
            lines.extend(f"[mipipe watchdog]   {u}" for u in unfinished[:64])
            if len(unfinished) > 64:
                lines.append(f"[mipipe watchdog]   ... and {len(unfinished) - 64} more")
        else:
            lines.append(f"[mipipe watchdog] rank {self.rank}: no transfer of this step is pending "
                         f"(a peer or a collective outside the engine is stuck)")
        if self.describe is not None:
            try:
                lines.append(f"[mipipe watchdog] rank {self.rank}: {self.describe()}")
            except Exception as exc:  # the report must not die on a broken hook
                lines.append(f"[mipipe watchdog] rank {self.rank}: describe() failed: {exc!r}")
        return "\n".join(lines)

    def _run(self) -> None:
        while True:
            with self._cv:
                self._cv.wait(self._poll)
                if self._stop:
                    return
                if self._armed <= 0 or self._fired:
                    continue
                stalled = time.monotonic() - self._last
                if stalled < self.timeout:
                    continue
                self._fired = True
            text = self.report(stalled)
            if self.on_timeout is not None:
                self.on_timeout(text)
                continue
            print(text, file=sys.stderr, flush=True)
            self._abort_groups()
            os._exit(self.exit_code)

    def _abort_groups(self) -> None:
        """Best-effort abort of the process groups (bounded: abort itself may block)."""
        if not (dist.is_available() and dist.is_initialized()):
            return

        def _abort():
            try:
                from torch.distributed.distributed_c10d import _abort_process_group

                for g in (self.groups or [None]):
                    _abort_process_group(g)
            except Exception:
                pass

        t = threading.Thread(target=_abort, daemon=True)
        t.start()
        t.join(timeout=10)
