"""Step watchdog (failure detection).

The reference has no failure detection: a dead SMDDP peer hangs every other rank inside
``loss.backward()`` (``src/trainer.py:187``). This thread catches what stops progress:

* **no progress**: if no ``beat()`` arrives for ``timeout_s`` (a wedged data pipeline, a host
  deadlock, a collective that never completes) it dumps every thread's Python stack to stderr
  and terminates the process with exit code 124, so the launcher (torchrun) sees a failure and
  tears the job down instead of hanging until the 30-minute process-group timeout;
* **collective health**: registered probes -- e.g. the native RCCL communicator's
  ``async_error()`` (``ncclCommGetAsyncError``) or the xGMI all-reduce's sticky error word --
  are polled every ``poll_s``; a non-empty answer runs the abort hooks (``ncclCommAbort``, which
  unblocks a collective stuck inside a replayed hipGraph) and exits with code 125.

Phases that legitimately make no step progress (validation, rank-0 checkpoint + barrier) run
inside ``paused()``.
"""
from __future__ import annotations

import contextlib
import faulthandler
import os
import sys
import threading
import time
from typing import Callable, List

from ml_trainer_amd.utils.logging import get_logger

logger = get_logger("ml_trainer_amd.watchdog")

EXIT_NO_PROGRESS = 124
EXIT_COMM_ERROR = 125


class Watchdog:
    def __init__(self, timeout_s: float, on_timeout=None, poll_s: float = 1.0):
        self.timeout_s = float(timeout_s)
        self.poll_s = min(poll_s, max(self.timeout_s / 4, 0.05))
        self.on_timeout = on_timeout
        self._last = time.monotonic()
        self._paused = 0
        self._stop = threading.Event()
        self._thread = None
        self._probes: List[Callable[[], str]] = []
        self._aborts: List[Callable[[], None]] = []
        self.fired = False
        self.reason = ""

    def beat(self) -> None:
        self._last = time.monotonic()

    def add_probe(self, probe: Callable[[], str], abort: Callable[[], None] = None) -> None:
        """``probe()`` returns "" when healthy, else an error description; ``abort()`` runs first
        when any probe fails."""
        self._probes.append(probe)
        if abort is not None:
            self._aborts.append(abort)

    @contextlib.contextmanager
    def paused(self):
        """No-progress detection off (probes stay on) for a phase without training steps."""
        self._paused += 1
        try:
            yield
        finally:
            self._paused -= 1
            self.beat()

    def start(self) -> "Watchdog":
        self.beat()
        self._stop.clear()
        self._thread = threading.Thread(target=self._run, name="mlt-watchdog", daemon=True)
        self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)

    def _probe(self) -> str:
        for p in self._probes:
            try:
                err = p()
            except Exception as e:  # a probe that cannot answer is itself a failure
                err = f"probe raised {type(e).__name__}: {e}"
            if err:
                return err
        return ""

    def _fire(self, reason: str, code: int) -> None:
        self.fired = True
        self.reason = reason
        if code == EXIT_COMM_ERROR:
            for a in self._aborts:
                try:
                    a()
                except Exception:  # pragma: no cover - best effort before exiting
                    pass
        if self.on_timeout is not None:
            self.on_timeout()
            return
        faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
        sys.stderr.flush()
        os._exit(code)

    def _run(self) -> None:
        while not self._stop.wait(self.poll_s):
            err = self._probe()
            if err:
                logger.error("watchdog: collective failed", error=err)
                self._fire(err, EXIT_COMM_ERROR)
                return
            idle = time.monotonic() - self._last
            if not self._paused and idle > self.timeout_s:
                logger.error("watchdog: no training progress", idle_s=round(idle, 1), timeout_s=self.timeout_s)
                self._fire(f"no progress for {idle:.1f}s", EXIT_NO_PROGRESS)
                return
