"""Step watchdog (failure detection).

Collectives already time out inside the process group (``dist_timeout_s``);
this thread catches everything else that stops progress (a wedged data
pipeline, a host deadlock): if no ``beat()`` arrives for ``timeout_s`` it dumps
every thread's Python stack to stderr and terminates the process with exit
code 124, so the launcher sees a failure instead of a silent hang.
"""
from __future__ import annotations

import faulthandler
import os
import sys
import threading
import time

from ml_trainer_amd.utils.logging import get_logger

logger = get_logger("ml_trainer_amd.watchdog")


class Watchdog:
    def __init__(self, timeout_s: float, on_timeout=None, poll_s: float = 1.0):
        self.timeout_s = float(timeout_s)
        self.poll_s = min(poll_s, max(self.timeout_s / 4, 0.05))
        self.on_timeout = on_timeout
        self._last = time.monotonic()
        self._stop = threading.Event()
        self._thread = None
        self.fired = False

    def beat(self) -> None:
        self._last = time.monotonic()

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

    def _run(self) -> None:
        while not self._stop.wait(self.poll_s):
            idle = time.monotonic() - self._last
            if idle > self.timeout_s:
                self.fired = True
                logger.error("watchdog: no training progress", idle_s=round(idle, 1), timeout_s=self.timeout_s)
                if self.on_timeout is not None:
                    self.on_timeout()
                    return
                faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
                os._exit(124)
