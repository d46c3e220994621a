"""roctx ranges (visible with ``rocprofv3 --marker-trace``) and step timers.

``range_ctx(name, enabled)`` pushes/pops a roctx range through torch's
``torch.cuda.nvtx`` binding, which on ROCm builds calls roctx. Disabled ranges
cost nothing.
"""
from __future__ import annotations

import contextlib
import time

import torch


@contextlib.contextmanager
def range_ctx(name: str, enabled: bool = True):
    pushed = False
    if enabled and torch.cuda.is_available():
        try:
            torch.cuda.nvtx.range_push(name)
            pushed = True
        except Exception:  # pragma: no cover - profiler library absent
            pushed = False
    try:
        yield
    finally:
        if pushed:
            torch.cuda.nvtx.range_pop()


class StepTimer:
    """Device-time (HIP events) + wall-time timer for a block of steps."""

    def __init__(self, device=None):
        self.cuda = torch.cuda.is_available() and (device is None or torch.device(device).type == "cuda")

    def __enter__(self):
        self.t0 = time.perf_counter()
        if self.cuda:
            self.e0 = torch.cuda.Event(enable_timing=True)
            self.e1 = torch.cuda.Event(enable_timing=True)
            self.e0.record()
        return self

    def __exit__(self, *a):
        if self.cuda:
            self.e1.record()
            self.e1.synchronize()
            self.device_ms = self.e0.elapsed_time(self.e1)
        self.wall_ms = (time.perf_counter() - self.t0) * 1e3
        if not self.cuda:
            self.device_ms = self.wall_ms
        return False
