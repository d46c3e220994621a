"""Structured key=value console logger.

The reference logs through ``structlog`` with its default ``ConsoleRenderer``
(``src/trainer.py:6,19``; rendered output visible at
``01_ML_Training_local.ipynb:191``)::

    2023-02-03 15:21.11 [info     ] Config inputs.                 config={...}

structlog is not installed in this environment, so this module provides a small
logger with the same call surface (``get_logger(name)``, ``.info/.warning/
.debug/.error(event, **kv)``) and the same line format. Only rank 0 prints by
default in a distributed job (set ``MLT_LOG_ALL_RANKS=1`` to see every rank),
which avoids N-fold duplicated logs on an 8-GPU node.

Extra sinks: :func:`add_jsonl_sink` appends every record as one JSON object
per line (used by the step timers and the benchmark harness).
"""
from __future__ import annotations

import datetime as _dt
import json
import os
import sys
import threading
from typing import Any, Dict, List, Optional, TextIO

_LEVELS = {"debug": 10, "info": 20, "warning": 30, "error": 40, "critical": 50}
_lock = threading.Lock()
_jsonl_sinks: List[TextIO] = []
_min_level = _LEVELS.get(os.environ.get("MLT_LOG_LEVEL", "info").lower(), 20)


def set_level(level: str) -> None:
    global _min_level
    _min_level = _LEVELS[level.lower()]


def add_jsonl_sink(path: str) -> None:
    """Mirror every log record into ``path`` as JSON lines."""
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    _jsonl_sinks.append(open(path, "a", buffering=1))


def _rank() -> int:
    for k in ("RANK", "SLURM_PROCID", "OMPI_COMM_WORLD_RANK"):
        v = os.environ.get(k)
        if v is not None:
            try:
                return int(v)
            except ValueError:
                pass
    return 0


def _fmt_value(v: Any) -> str:
    if isinstance(v, str):
        return repr(v) if (" " in v or not v) else v
    return repr(v)


def render(level: str, event: str, kv: Dict[str, Any], now: Optional[_dt.datetime] = None) -> str:
    """Render one record exactly like structlog's default ConsoleRenderer
    (timestamp ``%Y-%m-%d %H:%M.%S``, level padded to 9, event padded to 30,
    then sorted key=value pairs)."""
    now = now or _dt.datetime.now()
    ts = now.strftime("%Y-%m-%d %H:%M.%S")
    parts = [f"{ts} [{level:<9s}] {event:<30s}"]
    for k in sorted(kv):
        parts.append(f"{k}={_fmt_value(kv[k])}")
    return " ".join(parts).rstrip()


class Logger:
    def __init__(self, name: str, stream: Optional[TextIO] = None):
        self.name = name
        self._stream = stream
        self._bound: Dict[str, Any] = {}

    def bind(self, **kv: Any) -> "Logger":
        child = Logger(self.name, self._stream)
        child._bound = {**self._bound, **kv}
        return child

    def _log(self, level: str, event: Any, kv: Dict[str, Any]) -> None:
        if _LEVELS[level] < _min_level:
            return
        event = str(event)
        merged = {**self._bound, **kv}
        all_ranks = os.environ.get("MLT_LOG_ALL_RANKS", "0") == "1"
        rank = _rank()
        if all_ranks and rank != 0:
            merged.setdefault("rank", rank)
        line = render(level, event, merged)
        with _lock:
            if rank == 0 or all_ranks:
                stream = self._stream or sys.stdout
                stream.write(line + "\n")
                stream.flush()
            if _jsonl_sinks:
                rec = {"ts": _dt.datetime.now().isoformat(), "level": level, "event": event,
                       "logger": self.name, "rank": rank}
                for k, v in merged.items():
                    try:
                        json.dumps(v)
                        rec[k] = v
                    except TypeError:
                        rec[k] = repr(v)
                for s in _jsonl_sinks:
                    s.write(json.dumps(rec) + "\n")

    def debug(self, event: Any, **kv: Any) -> None:
        self._log("debug", event, kv)

    def info(self, event: Any, **kv: Any) -> None:
        self._log("info", event, kv)

    msg = info

    def warning(self, event: Any, **kv: Any) -> None:
        self._log("warning", event, kv)

    warn = warning

    def error(self, event: Any, **kv: Any) -> None:
        self._log("error", event, kv)

    def exception(self, event: Any, **kv: Any) -> None:
        import traceback
        kv = {**kv, "exc": traceback.format_exc()}
        self._log("error", event, kv)


_loggers: Dict[str, Logger] = {}


def get_logger(name: str = "ml_trainer_amd") -> Logger:
    if name not in _loggers:
        _loggers[name] = Logger(name)
    return _loggers[name]
