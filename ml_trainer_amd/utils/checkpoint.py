"""Checkpoint / history artifacts.

Byte-compatible with the reference layout (``src/trainer.py:232-241``,
SURVEY.md B4/§5.4):

* ``model_dir/model.pth`` -- ``torch.save(state_dict)`` of fp32 CPU tensors with
  the reference key names (``module.`` prefix when DDP-wrapped);
* ``model_dir/history.pkl`` -- pickled dict with keys ``epochs, train_loss,
  val_loss, train_metric, val_metric, metric_type``.

Fixes over the reference: the live model is never moved to the CPU (B5: a
detached host snapshot is taken instead), the directory is created, and writes
are atomic (temp file + ``os.replace``) so a crash cannot leave a torn
``model.pth``. The optional ``trainer_state.pt`` (optimizer, scheduler, epoch,
RNG) enables ``--resume`` without touching the reference artifacts.

``AsyncCheckpointer`` takes the epoch checkpoint off the training loop's critical path (SURVEY.md
§5.4 "snapshot asynchronously from device to pinned host"): same bytes on disk, written by a
background thread from a pinned host snapshot.
"""
from __future__ import annotations

import os
import pickle
import tempfile
from collections import OrderedDict
from concurrent.futures import Future, ThreadPoolExecutor
from typing import Any, Dict, Optional

import torch


def _atomic_write(path: str, write_fn) -> None:
    d = os.path.dirname(os.path.abspath(path)) or "."
    os.makedirs(d, exist_ok=True)
    fd, tmp = tempfile.mkstemp(dir=d, prefix=".tmp_" + os.path.basename(path))
    try:
        with os.fdopen(fd, "wb") as f:
            write_fn(f)
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, path)
    except BaseException:
        if os.path.exists(tmp):
            os.unlink(tmp)
        raise


def host_state_dict(module: torch.nn.Module) -> "OrderedDict[str, torch.Tensor]":
    """Snapshot a module's state_dict to CPU without moving the module (B5 fix)."""
    sd = module.state_dict()
    out = OrderedDict()
    for k, v in sd.items():
        out[k] = v.detach().to("cpu", copy=True) if isinstance(v, torch.Tensor) else v
    return out


def save_model_file(module: torch.nn.Module, model_dir: str, filename: str = "model.pth") -> str:
    path = os.path.join(model_dir, filename)
    sd = host_state_dict(module)
    _atomic_write(path, lambda f: torch.save(sd, f))
    return path


def save_history_file(history: Dict[str, Any], model_dir: str, filename: str = "history.pkl") -> str:
    path = os.path.join(model_dir, filename)
    _atomic_write(path, lambda f: pickle.dump(history, f))
    return path


def save_trainer_state(state: Dict[str, Any], model_dir: str, filename: str = "trainer_state.pt") -> str:
    path = os.path.join(model_dir, filename)
    _atomic_write(path, lambda f: torch.save(state, f))
    return path


def load_trainer_state(model_dir: str, filename: str = "trainer_state.pt"):
    path = os.path.join(model_dir, filename)
    if not os.path.exists(path):
        return None
    # written by this framework: plain containers + tensors only
    return torch.load(path, map_location="cpu", weights_only=True)


def strip_module_prefix(sd: Dict[str, Any]) -> "OrderedDict[str, Any]":
    return OrderedDict((k[7:] if k.startswith("module.") else k, v) for k, v in sd.items())


def to_host(obj):
    """Deep copy of a nest of dicts / lists / tuples with every tensor copied to the CPU (a
    snapshot that later device updates cannot change)."""
    if isinstance(obj, torch.Tensor):
        return obj.detach().to("cpu", copy=True)
    if isinstance(obj, dict):
        return type(obj)((k, to_host(v)) for k, v in obj.items()) if isinstance(obj, OrderedDict) \
            else {k: to_host(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(to_host(v) for v in obj)
    return obj


class AsyncCheckpointer:
    """Epoch checkpoints written in the background.

    ``save(module, path)``: the state_dict's device tensors are copied device -> pinned host buffers
    on a side HIP stream that is ordered after the work already queued on the current stream, and
    the current stream then waits for that copy (so the next optimizer steps cannot overwrite a
    parameter before it is captured) -- no host synchronisation. One worker thread waits for the
    copy's event, serialises the host snapshot (``torch.save`` of CPU tensors: the bytes of the
    synchronous ``save_model_file``) and writes it atomically. Host buffers are reused from save to
    save; a save first waits for the previous write to finish. ``wait()`` re-raises a failed write.
    Other entries of the state_dict (CPU tensors, non-tensors) are snapshotted synchronously."""

    def __init__(self) -> None:
        self._bufs: Dict[str, torch.Tensor] = {}
        self._pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix="mlt-ckpt")
        self._pending: Optional[Future] = None
        self._streams: Dict[torch.device, "torch.cuda.Stream"] = {}

    def _host_buf(self, key: str, v: torch.Tensor) -> torch.Tensor:
        buf = self._bufs.get(key)
        if buf is None or buf.shape != v.shape or buf.dtype != v.dtype:
            buf = torch.empty(v.shape, dtype=v.dtype, pin_memory=True)
            self._bufs[key] = buf
        return buf

    def snapshot(self, module: torch.nn.Module):
        """(host state_dict, event of the device -> host copies or None)."""
        sd = module.state_dict()
        out: "OrderedDict[str, Any]" = OrderedDict()
        dev = next((v.device for v in sd.values() if isinstance(v, torch.Tensor) and v.is_cuda), None)
        event = None
        if dev is not None:
            cur = torch.cuda.current_stream(dev)
            side = self._streams.get(dev)
            if side is None:
                side = self._streams[dev] = torch.cuda.Stream(device=dev)
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                for k, v in sd.items():
                    if isinstance(v, torch.Tensor) and v.is_cuda:
                        self._host_buf(k, v).copy_(v.detach(), non_blocking=True)
            event = torch.cuda.Event()
            event.record(side)
            cur.wait_stream(side)  # later updates of the parameters run after the copy
        for k, v in sd.items():
            if isinstance(v, torch.Tensor):
                out[k] = self._bufs[k] if v.is_cuda else v.detach().to("cpu", copy=True)
            else:
                out[k] = v
        return out, event

    def save(self, module: torch.nn.Module, path: str, extra=()) -> None:
        """Snapshot ``module`` now; write it to ``path``, then each ``(path, obj)`` of ``extra``
        (already host-resident objects, e.g. a ``to_host``'d trainer state), in the background."""
        self.wait()  # the host buffers are about to be overwritten
        sd, event = self.snapshot(module)
        extra = list(extra)

        def job() -> str:
            if event is not None:
                event.synchronize()
            _atomic_write(path, lambda f: torch.save(sd, f))
            for p, obj in extra:
                _atomic_write(p, lambda f, o=obj: torch.save(o, f))
            return path

        self._pending = self._pool.submit(job)

    def wait(self) -> Optional[str]:
        """Block until the last save is on disk; returns its path (re-raises a failed write)."""
        p, self._pending = self._pending, None
        return p.result() if p is not None else None

    def close(self) -> None:
        try:
            self.wait()
        finally:
            self._pool.shutdown(wait=True)
