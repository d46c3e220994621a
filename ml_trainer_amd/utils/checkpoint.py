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
"""
from __future__ import annotations

import os
import pickle
import tempfile
from collections import OrderedDict
from typing import Any, Dict

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
