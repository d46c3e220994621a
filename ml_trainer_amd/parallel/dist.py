"""Process-group bootstrap for one-process-per-GPU training.

The reference initialises ``torch.distributed`` with the SageMaker ``smddp``
backend (``src/trainer.py:43-44,59``) and binds ``LOCAL_RANK`` *after* wrapping
the model (defect B6). Here:

* ``backend`` names map onto what exists on an MI355X node: ``smddp`` / ``rccl``
  / ``nccl`` -> torch's ``nccl`` backend, which on ROCm **is RCCL** (collectives
  over xGMI); ``gloo`` stays gloo (CPU plumbing config). Without a GPU every
  name falls back to gloo so the CPU world_size>=1 path runs anywhere.
* the device is bound from ``LOCAL_RANK`` *before* any model placement;
* rendezvous is the standard ``env://`` (RANK / WORLD_SIZE / MASTER_ADDR /
  MASTER_PORT from torchrun or SageMaker), with ``MASTER_ADDR`` defaulting to
  127.0.0.1 for single-node runs.
"""
from __future__ import annotations

import datetime
import os
from typing import Optional, Tuple

import torch
import torch.distributed as dist

from ml_trainer_amd.utils.logging import get_logger

logger = get_logger("ml_trainer_amd.parallel")

_GPU_BACKENDS = {"smddp", "rccl", "nccl"}


def resolve_backend(name: Optional[str], have_gpu: bool) -> str:
    n = (name or "smddp").lower()
    if n in _GPU_BACKENDS:
        return "nccl" if have_gpu else "gloo"
    if n == "gloo":
        return "gloo"
    raise ValueError(f"unsupported distributed backend {name!r} (use smddp|rccl|nccl|gloo)")


def local_rank() -> int:
    return int(os.environ.get("LOCAL_RANK", os.environ.get("SLURM_LOCALID", "0")))


def set_sync_spin(device_index: int) -> bool:
    """Make host waits on ``device_index`` spin instead of yield (``hipDeviceScheduleSpin``; ROCm's
    default heuristic yields when the host has more cores than HIP contexts). Must run before the
    device's context is active -- i.e. before the first tensor / stream / graph on it. Opt out with
    MLT_SYNC_SPIN=0. Returns whether the flag took effect."""
    if os.environ.get("MLT_SYNC_SPIN", "1") == "0":
        return False
    try:
        from ml_trainer_amd.ops._ext import native_available, require_native
        if not native_available():
            return False
        err = require_native().set_device_sync_spin(int(device_index))
    except Exception as e:  # pragma: no cover - best effort, never fatal
        logger.warning(f"spin sync not set: {e!r}")
        return False
    if err != 0:
        logger.warning(f"spin sync not set on device {device_index}: hipError {err}")
    return err == 0


def bind_device(prefer_gpu: bool = True) -> torch.device:
    """Select the device for this process (LOCAL_RANK-th GPU) before anything touches it."""
    if prefer_gpu and torch.cuda.is_available():
        # MLT_SAME_DEVICE=1: every rank on GPU 0 -- the rehearsal knob for exercising the multi-rank
        # paths on a one-GPU box (gloo group + MLT_XGMI_ALLOW_GLOO); never for real runs
        lr = 0 if os.environ.get("MLT_SAME_DEVICE") == "1" else local_rank()
        n = torch.cuda.device_count()
        if lr >= n:
            raise RuntimeError(f"LOCAL_RANK={lr} but only {n} GPUs are visible")
        set_sync_spin(lr)
        torch.cuda.set_device(lr)
        return torch.device("cuda", lr)
    return torch.device("cpu")


def init_distributed(backend: Optional[str] = None, timeout_s: float = 1800.0) -> Tuple[int, int, str]:
    """Initialise (or reuse) the default process group. Returns (rank, world, backend)."""
    if dist.is_initialized():
        return dist.get_rank(), dist.get_world_size(), dist.get_backend()
    have_gpu = torch.cuda.is_available()
    be = resolve_backend(backend, have_gpu)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29500")
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    kw = dict(backend=be, timeout=datetime.timedelta(seconds=timeout_s))
    if be == "nccl":
        dev = bind_device(True)
        kw["device_id"] = dev
    dist.init_process_group(**kw)
    if (backend or "smddp").lower() == "smddp":
        logger.info("smddp backend requested: using the native RCCL process group over xGMI" if be == "nccl"
                    else "smddp backend requested without GPUs: using gloo")
    return dist.get_rank(), dist.get_world_size(), be


def is_dist() -> bool:
    return dist.is_available() and dist.is_initialized()


def rank() -> int:
    return dist.get_rank() if is_dist() else 0


def world_size() -> int:
    return dist.get_world_size() if is_dist() else 1


def barrier() -> None:
    if is_dist():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def all_reduce_scalars(values, op: str = "sum", device=None):
    """All-reduce a small list of python floats in ONE collective (metrics)."""
    if not is_dist():
        return list(values)
    dev = device or (torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl"
                     else torch.device("cpu"))
    t = torch.tensor(list(values), dtype=torch.float64, device=dev)
    dist.all_reduce(t, op={"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op])
    return t.cpu().tolist()


def destroy() -> None:
    if is_dist():
        dist.destroy_process_group()
