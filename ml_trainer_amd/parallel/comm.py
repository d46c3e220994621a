"""Native RCCL communicator (csrc/comm/comm.cpp) for one-process-per-GPU jobs.

The reference reaches its collectives through SMDDP's process group
(``src/trainer.py:43-44,59``). Here the torch.distributed process
group is only the rendezvous: rank 0 draws an RCCL unique id, it travels through
the existing group (``broadcast_object_list``), and every rank builds its own
``ncclComm`` on its GPU. Collectives are enqueued on the caller's current HIP
stream, so they order with compute without events and can be captured inside a
hipGraph together with a whole training step (``LeNetStepEngine``).

``MLT_NATIVE_COMM=0`` disables it (callers fall back to torch.distributed).
"""
from __future__ import annotations

import os
from typing import Optional

import torch


def native_comm_enabled() -> bool:
    return os.environ.get("MLT_NATIVE_COMM", "1") != "0"


def create_native_comm(process_group=None, device: Optional[torch.device] = None):
    """Collective over ``process_group``: returns a ``_C.Communicator`` bound to ``device``
    (default: the current CUDA device), or None when not applicable (CPU, world size 1,
    disabled). Raises if RCCL initialisation fails on some rank."""
    import torch.distributed as dist
    if not native_comm_enabled() or not torch.cuda.is_available():
        return None
    if not dist.is_available() or not dist.is_initialized():
        return None
    world = dist.get_world_size(process_group)
    if world < 2 or dist.get_backend(process_group) != "nccl":
        return None  # gloo (CPU / tests) keeps torch.distributed; RCCL needs one GPU per rank
    from ml_trainer_amd.ops._ext import require_native
    C = require_native()
    rank = dist.get_rank(process_group)
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    obj = [C.Communicator.unique_id() if rank == 0 else None]
    src = 0 if process_group is None else dist.get_global_rank(process_group, 0)
    dist.broadcast_object_list(obj, src=src, group=process_group, device=dev)
    return C.Communicator(obj[0], world, rank, dev.index)
