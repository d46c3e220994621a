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


def xgmi_enabled() -> bool:
    return os.environ.get("MLT_XGMI_AR", "1") != "0"


def create_xgmi_allreduce(process_group=None, capacity: int = 0, device: Optional[torch.device] = None,
                          allow_gloo: Optional[bool] = None):
    """One-shot / two-shot xGMI all-reduce (csrc/kernels/allreduce.hip) for vectors of <=
    ``capacity`` fp32 (``.algo`` 0 / 1; the LeNet engine picks by a timed vote).

    Collective. IPC handles of every rank's uncached region travel through the process group;
    a self-test (sum of rank-dependent vectors, bit-exact, bounded wait) must pass on EVERY rank
    or all ranks get None and keep RCCL. Ranks must share one node (world <= 8)."""
    import torch.distributed as dist
    if allow_gloo is None:  # rehearsal of the multi-GPU path with several ranks on one GPU (tests)
        allow_gloo = os.environ.get("MLT_XGMI_ALLOW_GLOO") == "1"
    if not xgmi_enabled() or not torch.cuda.is_available() or not dist.is_initialized():
        return None
    world = dist.get_world_size(process_group)
    if world < 2 or world > 8:
        return None
    if dist.get_backend(process_group) != "nccl" and not allow_gloo:
        return None
    from ml_trainer_amd.ops._ext import require_native
    C = require_native()
    rank = dist.get_rank(process_group)
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    coll_dev = dev if dist.get_backend(process_group) == "nccl" else torch.device("cpu")
    x, ok = None, True
    try:
        x = C.XgmiAllReduce(int(capacity), world, rank, dev.index)
        # a timeout is fatal (sticky error word -> TransportError), and ranks are not lined up
        # before the first replay of a step graph (each builds its dataset / captures its graphs):
        # generous by default; dead peers are the watchdog's job (600 s)
        x.timeout_ms = int(os.environ.get("MLT_XGMI_TIMEOUT_MS", "30000"))
        h = x.handle()
    except RuntimeError:
        ok, h = False, b""
    hs = [None] * world
    dist.all_gather_object(hs, h, group=process_group)
    if ok and all(len(v) > 0 for v in hs):
        try:
            x.open(hs)
        except RuntimeError:
            ok = False
    else:
        ok = False
    flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=coll_dev)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=process_group)
    if int(flag.item()) == 0:
        return None
    # self-test of both algorithms (one-shot, then two-shot). A peer timeout (sticky error word)
    # disqualifies the object; wrong two-shot sums only disqualify the two-shot algorithm
    # (x.two_shot_ok), every rank agreeing through the MIN vote.
    n = max(4, min(int(capacity), 1 << 16))
    n -= 1 - n % 2  # odd length: tail handling
    good = [True, True]
    for algo in (0, 1):
        x.algo = algo
        good[algo] = _xgmi_selftest(x, world, rank, n, dev)
    x.algo = 0
    ok = x.error() == 0
    flag = torch.tensor([1 if (ok and good[0]) else 0, 1 if (ok and good[1]) else 0], dtype=torch.int32,
                        device=coll_dev)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=process_group)
    one, two = (int(v) for v in flag.tolist())
    if one != 1:
        return None
    x.two_shot_ok = two == 1
    # fault injection for the bring-up tests: MLT_XGMI_INJECT_FAULT="rank:code" sets x.fault = code
    # on that rank after the one-/two-shot self-tests (2: the fused exchange publishes corrupted
    # values -- its own self-test must then reject it on every rank)
    inj = os.environ.get("MLT_XGMI_INJECT_FAULT", "")
    if inj:
        r, code = (int(v) for v in inj.split(":"))
        if r == rank:
            x.fault = code
    return x


def _payload(q: int, it: int, n: int) -> torch.Tensor:
    """Rank q's random fp32 test payload of round ``it`` (any rank can regenerate any peer's)."""
    g = torch.Generator().manual_seed(0x5EED + 7919 * q + 104729 * it)
    return torch.randn(n, generator=g, dtype=torch.float32) * torch.exp2(torch.randint(-8, 9, (n,), generator=g)).float()


def _xgmi_selftest(x, world: int, rank: int, n: int, dev, rounds: int = 12) -> bool:
    """Visibility test of the current algorithm on the real fabric, every word checked:
    (1) two launches with exact small-integer sums (both buffer parities);
    (2) ``rounds`` back-to-back launches of random fp32 payloads (no synchronisation between
        them, so parity reuse runs at full speed) while a side stream keeps the GPU busy with
        GEMMs (uneven load), each result compared bitwise with the host sum in RANK ORDER --
        what every rank's kernel computes. A stale peer read anywhere fails the test, and the
        caller then keeps RCCL instead of training on stale data."""
    ok = True
    for it in range(2):
        t = torch.arange(n, dtype=torch.float32, device=dev).remainder_(97).add_(rank + 1 + it)
        x.all_reduce(t, average=False)
        ref = torch.arange(n, dtype=torch.float32, device=dev).remainder_(97) * world + (
            world * (world + 1) // 2 + it * world)
        torch.cuda.synchronize(dev)
        ok = ok and bool(torch.equal(t, ref))
    bufs = [_payload(rank, it, n).to(dev) for it in range(rounds)]
    side = torch.cuda.Stream(dev)
    a = torch.randn(2048, 2048, device=dev)
    torch.cuda.synchronize(dev)
    with torch.cuda.stream(side):  # load on the chip while the exchanges run
        for _ in range(8):
            a = torch.tanh(a @ a * 1e-3)
    for t in bufs:
        x.all_reduce(t, average=False)
    torch.cuda.synchronize(dev)
    for it, t in enumerate(bufs):
        ref = _payload(0, it, n)
        for q in range(1, world):
            ref = ref + _payload(q, it, n)  # rank order, fp32: bit-identical to the kernels' sums
        ok = ok and bool(torch.equal(t.cpu(), ref))
    return ok and x.error() == 0


def create_xgmi_loopback(capacity: int, device: Optional[torch.device] = None, timeout_ms: int = 30000):
    """A one-rank xGMI transport whose only peer is this rank itself: times the data-parallel
    step's exchange (publish, flag, poll, pull, rank-ordered sum) on a single GPU."""
    from ml_trainer_amd.ops._ext import require_native
    C = require_native()
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    x = C.XgmiAllReduce(int(capacity), 1, 0, dev.index)
    x.timeout_ms = int(timeout_ms)
    x.open([x.handle()])
    return x
