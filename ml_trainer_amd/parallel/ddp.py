"""Native data-parallel wrapper: flat gradient buckets, all-reduce overlapped with backward.

Replaces the reference's ``torch.nn.parallel.DistributedDataParallel`` on the
SMDDP backend (``src/trainer.py:97-101``) and its dead manual
``_average_gradients`` helper (``src/trainer.py:152-158``):

* parameters and gradients live in ONE contiguous buffer
  (:class:`~ml_trainer_amd.utils.flat.FlatParams`), laid out in *reverse*
  registration order -- the order autograd produces gradients -- so each bucket
  is a contiguous slice that is all-reduced in place (no copy-in/out);
* a per-bucket countdown driven by ``post_accumulate_grad`` hooks launches the
  bucket's all-reduce (``async_op=True`` on RCCL's own stream, ordered after the
  producing kernels) as soon as its last gradient lands, so communication
  overlaps the rest of backward; the end-of-backward callback only waits;
* bucket sizing for xGMI: every MI355X has 7 point-to-point links of ~153 GB/s.
  A ring all-reduce moves 2(W-1)/W * M bytes per GPU; RCCL spreads rings over
  all links, so ~25-64 MB buckets are bandwidth-efficient while still starting
  early in backward; small models (LeNet: 248 KB) get exactly one bucket --
  latency-bound, so splitting it would only add collective launches;
* ``ReduceOp.AVG`` on RCCL (no separate divide kernel); gloo gets SUM + scale;
* ``no_sync()`` skips communication for gradient accumulation;
* ``mode='manual'``: one flat all-reduce after backward (the reference's
  ``_average_gradients`` semantics, non-overlapped; A/B baseline).

``state_dict()`` keys carry the ``module.`` prefix, exactly as the reference's
DDP checkpoints.
"""
from __future__ import annotations

import contextlib
from typing import List, Optional

import torch
import torch.distributed as dist
from torch import nn

from ml_trainer_amd.utils.flat import FlatParams

DEFAULT_BUCKET_MB = 32.0
DEFAULT_FIRST_BUCKET_MB = 4.0


class DistributedDataParallel(nn.Module):
    def __init__(self, module: nn.Module, process_group=None, bucket_cap_mb: Optional[float] = None,
                 first_bucket_mb: Optional[float] = None, broadcast_parameters: bool = True,
                 mode: str = "overlap", flat: Optional[FlatParams] = None):
        super().__init__()
        if mode not in ("overlap", "manual"):
            raise ValueError("mode must be 'overlap' or 'manual'")
        self.module = module
        self.process_group = process_group
        self.mode = mode
        self.world_size = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.backend = dist.get_backend(process_group) if dist.is_initialized() else "none"
        self.flat = flat if flat is not None else FlatParams(module.parameters(), reverse=True)
        self._bucket_cap = int((bucket_cap_mb or DEFAULT_BUCKET_MB) * 2 ** 20)
        self._first_cap = int((first_bucket_mb or DEFAULT_FIRST_BUCKET_MB) * 2 ** 20)
        self._build_buckets()
        self.require_sync = True
        self._works: List = []
        self._pending: List[int] = list(self._bucket_counts)
        self._launched: List[bool] = [False] * len(self._buckets)
        self._callback_queued = False
        self._hooks = []
        if mode == "overlap":
            for i, p in enumerate(self.flat.params):
                self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(i)))
            # fused backwards that accumulate straight into the flat gradient notify here instead
            self._direct_hooks = {id(p): self._make_hook(i) for i, p in enumerate(self.flat.params)}
            self.flat.grad_ready_hooks.append(lambda p: self._direct_hooks[id(p)](p))
        if broadcast_parameters and self.world_size > 1:
            self.broadcast_state()

    # ------------------------------------------------------------------ buckets
    def _build_buckets(self) -> None:
        fp = self.flat
        esz = fp.data.element_size()
        buckets, counts, pb = [], [], []
        start, cnt, cap = 0, 0, self._first_cap
        for i, (p, o) in enumerate(zip(fp.params, fp.offsets)):
            end = o + p.numel()
            pb.append(len(buckets))
            cnt += 1
            if (end - start) * esz >= cap:
                nxt = fp.offsets[i + 1] if i + 1 < len(fp.params) else fp.numel
                buckets.append((start, nxt))
                counts.append(cnt)
                start, cnt, cap = nxt, 0, self._bucket_cap
        if cnt:
            buckets.append((start, fp.numel))
            counts.append(cnt)
        if not buckets:
            buckets, counts = [(0, fp.numel)], [0]
        self._buckets = buckets
        self._bucket_counts = counts
        self._param_bucket = pb

    @property
    def bucket_sizes_bytes(self) -> List[int]:
        esz = self.flat.grad.element_size()
        return [(e - s) * esz for s, e in self._buckets]

    # ------------------------------------------------------------------ comm
    def broadcast_state(self, src: int = 0) -> None:
        """Initial parameter/buffer broadcast from rank 0 (reference X3)."""
        dist.broadcast(self.flat.data, src=src, group=self.process_group)
        for b in self.module.buffers():
            dist.broadcast(b, src=src, group=self.process_group)

    def _reduce_bucket(self, bi: int, async_op: bool = True):
        s, e = self._buckets[bi]
        view = self.flat.grad[s:e]
        if self.backend == "nccl":
            return dist.all_reduce(view, op=dist.ReduceOp.AVG, group=self.process_group, async_op=async_op)
        w = dist.all_reduce(view, op=dist.ReduceOp.SUM, group=self.process_group, async_op=async_op)
        return (w, view)

    def _make_hook(self, i: int):
        def hook(p):
            if not self.require_sync or self.world_size == 1:
                return
            if not self._callback_queued:
                torch.autograd.Variable._execution_engine.queue_callback(self._finish)
                self._callback_queued = True
            b = self._param_bucket[i]
            self._pending[b] -= 1
            if self._pending[b] == 0 and not self._launched[b]:
                self._launched[b] = True
                self._works.append(self._reduce_bucket(b))
        return hook

    def _finish(self) -> None:
        # buckets whose params got no gradient this step (unused params): reduce them now
        for b in range(len(self._buckets)):
            if not self._launched[b] and self._bucket_counts[b] > 0:
                self._launched[b] = True
                self._works.append(self._reduce_bucket(b))
        self._wait_all()

    def _wait_all(self) -> None:
        for w in self._works:
            if isinstance(w, tuple):
                w[0].wait()
                w[1].mul_(1.0 / self.world_size)
            else:
                w.wait()
        self._works.clear()
        self._pending = list(self._bucket_counts)
        self._launched = [False] * len(self._buckets)
        self._callback_queued = False

    def sync_gradients(self) -> None:
        """Manual mode (or after no_sync accumulation): all-reduce the whole flat gradient."""
        if self.world_size == 1:
            return
        if self.backend == "nccl":
            dist.all_reduce(self.flat.grad, op=dist.ReduceOp.AVG, group=self.process_group)
        else:
            dist.all_reduce(self.flat.grad, group=self.process_group)
            self.flat.grad.mul_(1.0 / self.world_size)

    @contextlib.contextmanager
    def no_sync(self):
        old = self.require_sync
        self.require_sync = False
        try:
            yield
        finally:
            self.require_sync = old

    # ------------------------------------------------------------------ module
    def forward(self, *args, **kwargs):
        if self.flat.rebind_params():
            pass  # something replaced p.data (e.g. .to()); views restored
        return self.module(*args, **kwargs)

    def after_backward(self) -> None:
        """Call after ``loss.backward()``: in manual mode performs the flat all-reduce."""
        if self.mode == "manual" and self.require_sync:
            self.sync_gradients()
