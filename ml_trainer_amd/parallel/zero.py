"""ZeRO-1 data parallelism: reduce-scattered gradients, sharded optimizer state, all-gathered weights.

The reference has only replicated DDP (``src/trainer.py:97-101``; SURVEY.md §2.5 lists a
ZeRO-1 style sharded optimizer as the natural extension of flat buffers). This module builds it
on the same flat-buffer / reverse-order bucket machinery as :mod:`ml_trainer_amd.parallel.ddp`:

* every bucket ``[s, e)`` of the flat gradient is split into W equal chunks; when the bucket's
  last gradient lands (overlapped with backward, exactly like DDP) it is
  ``reduce_scatter``-ed so rank r receives the averaged chunk r -- the same bytes on the wire as
  half an all-reduce;
* rank r's chunks of all buckets are packed into ONE contiguous shard (:class:`ShardView`): fp32
  master copy, averaged gradient, and the optimizer state (``exp_avg`` / ``exp_avg_sq`` ...) exist
  only for the shard, so optimizer memory and optimizer time shrink by W and the fused optimizer
  is still a single launch (``csrc/kernels/optim.hip``) over a contiguous buffer;
* after the step each bucket's updated chunk is ``all_gather``-ed back into the replicated flat
  parameter buffer (the other half of the all-reduce bytes), the bf16 shadow used by the GEMMs is
  re-cast once, and ``generation`` is bumped so derived weight copies (fp8 casts) are rebuilt.
  The gathers are issued asynchronously right after the step and waited on at the next forward.

xGMI sizing: reduce-scatter + all-gather move the same 2(W-1)/W * M bytes per GPU as the ring
all-reduce of DDP, so the bucket sizes tuned for 7 point-to-point links carry over unchanged.
The flat buffer is laid out with ``align = 16 * W`` so every chunk is a multiple of 16 fp32
(float4 accesses, 64-byte aligned chunk starts) for any world size.

Optimizer state checkpoints are gathered into the full flat layout (collective: every rank must
call ``state_dict()``); loading slices the local shard back out. The layout depends on W.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
import torch.distributed as dist
from torch import nn

from ml_trainer_amd.parallel.ddp import DistributedDataParallel
from ml_trainer_amd.utils.flat import FlatParams


class ShardView:
    """This rank's contiguous shard of a :class:`FlatParams`, duck-typed so the fused optimizers
    (``ops/optim.py``) run over it unchanged. ``chunks[i] = (s, e, so, c)``: bucket ``[s, e)`` of
    the full buffer, this rank's chunk ``[s + rank*c, s + (rank+1)*c)`` lives at ``[so, so + c)``."""

    def __init__(self, full: FlatParams, chunks: List[Tuple[int, int, int, int]], rank: int, world: int,
                 process_group=None):
        self.full = full
        self.params = full.params
        self.device = full.device
        self.chunks = chunks
        self.rank, self.world, self.process_group = rank, world, process_group
        self.numel = sum(c for _, _, _, c in chunks)
        if world == 1:  # nothing to shard: the shard IS the replicated buffer
            self.data, self.grad = full.data, full.grad
        else:
            self.data = torch.empty(self.numel, dtype=full.data.dtype, device=self.device)
            self.grad = torch.zeros(self.numel, dtype=full.grad.dtype, device=self.device)
        self.generation = 0
        self.grad_ready_hooks: List = []
        self.load_from_full()

    # ---- FlatParams duck-typing used by FusedOptimizer.step -------------------------------
    def rebind_params(self) -> bool:
        return False

    def rebind_grads(self) -> None:
        self.full.rebind_grads()

    def zero_grad(self) -> None:
        self.full.zero_grad()
        if self.world > 1:
            self.grad.zero_()

    # bf16 shadow: with world > 1 the replicated buffer's shadow is re-cast after the all-gather;
    # with world 1 the shard IS the replicated buffer, so the fused optimizer rewrites its shadow
    # directly (a native kernel does not bump data._version, so a lazily refreshed shadow would
    # otherwise go stale)
    @property
    def shadow(self):
        return self.full.shadow if self.world == 1 else None

    @property
    def _shadow_ver(self) -> int:
        return self.full._shadow_ver if self.world == 1 else -1

    def mark_shadow_fresh(self) -> None:
        if self.world == 1:
            self.full.mark_shadow_fresh()

    # ---- shard <-> full -------------------------------------------------------------------
    def local_slices(self):
        for s, e, so, c in self.chunks:
            yield slice(s + self.rank * c, s + (self.rank + 1) * c), slice(so, so + c)

    @torch.no_grad()
    def load_from_full(self) -> None:
        """Copy this rank's chunks of the replicated parameters into the shard master
        (construction, and after anything rewrote the replicated weights, e.g. a resume)."""
        if self.world == 1:
            return
        for fs, ss in self.local_slices():
            self.data[ss].copy_(self.full.data[fs])

    def gather_into(self, out: torch.Tensor, shard: torch.Tensor, async_op: bool = False):
        """All-gather ``shard`` (this rank's chunks) into the full-layout tensor ``out``."""
        nc = getattr(self, "ncomm", None)
        if nc is not None and out.is_cuda:
            # native RCCL all-gathers: on the comm stream (after a hipEvent edge from the
            # compute stream) when asynchronous, else on the current stream
            cs = self.comm_stream if async_op else None
            if cs is not None:
                ready = torch.cuda.Event()
                ready.record()
                with torch.cuda.stream(cs):
                    cs.wait_event(ready)
                    for s, e, so, c in self.chunks:
                        nc.all_gather(shard[so:so + c], out[s:e])
                return [_StreamDone(cs)]
            for s, e, so, c in self.chunks:
                nc.all_gather(shard[so:so + c], out[s:e])
            return []
        if out.is_cuda and dist.get_backend(self.process_group) != "nccl":
            # gloo rehearsal of the GPU path (several ranks on one GPU): stage through the host
            host = out.cpu()
            self.gather_into(host, shard.cpu())
            out.copy_(host)
            return []
        works = []
        for s, e, so, c in self.chunks:
            works.append(dist.all_gather_into_tensor(out[s:e], shard[so:so + c], group=self.process_group,
                                                     async_op=async_op))
        return works

    def export_state(self, shard: torch.Tensor) -> torch.Tensor:
        """Collective: the full-layout copy (on CPU) of a shard-sized state tensor."""
        coll = shard if dist.get_backend(self.process_group) == "nccl" else shard.cpu()
        full = torch.zeros(self.full.numel, dtype=shard.dtype, device=coll.device)
        self.gather_into(full, coll)
        return full.cpu()

    def import_state(self, full: torch.Tensor, shard: torch.Tensor) -> None:
        full = full.to(shard.device)
        if full.numel() != self.full.numel:
            raise ValueError(f"ZeRO optimizer state has {full.numel()} elements, this layout {self.full.numel}"
                             " (saved with a different world size?)")
        for fs, ss in self.local_slices():
            shard[ss].copy_(full[fs])


class _Done:
    def wait(self) -> None:
        pass


class _StreamDone:
    """``wait()`` makes the current (compute) stream wait for the comm stream -- no host block."""

    def __init__(self, stream):
        self.stream = stream

    def wait(self) -> None:
        torch.cuda.current_stream(self.stream.device).wait_stream(self.stream)


class ZeroDataParallel(DistributedDataParallel):
    """DDP with ZeRO stage-1 optimizer sharding. Usage::

        model = ZeroDataParallel(module)
        opt = model.make_optimizer(FusedAdamW, lr=1e-4)   # or build_optimizer(..., flat=model.shard)
        loss(model(x)).backward(); opt.step()

    ``make_optimizer`` / :meth:`attach_optimizer` register the post-step all-gather."""

    def __init__(self, module: nn.Module, process_group=None, bucket_cap_mb: Optional[float] = None,
                 first_bucket_mb: Optional[float] = None, broadcast_parameters: bool = True,
                 mode: str = "overlap", comm=None):
        world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        rank = dist.get_rank(process_group) if dist.is_initialized() else 0
        if comm is not None and comm is not False:  # an explicit native communicator sets the layout
            world, rank = int(comm.size), int(comm.rank)
        dev = next((p.device for p in module.parameters()), torch.device("cpu"))
        flat = FlatParams(module.parameters(), device=dev, reverse=True, align=16 * max(world, 1))
        # auto_plan=False: the shard layout (chunks, sharded optimizer state) is fixed by the
        # buckets built here, so the buckets must never be re-planned after construction
        super().__init__(module, process_group=process_group, bucket_cap_mb=bucket_cap_mb,
                         first_bucket_mb=first_bucket_mb, broadcast_parameters=broadcast_parameters,
                         mode=mode, flat=flat, comm=comm, auto_plan=False)
        chunks, so = [], 0
        for s, e in self._buckets:
            assert (e - s) % world == 0, "bucket not divisible by the world size"
            c = (e - s) // world
            chunks.append((s, e, so, c))
            so += c
        self.shard = ShardView(self.flat, chunks, rank, world, process_group)
        self.shard.ncomm = self._ncomm
        self.shard.comm_stream = self._comm_stream
        self._gather_works: List = []

    def _maybe_replan(self) -> None:
        """Never: the shard chunks and the optimizer's sharded state follow the construction-time
        buckets (a re-plan would reduce-scatter wrong ranges)."""
        self._auto_plan = False

    # ---- gradients: reduce-scatter instead of all-reduce ------------------------------------
    def _reduce_bucket(self, bi: int, async_op: bool = True):
        s, e, so, c = self.shard.chunks[bi]
        out = self.shard.grad[so:so + c]
        inp = self.flat.grad[s:e]
        if self._ncomm is not None:  # native RCCL on the comm stream, after the bucket's producers
            cs = self._comm_stream
            ready = torch.cuda.Event()
            ready.record()
            with torch.cuda.stream(cs):
                cs.wait_event(ready)
                self._ncomm.reduce_scatter(inp, out, "avg")
            return None
        if self.backend == "nccl":
            return dist.reduce_scatter_tensor(out, inp, op=dist.ReduceOp.AVG, group=self.process_group,
                                              async_op=async_op)
        if inp.is_cuda:  # gloo rehearsal on a GPU: host staging, synchronous
            host = torch.empty(c, dtype=out.dtype)
            dist.reduce_scatter_tensor(host, inp.cpu(), op=dist.ReduceOp.SUM, group=self.process_group)
            out.copy_(host.mul_(1.0 / self.world_size))
            return _Done()
        w = dist.reduce_scatter_tensor(out, inp, op=dist.ReduceOp.SUM, group=self.process_group,
                                       async_op=async_op)
        return (w, out)

    def sync_gradients(self) -> None:
        if self.world_size == 1 and self._ncomm is None:
            return  # the shard aliases the full gradient
        self._works.extend(self._reduce_bucket(b) for b in range(len(self._buckets)))
        if self._ncomm is not None:
            torch.cuda.current_stream(self.flat.device).wait_stream(self._comm_stream)
        self._wait_all()

    # ---- parameters: all-gather after the optimizer step --------------------------------------
    def attach_optimizer(self, optimizer: torch.optim.Optimizer) -> torch.optim.Optimizer:
        optimizer.register_step_post_hook(lambda opt, args, kwargs: self.gather_parameters())
        return optimizer

    def make_optimizer(self, cls, **kwargs) -> torch.optim.Optimizer:
        return self.attach_optimizer(cls(self.module.parameters(), flat=self.shard, **kwargs))

    @torch.no_grad()
    def gather_parameters(self, async_op: bool = True) -> None:
        if self.world_size > 1 or self._ncomm is not None:
            self._gather_works.extend(self.shard.gather_into(self.flat.data, self.shard.data, async_op=async_op))
        self.flat.generation += 1
        if not async_op:
            self.wait_parameters()

    def wait_parameters(self) -> None:
        if not self._gather_works:
            return
        for w in self._gather_works:
            w.wait()
        self._gather_works.clear()
        if self.flat.shadow is not None:
            self.flat._shadow_ver = -1  # the gathered master is new: re-cast the bf16 copy once
            self.flat.refresh_shadow()

    def forward(self, *args, **kwargs):
        self.wait_parameters()
        return super().forward(*args, **kwargs)

    def clip_grad_norm_(self, max_norm: float) -> torch.Tensor:
        """Global-norm clipping over the sharded (already averaged) gradient."""
        g = self.shard.grad
        sq = (g.double() * g.double()).sum().float().view(1)
        if self.world_size > 1:
            coll = sq if self.backend == "nccl" else sq.cpu()
            dist.all_reduce(coll, group=self.process_group)
            sq = coll.to(g.device)
        total = sq.sqrt()
        g.mul_(torch.clamp(max_norm / (total + 1e-6), max=1.0))
        return total.view(())

    def optimizer_state_bytes(self, optimizer) -> int:
        n = 0
        for gi in range(len(optimizer.param_groups)):
            for b in optimizer.state_buffers(gi):
                if b is not None:
                    n += b.numel() * b.element_size()
        return n

    def state_dict(self, *args, **kwargs):
        self.wait_parameters()  # checkpoints must see the gathered weights
        return super().state_dict(*args, **kwargs)
