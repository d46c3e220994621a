"""Native data-parallel wrapper: flat gradient buckets, all-reduce overlapped with backward.

Replaces the reference's ``torch.nn.parallel.DistributedDataParallel`` on the
SMDDP backend (``src/trainer.py:97-101``) and its dead manual
``_average_gradients`` helper (``src/trainer.py:152-158``):

* parameters and gradients live in ONE contiguous buffer
  (:class:`~ml_trainer_amd.utils.flat.FlatParams`), laid out in *reverse*
  registration order -- the order autograd produces gradients -- so each bucket
  is a contiguous slice that is all-reduced in place (no copy-in/out);
* a per-bucket countdown driven by ``post_accumulate_grad`` hooks launches the
  bucket's all-reduce as soon as its last gradient lands, so communication overlaps
  the rest of backward;
* GPU jobs on RCCL (``backend="nccl"``, W > 1) reduce through the NATIVE communicator
  (csrc/comm/comm.cpp, ``ncclAllReduce`` AVG) enqueued on a dedicated high-priority HIP
  comm stream: a hipEvent recorded on the compute stream when the bucket is ready, the
  comm stream waits on it, the collective runs there, and the end-of-backward callback
  makes the compute stream wait on the comm stream -- the host never blocks on a
  collective and torch.distributed is only the rendezvous (the unique id travels over it);
  ``comm=False`` keeps ``torch.distributed`` collectives instead (CPU / gloo always do);
* bucket sizing for xGMI: every MI355X has 7 point-to-point links of ~153 GB/s.
  A ring all-reduce moves 2(W-1)/W * M bytes per GPU; RCCL spreads rings over
  all links, so ~25-64 MB buckets are bandwidth-efficient while still starting
  early in backward; small models (LeNet: 248 KB) get exactly one bucket --
  latency-bound, so splitting it would only add collective launches;
* ``ReduceOp.AVG`` on RCCL (no separate divide kernel); gloo gets SUM + scale;
* ``no_sync()`` skips communication for gradient accumulation;
* ``mode='manual'``: one flat all-reduce after backward (the reference's
  ``_average_gradients`` semantics, non-overlapped; A/B baseline);
* ``comm_dtype=torch.bfloat16``: each bucket is cast into a persistent bf16 image, reduced
  in bf16 (half the xGMI bytes: BERT-base 220 MB instead of 440 MB per step) and cast back
  into the fp32 gradient; the fp32 masters and the optimizer are unchanged;
* ``timing=True``: hipEvents around every bucket's collective (on a dedicated high-priority
  comm stream) and around forward/backward; :meth:`comm_stats` reports all-reduce device
  time, the share of it hidden under backward (``overlap_pct``) and the bucket layout
  (SURVEY.md §5.1 / §7.6 "all-reduce time, overlap %").

``state_dict()`` keys carry the ``module.`` prefix, exactly as the reference's
DDP checkpoints.
"""
from __future__ import annotations

import contextlib
import os
from typing import Dict, List, Optional

import torch
import torch.distributed as dist
from torch import nn

from ml_trainer_amd.utils.flat import FlatParams

DEFAULT_BUCKET_MB = 32.0
DEFAULT_FIRST_BUCKET_MB = 4.0

# alpha-beta model of one bucket's ring all-reduce on an 8 x MI355X node (RCCL over xGMI):
#   t(M) = ALPHA + 2 (W - 1) / W * M / BUS
# ALPHA: per-collective launch + protocol latency; BUS: the all-reduce's bus bandwidth with RCCL's
# rings spread over the 7 point-to-point links (~153 GB/s each). These are the model's priors: the
# one-time re-plan fits both on the live process group (DistributedDataParallel._measure_alpha_beta:
# timed all-reduces of two sizes, MAX over ranks); MLT_DDP_ALPHA_US / MLT_DDP_BUS_GBPS override the
# fit (e.g. from scripts/bucket_sweep.sh), MLT_DDP_MEASURE_AB=0 keeps the priors.
XGMI_ALPHA_US = 25.0
XGMI_BUS_GBPS = 300.0
MIN_BUCKET_MB, MAX_BUCKET_MB = 4.0, 128.0


def allreduce_us(nbytes: float, world: int, alpha_us: Optional[float] = None, bus_gbps: Optional[float] = None) -> float:
    """Model time (us) of one ring all-reduce of ``nbytes`` over ``world`` ranks."""
    import os
    a = alpha_us if alpha_us is not None else float(os.environ.get("MLT_DDP_ALPHA_US", XGMI_ALPHA_US))
    b = bus_gbps if bus_gbps is not None else float(os.environ.get("MLT_DDP_BUS_GBPS", XGMI_BUS_GBPS))
    if world <= 1:
        return 0.0
    return a + 2.0 * (world - 1) / world * nbytes / (b * 1e3)  # GB/s = 1e3 bytes/us


def _min_bucket_mb() -> float:
    import os
    return float(os.environ.get("MLT_DDP_MIN_BUCKET_MB", MIN_BUCKET_MB))


def plan_buckets(grad_bytes: int, world: int, bwd_ms: Optional[float] = None, largest_param_bytes: int = 0,
                 alpha_us: Optional[float] = None, bus_gbps: Optional[float] = None):
    """Bucket caps (cap_mb, first_mb) from the alpha-beta model. Buckets launched during backward
    overlap it as long as the comm stream keeps up: n * ALPHA + beta * M <= T_bwd; what stays exposed
    is the last bucket's all-reduce (ALPHA + beta * C_last). So the cap is the SMALLEST that keeps
    the stream from falling behind -- C = M * ALPHA / (T_bwd - beta * M) -- clamped to
    [MIN, 128] MB (MIN = 4, MLT_DDP_MIN_BUCKET_MB); a comm-bound step (beta * M >= T_bwd) gets the
    largest cap (fewest collectives). The first bucket (the last layers' gradients, ready first)
    is the size at which the all-reduce stops being latency-bound -- beta * F = ALPHA, so smaller
    would not start the wire earlier and larger would delay it -- clamped to [1 MB, cap].
    Without a backward-time estimate: the defaults (32 / 4 MB)."""
    if world <= 1 or bwd_ms is None or bwd_ms <= 0:
        return DEFAULT_BUCKET_MB, DEFAULT_FIRST_BUCKET_MB
    a = allreduce_us(0, world, alpha_us, bus_gbps)  # alpha alone
    total_us = allreduce_us(grad_bytes, world, alpha_us, bus_gbps) - a  # beta * M
    slack = bwd_ms * 1e3 - total_us
    mb = 2 ** 20
    if slack <= a:
        cap = MAX_BUCKET_MB
    else:
        cap = grad_bytes * a / slack / mb
    cap = min(MAX_BUCKET_MB, max(_min_bucket_mb(), cap))
    beta_us_per_byte = total_us / grad_bytes if grad_bytes > 0 else 0.0
    first = a / beta_us_per_byte / mb if beta_us_per_byte > 0 else DEFAULT_FIRST_BUCKET_MB
    first = min(cap, max(min(1.0, cap), first))
    return cap, first


class DistributedDataParallel(nn.Module):
    def __init__(self, module: nn.Module, process_group=None, bucket_cap_mb: Optional[float] = None,
                 first_bucket_mb: Optional[float] = None, broadcast_parameters: bool = True,
                 mode: str = "overlap", flat: Optional[FlatParams] = None,
                 comm_dtype: Optional[torch.dtype] = None, timing: bool = False, comm=None,
                 bwd_ms_hint: Optional[float] = None, auto_plan: Optional[bool] = None):
        """``comm``: None = native RCCL communicator when the group is RCCL with W > 1 (else
        torch.distributed); False = always torch.distributed; a ``_C.Communicator`` = use that
        one (also at world size 1: the single-GPU rehearsal of the native collective path).
        ``bwd_ms_hint``: expected backward time; with no explicit caps the buckets are then sized
        by the alpha-beta model (:func:`plan_buckets`). ``auto_plan`` (default: on when neither
        caps nor a hint are given, W > 1, overlap mode; MLT_DDP_AUTOPLAN=0 turns it off): the
        second synchronised backward is timed (first gradient hook -> last gradient; device
        events on GPU); at the end of that backward, once its collectives are waited for, the
        MAX over ranks is agreed and the buckets are rebuilt ONCE from the alpha-beta model with
        that time (``bucket_plan["source"]`` = "alpha-beta", ``"bwd_ms"`` the agreed time). The
        re-plan is COLLECTIVE (a MAX all-reduce + the alpha-beta fit's timed all-reduces): it runs
        at the end of the second synchronised backward, which every rank reaches in the same order
        (``replan()`` runs it explicitly)."""
        super().__init__()
        if mode not in ("overlap", "manual"):
            raise ValueError("mode must be 'overlap' or 'manual'")
        self.module = module
        self.process_group = process_group
        self.mode = mode
        self.world_size = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.backend = dist.get_backend(process_group) if dist.is_initialized() else "none"
        self.flat = flat if flat is not None else FlatParams(module.parameters(), reverse=True)
        self._ncomm = None
        if comm is not None and comm is not False:
            self._ncomm = comm
            self.world_size = int(comm.size)
        elif comm is None and self.flat.device.type == "cuda" and self.world_size > 1:
            self._ncomm = self._native_comm_agreed(process_group)
        self.comm_backend = "native-rccl" if self._ncomm is not None else f"torch.distributed-{self.backend}"
        esz = 2 if comm_dtype == torch.bfloat16 else self.flat.grad.element_size()
        plan_cap, plan_first = plan_buckets(self.flat.numel * esz, self.world_size, bwd_ms_hint)
        self.bucket_plan = {"cap_mb": bucket_cap_mb or plan_cap, "first_mb": first_bucket_mb or plan_first,
                            "source": "explicit" if bucket_cap_mb else ("alpha-beta" if bwd_ms_hint else "default"),
                            "replans": 0}
        import os
        if auto_plan is None:
            auto_plan = (bucket_cap_mb is None and first_bucket_mb is None and bwd_ms_hint is None
                         and os.environ.get("MLT_DDP_AUTOPLAN", "1") != "0")
        self._auto_plan = bool(auto_plan) and mode == "overlap" and self.world_size > 1
        self._grad_bytes = self.flat.numel * esz
        self._synced_bwd = 0     # synchronised backwards seen
        self._bwd_t = None       # (start, end) of the timed backward: cuda events or host seconds
        self._bucket_cap = int(self.bucket_plan["cap_mb"] * 2 ** 20)
        self._first_cap = int(self.bucket_plan["first_mb"] * 2 ** 20)
        self._build_buckets()
        if comm_dtype is not None and comm_dtype not in (torch.float32, torch.bfloat16):
            raise ValueError("comm_dtype must be torch.float32 or torch.bfloat16")
        self.comm_dtype = comm_dtype if comm_dtype != self.flat.grad.dtype else None
        self._cbuf = (torch.zeros(self.flat.numel, dtype=self.comm_dtype, device=self.flat.device)
                      if self.comm_dtype is not None else None)
        self.timing = bool(timing)
        cuda = self.flat.device.type == "cuda"
        # native collectives, and collectives that need work of their own (casts, timing events),
        # run on a dedicated high-priority comm stream
        self._comm_stream = (torch.cuda.Stream(device=self.flat.device, priority=-1)
                             if cuda and (self._ncomm is not None or self.timing or self.comm_dtype is not None)
                             else None)
        self._step_rec: Optional[Dict] = None
        self._records: List[Dict] = []
        self.require_sync = True
        self._works: List = []
        self._pending: List[int] = list(self._bucket_counts)
        self._counted: List[bool] = [False] * len(self.flat.params)
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

    def _native_comm_agreed(self, process_group):
        """The native RCCL communicator on every rank, or on none: a bring-up failure on any rank
        (caught, warned) is agreed through a MIN vote, and then every rank keeps torch.distributed
        together (the LeNet engine's pattern, models/lenet_engine.py)."""
        import warnings
        from ml_trainer_amd.parallel.comm import create_native_comm, native_comm_enabled
        if not native_comm_enabled() or self.backend != "nccl":
            return None
        try:
            c = create_native_comm(process_group, self.flat.device)
        except RuntimeError as e:
            warnings.warn(f"native RCCL communicator unavailable ({e}); DDP uses torch.distributed")
            c = None
        ok = torch.tensor([1.0 if c is not None else 0.0], device=self.flat.device)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=process_group)
        return c if ok.item() == 1.0 else None

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
        if self._comm_stream is not None:
            return self._reduce_bucket_side(bi, view)
        if self._cbuf is not None:  # CPU / gloo with a narrower wire dtype: synchronous cast round trip
            cv = self._cbuf[s:e]
            cv.copy_(view)
            dist.all_reduce(cv, op=dist.ReduceOp.SUM, group=self.process_group)
            view.copy_(cv)
            view.mul_(1.0 / self.world_size)
            return None
        if self.backend == "nccl":
            return dist.all_reduce(view, op=dist.ReduceOp.AVG, group=self.process_group, async_op=async_op)
        w = dist.all_reduce(view, op=dist.ReduceOp.SUM, group=self.process_group, async_op=async_op)
        return (w, view)

    def _reduce_bucket_side(self, bi: int, view: torch.Tensor):
        """GPU bucket collective on the comm stream: wait for the producing kernels, [cast to the
        wire dtype], all-reduce (AVG), [cast back], with timing events around the collective. The
        host never blocks; ``_finish`` makes the compute stream wait for the comm stream."""
        s, e = self._buckets[bi]
        cs = self._comm_stream
        ready = torch.cuda.Event(enable_timing=self.timing)
        ready.record()
        rec = self._step_rec if self.timing else None
        with torch.cuda.stream(cs):
            cs.wait_event(ready)
            ev0 = torch.cuda.Event(enable_timing=True) if rec is not None else None
            if ev0 is not None:
                ev0.record(cs)
            buf = view
            if self._cbuf is not None:
                buf = self._cbuf[s:e]
                buf.copy_(view)
            if self._ncomm is not None:
                self._ncomm.all_reduce(buf, "avg")  # enqueued on the comm stream by C++
            else:
                op = dist.ReduceOp.AVG if self.backend == "nccl" else dist.ReduceOp.SUM
                w = dist.all_reduce(buf, op=op, group=self.process_group, async_op=True)
                w.wait()  # comm stream waits for the collective (no host block on RCCL)
                if self.backend != "nccl":
                    buf.mul_(1.0 / self.world_size)
            if buf is not view:
                view.copy_(buf)
            if rec is not None:
                ev1 = torch.cuda.Event(enable_timing=True)
                ev1.record(cs)
                rec["buckets"].append((bi, ready, ev0, ev1))
        return None

    def _make_hook(self, i: int):
        def hook(p):
            if not self.require_sync or (self.world_size == 1 and self._ncomm is None):
                return
            # A fused backward that wrote p's gradient straight into the flat buffer notifies here
            # (FlatParams.notify_grad_ready) AND autograd still runs p's AccumulateGrad node, whose
            # post-accumulate hook fires even for the None gradient the Function returned. Count
            # each parameter once per backward: a double count drains a bucket that spans two
            # fused blocks early and all-reduces it before the second block wrote its gradients.
            if self._counted[i]:
                return
            self._counted[i] = True
            if not self._callback_queued:
                torch.autograd.Variable._execution_engine.queue_callback(self._finish)
                self._callback_queued = True
                if self._auto_plan and self._synced_bwd == 1 and self._bwd_t is None:
                    self._bwd_t = [self._mark(), None]  # the second synced backward: timed
            b = self._param_bucket[i]
            self._pending[b] -= 1
            if self._pending[b] == 0 and not self._launched[b]:
                self._launched[b] = True
                self._works.append(self._reduce_bucket(b))
        return hook

    def _mark(self):
        if self.flat.device.type == "cuda":
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            return ev
        import time
        return time.perf_counter()

    def _measure_alpha_beta(self) -> Optional[tuple]:
        """Fit the alpha-beta model on this group's real wire: all-reduces of 64 KB (latency-bound) and
        min(max(M, 4 MB), 64 MB) (bandwidth-bound) through the same path the buckets take (native
        RCCL communicator or torch.distributed), each timed host-side around device syncs after
        a warmup; the MAX over ranks is agreed so every rank plans alike. Returns (alpha_us,
        bus_gbps), or None when the two points do not give a positive slope (then the priors stay)."""
        import time
        dev = self.flat.device
        cuda = dev.type == "cuda"
        dt = self.comm_dtype or self.flat.grad.dtype
        esz = torch.empty((), dtype=dt).element_size()
        small, large = 64 * 1024, int(min(max(self._grad_bytes, 4 * 2 ** 20), 64 * 2 ** 20))
        buf = torch.zeros(large // esz, dtype=dt, device=dev)

        def timed(nbytes: int, reps: int) -> float:
            v = buf[:max(1, nbytes // esz)]

            def once():
                if self._ncomm is not None:
                    self._ncomm.all_reduce(v, "avg")
                else:
                    dist.all_reduce(v, op=dist.ReduceOp.SUM, group=self.process_group)
            once()
            if cuda:
                torch.cuda.synchronize(dev)
            dist.barrier(group=self.process_group)
            t0 = time.perf_counter()
            for _ in range(reps):
                once()
            if cuda:
                torch.cuda.synchronize(dev)
            return (time.perf_counter() - t0) * 1e6 / reps

        ts, tl = timed(small, 8), timed(large, 3)
        del buf
        t = torch.tensor([ts, tl], dtype=torch.float64, device=dev if self.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.process_group)
        ts, tl = (float(x) for x in t.tolist())
        slope = (tl - ts) / (large - small)  # us per byte
        if not slope > 0:
            return None
        bus = 2.0 * (self.world_size - 1) / self.world_size / (slope * 1e3)
        alpha = max(ts - slope * small, 0.5 * ts)
        return alpha, bus

    def replan(self) -> None:
        """Collective: the one-time alpha-beta re-plan of the buckets, if the timed backward is done
        and it has not run yet (every rank must call it at the same point)."""
        self._maybe_replan()

    def _maybe_replan(self) -> None:
        """After the timed backward (collective, see __init__): agree the backward time (MAX over
        ranks, so every rank computes the same plan), then rebuild the buckets once from the
        alpha-beta model."""
        if not self._auto_plan or self._bwd_t is None or self._bwd_t[1] is None:
            return
        t0, t1 = self._bwd_t
        self._auto_plan = False
        if isinstance(t0, float):
            ms = (t1 - t0) * 1e3
        else:
            t1.synchronize()
            ms = t0.elapsed_time(t1)
        dev = self.flat.device if self.backend == "nccl" else torch.device("cpu")
        t = torch.tensor([ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.process_group)
        ms = float(t.item())
        alpha = bus = None
        ab = "model"
        if "MLT_DDP_ALPHA_US" in os.environ or "MLT_DDP_BUS_GBPS" in os.environ:
            ab = "env"
        elif os.environ.get("MLT_DDP_MEASURE_AB", "1") != "0":
            fit = self._measure_alpha_beta()
            if fit is not None:
                alpha, bus = fit
                ab = "measured"
        cap, first = plan_buckets(self._grad_bytes, self.world_size, ms, alpha_us=alpha, bus_gbps=bus)
        self.bucket_plan = {"cap_mb": cap, "first_mb": first, "source": "alpha-beta", "bwd_ms": round(ms, 4),
                            "replans": 1, "ab": ab,
                            "alpha_us": round(alpha if alpha is not None else allreduce_us(0, self.world_size), 3),
                            "bus_gbps": round(bus if bus is not None else float(
                                os.environ.get("MLT_DDP_BUS_GBPS", XGMI_BUS_GBPS)), 3)}
        self._bucket_cap = int(cap * 2 ** 20)
        self._first_cap = int(first * 2 ** 20)
        self._build_buckets()
        self._pending = list(self._bucket_counts)
        self._launched = [False] * len(self._buckets)

    def _finish(self) -> None:
        if self._bwd_t is not None and self._bwd_t[1] is None:
            self._bwd_t[1] = self._mark()  # backward compute done (before the last collectives)
        self._synced_bwd += 1
        # buckets whose params got no gradient this step (unused params): reduce them now
        for b in range(len(self._buckets)):
            if not self._launched[b] and self._bucket_counts[b] > 0:
                self._launched[b] = True
                self._works.append(self._reduce_bucket(b))
        if self._comm_stream is not None:
            if self.timing and self._step_rec is not None:
                ev = torch.cuda.Event(enable_timing=True)
                ev.record()  # backward compute done (compute stream)
                self._step_rec["bwd_end"] = ev
            torch.cuda.current_stream(self.flat.device).wait_stream(self._comm_stream)
            if self.timing and self._step_rec is not None:
                self._records.append(self._step_rec)
                del self._records[:-256]  # bounded history
                self._step_rec = None
        self._wait_all()
        if self._auto_plan and self._bwd_t is not None and self._bwd_t[1] is not None:
            self._maybe_replan()  # collective: every rank finishes this synced backward in order

    def _wait_all(self) -> None:
        for w in self._works:
            if w is None:
                continue
            if isinstance(w, tuple):
                w[0].wait()
                w[1].mul_(1.0 / self.world_size)
            else:
                w.wait()
        self._works.clear()
        self._pending = list(self._bucket_counts)
        self._counted = [False] * len(self.flat.params)
        self._launched = [False] * len(self._buckets)
        self._callback_queued = False

    # ------------------------------------------------------------------ observability
    def reset_comm_stats(self) -> None:
        self._records.clear()

    def comm_stats(self) -> Dict:
        """Per-step averages over the recorded steps (``timing=True``; synchronises the events):
        ``allreduce_ms`` device time of the bucket collectives (incl. wire-dtype casts),
        ``exposed_ms`` comm time after backward compute ended (what the step waits for),
        ``overlap_pct`` share of the collective time hidden under forward/backward,
        ``fwd_bwd_ms`` forward start -> backward compute end, plus the bucket layout."""
        out = {"comm": self.comm_backend, "buckets": len(self._buckets), "bucket_plan": self.bucket_plan,
               "bucket_mb": [round(b / 2 ** 20, 3) for b in self.bucket_sizes_bytes],
               "comm_dtype": str(self.comm_dtype or self.flat.grad.dtype).replace("torch.", ""),
               "steps_timed": 0}
        recs = [r for r in self._records if r.get("t0") is not None and r.get("bwd_end") is not None and r["buckets"]]
        if not recs:
            return out
        tot = hidden = exposed = fb = 0.0
        for r in recs:
            r["bwd_end"].synchronize()
            for _, _, ev0, ev1 in r["buckets"]:
                ev1.synchronize()
            t0 = r["t0"]
            bend = t0.elapsed_time(r["bwd_end"])
            fb += bend
            last = 0.0
            for _, _, ev0, ev1 in r["buckets"]:
                a, b = t0.elapsed_time(ev0), t0.elapsed_time(ev1)
                tot += b - a
                hidden += max(0.0, min(b, bend) - a)
                last = max(last, b)
            exposed += max(0.0, last - bend)
        n = len(recs)
        out.update(steps_timed=n, allreduce_ms=round(tot / n, 4), exposed_ms=round(exposed / n, 4),
                   fwd_bwd_ms=round(fb / n, 4), overlap_pct=round(100.0 * hidden / tot, 1) if tot > 0 else 0.0)
        return out

    def sync_gradients(self) -> None:
        """Manual mode (or after no_sync accumulation): all-reduce the whole flat gradient."""
        if self._ncomm is not None:
            self._ncomm.all_reduce(self.flat.grad, "avg")  # on the current stream
            return
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
        if self.timing and self._comm_stream is not None and self.require_sync and torch.is_grad_enabled():
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self._step_rec = {"t0": ev, "buckets": []}
        return self.module(*args, **kwargs)

    def after_backward(self) -> None:
        """Call after ``loss.backward()``: in manual mode performs the flat all-reduce."""
        if self.mode == "manual" and self.require_sync:
            self.sync_gradients()
