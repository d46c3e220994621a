"""Fused LeNet training-step engine (the Trainer's and bench.py's fast path).

One training step of the reference hot loop (``src/trainer.py:180-197``:
zero_grad -> H2D -> forward -> CE -> loss.item() -> backward (DDP all-reduce)
-> optimizer.step -> metric) becomes:

* W = 1, bf16 (the bench default, BASELINE configs 2/3): TWO kernels per step
  (csrc/kernels/lenet_mfma.inc). ``lenet_ms``: one CU per sample (the sample's
  input -- RandomCrop/HFlip/Normalize of the HBM-resident uint8 image, prepared by
  the previous step's second kernel -- conv/fc forward on MFMA, softmax-CE, the
  whole backward of the sample, its weight-gradient slab). ``lenet_mw``: the batch
  reductions in sample order, the on-device loss/accuracy sums, the fused optimizer
  update of the fp32 masters + bf16 shadow + fragment images, and (on CUs those
  leave idle) the NEXT step's augmented inputs. fp32 (the reference dtype): four
  kernels (csrc/kernels/lenet.hip). Either way captured as a multi-step hipGraph, so
  the host submits one graph per ``steps_per_graph`` steps and never synchronises
  inside an epoch (B12: no ``loss.item()``, no sklearn round trip);
* W > 1, bf16 over xGMI: still two kernels per step (``lenet_ms`` + ``lenet_mwx``):
  the reduction blocks publish their batch-reduced gradient slice into an IPC-shared
  region, pull the peers' slices over xGMI, sum them in rank order and apply the
  update ("xgmi-fused"; W = 1 loopback for timing);
* W > 1 otherwise: the step's kernels -> all-reduce (AVG) of the flat gradient
  (one 248 KB bucket; latency-bound, so a single collective: the one-/two-shot
  xGMI kernels or RCCL, chosen by a timed vote) -> optimizer launch reading
  lr/step from device memory, all enqueued from C++ on the capture stream, so the
  multi-step hipGraphs contain compute, collective and update of every step;
  without a native transport (MLT_NATIVE_COMM=0) each step is graph(kernels) +
  torch.distributed all-reduce + optimizer launch.

(A one-launch form -- the update folded into the next step's launch -- was measured
slower in round 5, profiles/r5/lenet_onelaunch_ab.jsonl, and deleted.)

The device step counter ``ctrl`` (``[global_step, step_in_epoch]``) drives
batch selection from the epoch permutation, the augmentation RNG, the lr table
and Adam's bias correction, so every replay of a captured graph is a new step.
"""
from __future__ import annotations

import math
from typing import Optional, Sequence

import torch

from ml_trainer_amd.models.lenet import MLModel, lenet_buffers, _param_names
from ml_trainer_amd.ops._ext import require_native
from ml_trainer_amd.utils.flat import FlatParams

CIFAR_MEAN = (0.4914, 0.4822, 0.4465)
CIFAR_STD = (0.2023, 0.1994, 0.2010)


def fused_dp_enabled() -> bool:
    """bf16 + xGMI: fold the gradient exchange into the step (MLT_LENET_FUSED_DP=0: the four-launch
    step, for A/B; 2: take the fused step whenever its self-test passes, without the timed vote)."""
    import os
    return os.environ.get("MLT_LENET_FUSED_DP", "1") != "0"


def fused_dp_forced() -> bool:
    import os
    return os.environ.get("MLT_LENET_FUSED_DP", "1") == "2"


def fused_two_mode() -> str:
    """The fused exchange's two-phase form (each 64-granule chunk reduced by one owner rank, which
    publishes the sum: 2 (W-1)/W of the granules read per rank instead of W - 1): MLT_XGMI_FUSED_TWO
    = "auto" (default: a vote candidate at W >= 4), "1" (forced whenever the fused step runs, any
    W > 1), "0" (never)."""
    import os
    v = os.environ.get("MLT_XGMI_FUSED_TWO", "auto")
    return v if v in ("0", "1") else "auto"


class TransportError(RuntimeError):
    """The data-parallel gradient collective failed (peer timeout / RCCL async error)."""


class LeNetStepEngine:
    """``precision``: "fp32" (default; the reference model's dtype, four fp32 kernels per step) or
    "bf16" (BASELINE.json configs 2/3: bf16 MFMA operands, fp32 accumulation / activations /
    master weights / optimizer state; two kernels per step, csrc/kernels/lenet_mfma.hip).
    Evaluation always runs the fp32 forward on the fp32 masters."""

    def __init__(self, model: MLModel, flat: FlatParams, max_batch: int, optimizer=None, process_group=None,
                 world_size: int = 1, seed: int = 0, precision: str = "fp32"):
        if precision not in ("fp32", "bf16"):
            raise ValueError("precision must be 'fp32' or 'bf16'")
        C = require_native()
        self.C = C
        self.model = model
        self.flat = flat
        self.max_batch = int(max_batch)
        self.device = flat.device
        self.world_size = int(world_size)
        self.pg = process_group
        self.seed = int(seed)
        params = model.param_list()
        for p in params:
            if id(p) not in flat._index:
                raise ValueError("model parameters must live in the flat buffer")
        bufs = lenet_buffers(model.cfg_id, self.max_batch, self.device)
        for name, p in zip(_param_names(), params):
            o, n = flat.segment(p)
            bufs[name] = flat.data[o:o + n]
            bufs["g" + name] = flat.grad[o:o + n]
        # bf16 engine: bf16 copy of the flat parameters + the conv-weight MFMA fragment image
        bufs["shadow"] = torch.zeros(flat.numel, dtype=torch.int16, device=self.device)
        bufs["wimg"] = torch.zeros(C.lenet_mfma_wimg_elems(), dtype=torch.int16, device=self.device)
        self.bufs = bufs
        self.stats = bufs["stats"]
        self.ctrl = torch.zeros(2, dtype=torch.int64, device=self.device)
        self.eng = C.LeNetEngine(model.cfg_id, self.max_batch, bufs)
        self.eng.set_ctrl(self.ctrl)
        self.precision = precision
        if precision == "bf16":
            self.eng.set_precision(1)
        self.offsets = [flat.segment(p)[0] for p in params]
        self.comm = None
        self.xgmi = None
        self.captures = 0  # hipGraphs captured so far (bench asserts none inside its timed region)
        self.dp_transport = "none" if self.world_size == 1 else "torch.distributed"
        self.fused_two = False  # the fused exchange runs in its two-phase form
        # the transport is chosen once the optimizer is known (its self-test / timing trial runs the
        # engine's batch-reduction kernels, which need the flat-buffer layout of set_optimizer)
        self._transport_pending = self.world_size > 1
        self.optimizer = None
        self.lr_table: Optional[torch.Tensor] = None
        self._use_table = False
        self.data = None
        self.perm: Optional[torch.Tensor] = None
        if optimizer is not None:
            self.set_optimizer(optimizer)

    # ------------------------------------------------------------------ setup
    def _setup_transport(self, process_group) -> None:
        """Gradient all-reduce transport for the data-parallel step, chosen by measurement:
        the one-shot and two-shot xGMI kernels vs RCCL (all enqueued from C++, so all live inside
        the step's hipGraph); torch.distributed when none is available."""
        import warnings
        import torch.distributed as dist
        from ml_trainer_amd.parallel.comm import create_native_comm, create_xgmi_allreduce
        try:
            self.comm = create_native_comm(process_group, self.device)
        except RuntimeError as e:  # RCCL bring-up failed: keep the torch.distributed path
            warnings.warn(f"native RCCL communicator unavailable ({e}); using torch.distributed")
            self.comm = None
        self.xgmi = create_xgmi_allreduce(process_group, self.flat.numel, self.device)
        # availability is agreed (MIN over ranks) BEFORE any rank times a candidate: every rank
        # then runs the same trials in the same order and the same MAX vote below (a rank whose
        # RCCL bring-up failed would otherwise skip the RCCL trial and desynchronise the group)
        coll_dev = self.device if dist.get_backend(process_group) == "nccl" else torch.device("cpu")
        x = self.xgmi
        avail = torch.tensor([float(self.comm is not None), float(x is not None),
                              float(x is not None and getattr(x, "two_shot_ok", True))], device=coll_dev)
        dist.all_reduce(avail, op=dist.ReduceOp.MIN, group=process_group)
        have_rccl, have_xgmi, have_two = (bool(v) for v in avail.tolist())
        if not have_rccl:
            self.comm = None
        if not have_xgmi:
            self.xgmi = x = None
        if self.comm is None and self.xgmi is None:
            return
        fused_ok = False
        W = dist.get_world_size(process_group)
        # (the fused exchange is offered for 2, 4 and 8 ranks)
        if x is not None and self.precision == "bf16" and fused_dp_enabled() and W in (2, 4, 8):
            # bf16 over xGMI: the exchange can run inside the step (two launches per step), but only
            # once its own protocol -- not just the one-/two-shot kernels -- proved bit-exact on
            # this fabric, on every rank
            fused_ok = self._fused_selftest(x, process_group)
            if not fused_ok:
                warnings.warn("fused xGMI exchange failed its self-test on some rank; using the "
                              "four-launch data-parallel step")
        tmode = fused_two_mode()
        two_ok = False
        if fused_ok and W > 1 and (tmode == "1" or (tmode == "auto" and W >= 4)):
            # the two-phase form proves itself the same way before it may be timed or chosen
            two_ok = self._fused_selftest(x, process_group, two=True)
            if not two_ok:
                warnings.warn("two-phase fused xGMI exchange failed its self-test on some rank")
        self.eng.fused_dp = False
        t = self.flat.grad.clone()
        cands = []
        if x is not None:
            def one():
                x.algo = 0
                x.all_reduce(t, True)

            def two():
                x.algo = 1
                x.all_reduce(t, True)
            cands.append(("xgmi", one))
            if have_two:  # passed its self-test on every rank
                cands.append(("xgmi2", two))
        if self.comm is not None:
            cands.append(("rccl", lambda: self.comm.all_reduce(t, "avg")))
        if fused_ok:
            # the fused step's exchange (batch reductions + granule exchange, one launch) against the
            # four-launch step's collective behind the same batch reductions
            B = self.max_batch
            self.eng.set_xgmi(x)

            def fused(two):
                x.fused_two = two
                self.eng.reduce_only(B, True)
            cands.append(("xgmi-fused", lambda: fused(False)))
            if two_ok:
                cands.append(("xgmi-fused2", lambda: fused(True)))
            cands.append(("reduce", lambda: self.eng.reduce_only(B, False)))
        times = {}
        for name, fn in cands:
            for _ in range(5):
                fn()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(50):
                fn()
            e.record()
            e.synchronize()
            times[name] = s.elapsed_time(e) / 50
        # every rank votes with its own timings and health: the slowest rank decides (MAX), and
        # an xGMI error word raised on ANY rank during the trial rules the xGMI kernels out
        names = ("xgmi", "xgmi2", "rccl", "xgmi-fused", "xgmi-fused2", "reduce")
        bad = 1.0 if (x is not None and x.error()) else 0.0
        coll_dev = self.device if dist.get_backend(process_group) == "nccl" else torch.device("cpu")
        vote = torch.tensor([bad] + [times.get(k, float("inf")) for k in names], device=coll_dev)
        dist.all_reduce(vote, op=dist.ReduceOp.MAX, group=process_group)
        v = [float(u) for u in vote.tolist()]
        bad, agreed = v[0], dict(zip(names, v[1:]))
        if x is not None and bad != 0.0:
            warnings.warn("xGMI all-reduce failed its timing trial on some rank; using RCCL")
            agreed["xgmi"] = agreed["xgmi2"] = agreed["xgmi-fused"] = agreed["xgmi-fused2"] = float("inf")
        self.transport_times_ms = {k: agreed[k] for k in names if k in times}
        self.flat.grad.zero_()
        self.stats.zero_()  # (the trial reductions accumulated their stats)
        four = min(("xgmi", "xgmi2", "rccl"), key=lambda k: agreed[k])
        if x is not None:
            x.fused_two = False
        # the fused step's form: two-phase when forced, else when it measured faster on every rank
        fk = "xgmi-fused2" if two_ok and (tmode == "1" or agreed["xgmi-fused2"] < agreed["xgmi-fused"]) else "xgmi-fused"
        if fused_ok and (fused_dp_forced() or agreed[fk] <= agreed["reduce"] + agreed[four]):
            x.fused_two = fk == "xgmi-fused2"
            self.fused_two = x.fused_two
            self.eng.set_comm(None)
            self.eng.set_xgmi(x)
            self.eng.fused_dp = True
            self.dp_transport = "xgmi-fused"
            return
        self.eng.set_xgmi(None)
        best = four
        if agreed[best] == float("inf"):  # only a failed xGMI and no RCCL: leave torch.distributed
            return
        if best == "rccl":
            self.eng.set_comm(self.comm)
            self.dp_transport = "rccl"
        else:
            x.algo = 0 if best == "xgmi" else 1
            self.eng.set_xgmi(x)
            self.dp_transport = "xgmi-oneshot" if best == "xgmi" else "xgmi-twoshot"

    def _fused_selftest(self, x, process_group, rounds: int = 12, two: bool = False) -> bool:
        """Bring-up test of the fused step's exchange protocol on the real fabric (collective):
        ``rounds`` back-to-back rounds, each with fresh random per-rank activations / slabs, of the
        batch reductions alone (this rank's gradient) and of the batch reductions + granule exchange
        (the lenet_mwx kernel the fused step's update blocks share), under GEMM load from a side
        stream; every exchanged gradient word is compared with the host's RANK-ORDERED sum of every
        rank's local gradient (what each rank's kernel computes), bitwise. MIN vote over ranks.
        two: the two-phase form of the exchange (XgmiAllReduce.fused_two)."""
        import torch.distributed as dist
        dev = self.device
        x.fused_two = two
        W = dist.get_world_size(process_group)
        rank = dist.get_rank(process_group)
        B = self.max_batch
        self.eng.set_xgmi(x)
        names = ("slab1", "p2", "h1", "h2", "dh1", "dh2", "dlogits")
        side = torch.cuda.Stream(dev)
        a = torch.randn(2048, 2048, device=dev)
        torch.cuda.synchronize(dev)
        with torch.cuda.stream(side):  # uneven load on the chip while the exchanges run
            for _ in range(8):
                a = torch.tanh(a @ a * 1e-3)
        gen = torch.Generator(device=dev)
        local, got = [], []
        for it in range(rounds):
            gen.manual_seed(0x5EED + 7919 * rank + 104729 * it)
            for nm in names:
                self.bufs[nm].normal_(generator=gen)
            self.eng.reduce_only(B, False)
            local.append(self.flat.grad.clone())
            self.eng.reduce_only(B, True)
            got.append(self.flat.grad.clone())
        torch.cuda.synchronize(dev)
        coll_dev = dev if dist.get_backend(process_group) == "nccl" else torch.device("cpu")
        mine = torch.stack(local).to(coll_dev)
        parts = [torch.empty_like(mine) for _ in range(W)]
        dist.all_gather(parts, mine, group=process_group)
        ref = parts[0].cpu().clone()
        for q in range(1, W):
            ref = ref + parts[q].cpu()  # rank order, fp32: what the kernel sums
        ref = ref * torch.tensor(1.0 / W, dtype=torch.float32)
        ok = bool(torch.equal(ref, torch.stack(got).cpu())) and x.error() == 0
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=coll_dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=process_group)
        for nm in names:
            self.bufs[nm].zero_()
        self.flat.grad.zero_()
        self.stats.zero_()
        self.eng.set_xgmi(None)
        x.fused_two = False
        ok = int(flag.item()) == 1
        if two:
            self.fused2_selftest_ok = ok
        else:
            self.fused_selftest_ok = ok
        return ok

    def _poll_transport(self) -> None:
        """Non-blocking health check of the in-graph collective, run after every graph replay:
        the xGMI kernel's sticky error word lives in mapped host memory and RCCL reports through
        ncclCommGetAsyncError, so neither read synchronises the device. A failure aborts the
        communicator (unblocking any stuck collective) and raises TransportError."""
        if self.dp_transport.startswith("xgmi") and self.xgmi is not None:
            if self.xgmi.error():
                if self.dp_transport == "xgmi-fused":
                    what = ("the update of every gradient slice whose peers did not arrive was skipped on "
                            "this rank, slices whose peers arrived were applied: replicas may differ, resume "
                            "from the last checkpoint")
                else:
                    what = "this rank applied no part of that step (a peer may have applied it)"
                raise TransportError(f"xGMI gradient exchange: a peer did not arrive within "
                                     f"{self.xgmi.timeout_ms} ms; {what}")
        elif self.dp_transport == "rccl" and self.comm is not None:
            err = self.comm.async_error()
            if err:
                self.comm.abort()
                raise TransportError(f"RCCL communicator failed: {err}")

    def check_transport(self) -> None:
        """Blocking health check: wait for the queued steps, then poll (see _poll_transport)."""
        if self.in_graph_collective:
            torch.cuda.current_stream(self.device).synchronize()
            self._poll_transport()

    def set_optimizer(self, optimizer, lr_table_len: int = 0) -> None:
        self.optimizer = optimizer
        s1, s2 = optimizer.state_buffers(0)
        h = optimizer.hyper(0)
        lr_t = optimizer.lr_tensor(0)
        self._use_table = lr_table_len > 0
        if self._use_table:
            if self.lr_table is None or self.lr_table.numel() < lr_table_len:
                self.lr_table = torch.zeros(lr_table_len, dtype=torch.float32, device=self.device)
            lr_t = self.lr_table
        self._lr_arg = lr_t
        self._hyper = h
        self.eng.set_opt(self.flat.data, self.flat.grad, s1, s2, h["kind"], h["lr"], h["momentum"], h["dampening"],
                         h["weight_decay"], h["beta1"], h["beta2"], h["eps"], h["lr_decay"], h["grad_scale"],
                         h["nesterov"], h["maximize"], lr_t, self._use_table, self.offsets)
        if self._transport_pending:  # collective: every rank sets its optimizer at the same point
            self._transport_pending = False
            self._setup_transport(self.pg)

    def set_dataset(self, data_u8: torch.Tensor, targets: torch.Tensor, batch_size: int, augment: bool = True,
                    pad: int = 4, flip: bool = True, mean: Sequence[float] = CIFAR_MEAN,
                    std: Sequence[float] = CIFAR_STD, perm_capacity: Optional[int] = None) -> None:
        """Make an HBM-resident uint8 dataset [N,32,32,3] the engine's input."""
        if data_u8.dtype != torch.uint8 or tuple(data_u8.shape[1:]) != (32, 32, 3):
            raise ValueError("expected uint8 [N,32,32,3] data")
        self.data = data_u8.to(self.device).contiguous()
        self.targets = targets.to(self.device, torch.int64).contiguous()
        cap = int(perm_capacity or self.data.shape[0])
        self.perm = torch.zeros(max(cap, 1), dtype=torch.int32, device=self.device)
        self.batch_size = int(batch_size)
        self._reset_staging()  # staged next-step images belong to the old dataset
        self.eng.set_aug(self.data, self.perm, self.ctrl, self.targets, self.seed, pad if augment else 0,
                         1 if (augment and flip) else 0, self.batch_size, list(mean), list(std))

    def start_epoch(self, indices: torch.Tensor, lr_values: Optional[Sequence[float]] = None) -> None:
        """Upload this epoch's sample order (and per-step lrs) and reset the in-epoch counter."""
        n = indices.numel()
        if n > self.perm.numel():
            raise ValueError("epoch permutation larger than perm capacity")
        self.perm[:n].copy_(indices.to(torch.int32), non_blocking=True)
        self.ctrl[1:2].zero_()
        self._reset_staging()  # images staged by the last step came from the old order
        if lr_values is not None:
            if not self._use_table:
                raise RuntimeError("engine not configured with an lr table")
            vals = torch.tensor(list(lr_values), dtype=torch.float32)
            self.lr_table[:vals.numel()].copy_(vals, non_blocking=False)
        elif self.optimizer is not None:
            self.optimizer.lr_tensor(0)  # sync group lr -> device scalar

    def _reset_staging(self) -> None:
        for k in ("stage_meta", "meta2", "metaN", "pmeta"):
            self.bufs[k].fill_(-1)

    def reset_stats(self) -> None:
        self.stats.zero_()

    def read_stats(self, n_batches: int):
        s = self.stats.cpu().tolist()
        return s[0] / max(n_batches, 1), s[1] / max(n_batches, 1)

    # ------------------------------------------------------------------ steps
    @property
    def fused(self) -> bool:
        """Single-rank step with the optimizer fused into the backward kernels."""
        return self.world_size == 1 and self.dp_transport == "none"

    def use_transport(self, comm=None, xgmi=None, fused: Optional[bool] = None) -> None:
        """Route the step's gradient through ``comm`` (a ``_C.Communicator``) or ``xgmi`` inside
        the captured graph -- also at world size 1, which rehearses the data-parallel step (RCCL
        all-reduce + flat optimizer launch, or the xGMI exchange against this rank itself) on a
        single GPU. ``fused`` (bf16 + xgmi; default: on unless MLT_LENET_FUSED_DP=0): the
        exchange runs inside the batch-reduction kernel (two launches per step) instead of a
        standalone all-reduce + apply launch (four)."""
        if (comm is None) == (xgmi is None):
            raise ValueError("pass exactly one of comm / xgmi")
        self.comm, self.xgmi = comm, xgmi
        if comm is not None:
            self.eng.set_xgmi(None)
            self.eng.set_comm(comm)
            self.dp_transport = "rccl"
        else:
            if fused is None:
                fused = fused_dp_enabled()
            fused = bool(fused) and self.precision == "bf16"
            self.eng.set_comm(None)
            self.eng.set_xgmi(xgmi)
            self.eng.fused_dp = fused
            self.fused_two = fused and bool(getattr(xgmi, "fused_two", False))
            if fused:
                self.dp_transport = "xgmi-fused"
            else:
                self.dp_transport = "xgmi-twoshot" if getattr(xgmi, "algo", 0) == 1 else "xgmi-oneshot"

    @property
    def in_graph_collective(self) -> bool:
        return self.dp_transport in ("rccl", "xgmi-oneshot", "xgmi-twoshot", "xgmi-fused")

    def _train_mode(self) -> int:
        C = self.C
        base = C.LENET_FWD | C.LENET_CE | C.LENET_BWD
        if self.fused:
            return base | C.LENET_OPT
        return base | (C.LENET_REDUCE if self.in_graph_collective else 0)

    def graph_shapes(self, B: int, n: int, use_graph: bool = True, steps_per_graph: int = 8):
        """The (mode, B, nsteps) hipGraphs ``train_steps(B, n, ...)`` replays, in order (empty
        without graphs). Lets a caller capture them all before a timed region."""
        if not use_graph or n <= 0:
            return []
        mode = self._train_mode()
        if not (self.fused or self.in_graph_collective):
            return [(mode, B, 1)]
        k = max(1, min(steps_per_graph, n))
        full, rem = divmod(n, k)
        return ([(mode, B, k)] if full else []) + ([(mode, B, rem)] if rem else [])

    def prepare(self, B: int, n: int, use_graph: bool = True, steps_per_graph: int = 8) -> int:
        """Capture (and upload) every graph ``train_steps(B, n, ...)`` needs without running a
        step. Returns the number of graphs newly captured."""
        new = 0
        for shape in self.graph_shapes(B, n, use_graph, steps_per_graph):
            new += self._ensure_graph(*shape)
        return new

    def can_prewarm(self) -> bool:
        """Whether prewarm() applies: the step replayed from graphs on a single rank (bf16 or fp32)
        or through the fused xGMI exchange (every buffer those graphs write is engine / optimizer
        state it can snapshot; the exchange's own launch counters are not restored: they advance on
        every rank alike)."""
        return (self.fused or self.in_graph_collective) and self.dp_transport in ("none", "xgmi-fused")

    def _state_tensors(self):
        """Every device tensor the step graphs write: engine buffers (activations, slabs, staging,
        prepared inputs, tags, statistics, bf16 shadow / fragment images), the flat parameters and
        gradients, the optimizer state and the step counters (distinct storages only)."""
        out, seen = [], set()
        cands = list(self.bufs.values()) + [self.flat.data, self.flat.grad, self.ctrl]
        opt = self.optimizer
        if opt is not None:
            cands += [t for t in getattr(opt, "_s1", []) + getattr(opt, "_s2", []) if t is not None]
        for t in cands:
            if not isinstance(t, torch.Tensor) or not t.is_cuda:
                continue
            key = (t.untyped_storage().data_ptr(), t.storage_offset(), t.numel(), t.dtype)
            if key not in seen:
                seen.add(key)
                out.append(t)
        return out

    def prewarm(self, B: int, n: int, steps_per_graph: int = 8) -> int:
        """Capture every graph ``train_steps(B, n, ...)`` replays and launch each once, then put
        every tensor those launches wrote back to its value before them (device copies of a
        snapshot): the engine's state afterwards is bitwise what it was, so the steps that follow
        are bitwise those without it (tests/test_lenet_bf16.py; at W = 2 / 8 through the fused
        exchange, tests/test_multiproc_gpu.py -- its launch counters advance on every rank alike).
        A captured graph's FIRST launch on this stack costs ~20 us more than later ones even after
        hipGraphUpload (profiles/r6/lenet_spg_sync_ab.jsonl); this pays it outside any timed
        region, as capture and upload are. Returns the number of graphs launched."""
        if not self.can_prewarm():
            return 0
        shapes = self.graph_shapes(B, n, True, steps_per_graph)
        for shape in shapes:
            self._ensure_graph(*shape)
        torch.cuda.synchronize(self.device)
        state = self._state_tensors()
        snap = [t.clone() for t in state]
        for mode, b, k in shapes:
            self.eng.replay(mode, b, k)
            self._poll_transport()
        torch.cuda.synchronize(self.device)
        for t, s in zip(state, snap):
            t.copy_(s)
        torch.cuda.synchronize(self.device)
        return len(shapes)

    def _ensure_graph(self, mode: int, B: int, k: int) -> int:
        if self.eng.has_graph(mode, B, k):
            return 0
        self.eng.capture(mode, B, k)
        self.captures += 1
        return 1

    def _note_host_writes(self) -> None:
        """bf16: a torch in-place change of any parameter (each Parameter keeps its own version
        counter, not the flat buffer's) since the last replay -> re-pack the bf16 shadow / fragment
        images ahead of the next one (the engine also watches the flat buffer's own counter)."""
        if self.precision != "bf16":
            return
        sig = tuple(p._version for p in self.flat.params)
        if sig != getattr(self, "_host_sig", None):
            self.eng.invalidate_shadow()
            self._host_sig = sig

    def train_steps(self, B: int, n: int = 1, use_graph: bool = True, steps_per_graph: int = 8) -> None:
        """Run ``n`` full training steps of batch ``B`` from the device dataset."""
        mode = self._train_mode()
        self._note_host_writes()
        if self.fused or self.in_graph_collective:
            if not use_graph:
                for _ in range(n):
                    self.eng.run(mode, B)
                return
            k = max(1, min(steps_per_graph, n))
            full, rem = divmod(n, k)
            if full:
                self._ensure_graph(mode, B, k)
            for _ in range(full):
                self.eng.replay(mode, B, k)
                self._poll_transport()
            if rem:
                self._ensure_graph(mode, B, rem)
                self.eng.replay(mode, B, rem)
                self._poll_transport()
            return
        for _ in range(n):
            self._dist_step(mode, B, use_graph)

    def _dist_step(self, mode: int, B: int, use_graph: bool) -> None:
        import torch.distributed as dist
        if use_graph:
            self._ensure_graph(mode, B, 1)
            self.eng.replay(mode, B, 1)
        else:
            self.eng.run(mode, B)
        g = self.flat.grad
        if self.pg is not None or dist.is_initialized():
            if dist.get_backend(self.pg) == "nccl":
                dist.all_reduce(g, op=dist.ReduceOp.AVG, group=self.pg)
            else:
                dist.all_reduce(g, group=self.pg)
                g.mul_(1.0 / self.world_size)
        h = self._hyper
        s1, s2 = self.optimizer.state_buffers(0)
        self.C.flat_optim(self.flat.data, g, s1, s2, h["kind"], h["lr"], h["momentum"], h["dampening"],
                          h["weight_decay"], h["beta1"], h["beta2"], h["eps"], h["lr_decay"], h["grad_scale"],
                          h["nesterov"], h["maximize"], self._lr_arg, self.ctrl[1:2] if self._use_table else None,
                          self.ctrl[0:1], 1.0, None, None)
        self.eng.invalidate_shadow()  # a native write of the masters: the bf16 step re-packs before its next replay

    def eval_steps(self, B: int, n: int = 1) -> None:
        """Forward + CE + accuracy only (validation / test)."""
        C = self.C
        for _ in range(n):
            self.eng.run(C.LENET_FWD | C.LENET_CE, B)
            self._advance_eval()

    def _advance_eval(self) -> None:
        # eval kernels do not touch the counters (no K5); advance the in-epoch index here
        self.ctrl[1:2].add_(1)

    def step_from_tensors(self, x: torch.Tensor, y: torch.Tensor, train: bool = True) -> None:
        """One step from a host/device batch (generic datasets): x [B,3,32,32], y [B]."""
        C = self.C
        B = x.shape[0]
        if B > self.max_batch:
            raise ValueError("batch larger than engine max_batch")
        self.bufs["x"][:B * 3072].copy_(x.reshape(-1), non_blocking=True)
        self.bufs["targets"][:B].copy_(y.reshape(-1), non_blocking=True)
        if self.data is not None:
            self.eng.clear_aug()
            self.data = None
        if train:
            mode = self._train_mode()
            if self.fused:
                self.eng.run(mode, B)
            else:
                if self.in_graph_collective:
                    self.eng.run(self._train_mode(), B)
                else:
                    self._dist_step(mode, B, use_graph=False)
        else:
            self.eng.run(C.LENET_FWD | C.LENET_CE, B)
