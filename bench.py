#!/usr/bin/env python3
"""Headline benchmark: samples/sec/node + step time of the reference model
(src/model.py LeNet-5, "default" config) trained with DDP on 1/2/4/8 MI355X.

BASELINE.json metric: "samples/sec/node + step time, src/model.py default, DDP
1/2/4/8 MI355X"; the reference's published number is 892 samples/s (mean over 6
epochs, batch 32).

Each timed step is a FULL reference training step (src/trainer.py:180-197):
sample a batch from the dataset (synthetic CIFAR-shaped uint8 data resident in
HBM), RandomCrop(32, pad 4) + HFlip + Normalize (src/utils/functions.py:5-12),
forward, softmax-cross-entropy, loss + accuracy accumulation (on device),
backward, DDP gradient all-reduce (W > 1) and the SGD(lr=1e-3, momentum=0.9)
update -- random-init weights. Compute dtype: bf16 by default (BASELINE.json
configs 2/3 "default config bf16": bf16 MFMA operands, fp32 accumulation,
activations, master weights and optimizer state; two kernels per step at every
W, the gradient exchange over xGMI folded into the second); ``--precision fp32``
is the reference model's own dtype. The headline run is followed by the same
measurement of the fp32 engine (same steps / warmup / protocol), reported as
config.fp32_samples_per_s / config.fp32_ms_per_step: a same-dtype comparison with
the reference every run (``--no-fp32-companion`` skips it).

Scaling modes:
  weak (default)  per-GPU batch fixed at --batch (32 = the reference's batch), global batch = 32*N
  reference       global batch 32 split across ranks (src/trainer.py:62-64)

Usage:  python bench.py --gpus N --steps K --warmup W
  N > 1 under a launcher (torch.distributed.run / torchrun): one rank per GPU over RCCL.
  N > 1 without one: bench.py starts torch.distributed.run --nproc-per-node N itself.

Timing: every hipGraph the K timed steps replay is captured and uploaded before the timed
region (a capture counter is checked after it); wall time between barrier+synchronize pairs is
reported. The LeNet timed region holds no hipEvent (two timing-event records cost ~30 us of wall
time per region here); per-kernel device time comes from rocprofv3 (profiles/).

BASELINE.json config 5 ("large" fp8: 24L/1024H BERT encoder, OCP fp8 forward/dgrad GEMMs with
delayed scaling): ``--model large [--grad-accum N]`` (``--model bert-large`` = same model in bf16).

BASELINE.json config 4 (BERT-base classifier, seq 512, bf16, DDP): ``--model bert-base``
(per-GPU batch --batch, default 1536; native MFMA GEMM / flash-attention / LayerNorm kernels,
fused AdamW on flat fp32 masters with bf16 shadows, bucketed RCCL all-reduce overlapped with
backward for N > 1).
"""
from __future__ import annotations

import argparse
import contextlib
import json
import math
import os
import sys
import time

BASELINE_SAMPLES_PER_S = 892.0  # BASELINE.md headline (CPU, batch 32)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3000)
    ap.add_argument("--warmup", type=int, default=300)
    ap.add_argument("--batch", type=int, default=None,
                    help="per-GPU batch (weak) / global batch (reference); default 32 (LeNet), "
                         "1536 (bert-base: 228 GiB), 256 (bert-large), 512 (large fp8: 245 GiB of HBM)")
    ap.add_argument("--scaling", choices=["weak", "reference"], default="weak")
    ap.add_argument("--model", default="default",
                    choices=["default", "tiny", "bert-base", "bert-tiny", "bert-large", "large"])
    ap.add_argument("--seq-len", type=int, default=512)
    ap.add_argument("--zero", type=int, default=0, choices=(0, 1),
                    help="BERT modes, N>1: 1 = ZeRO-1 sharded optimizer state instead of replicated DDP")
    ap.add_argument("--grad-accum", type=int, default=1, help="micro-batches per optimizer step (BERT modes)")
    ap.add_argument("--bucket-mb", type=float, default=None, help="BERT modes, N>1: DDP bucket cap (MB)")
    ap.add_argument("--first-bucket-mb", type=float, default=None, help="BERT modes, N>1: first DDP bucket (MB)")
    ap.add_argument("--ddp-timing", action="store_true",
                    help="BERT modes, N>1: hipEvent bucket timings (all-reduce ms, overlap %%) in the JSON line; "
                         "off by default so the timed steps take the Trainer's gradient path")
    ap.add_argument("--grad-comm", choices=["fp32", "bf16"], default="fp32",
                    help="BERT modes, N>1: gradient all-reduce wire dtype (bf16 = cast in the bucket, reduce, "
                         "cast back into the fp32 gradient)")
    ap.add_argument("--no-prewarm", action="store_true",
                    help="LeNet: no pre-launch of the timed graphs (steps per graph then divide the warmup)")
    ap.add_argument("--steps-per-graph", type=int, default=0,
                    help="LeNet steps per captured hipGraph (0 = auto: min(steps, 64))")
    ap.add_argument("--device", choices=["gpu", "cpu"], default="gpu",
                    help="cpu: BASELINE config 1 plumbing (stock torch ops, gloo); also used without a GPU")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--dataset-size", type=int, default=50000)
    ap.add_argument("--optimizer", default="sgd")
    ap.add_argument("--precision", choices=["bf16", "fp32"], default="bf16",
                    help="LeNet step: bf16 (BASELINE.json configs 2/3 'default config bf16': bf16 MFMA "
                         "operands, fp32 accumulation / activations / masters / optimizer state; 2 kernels "
                         "per step) or fp32 (the reference model's dtype; 4 kernels per step)")
    ap.add_argument("--no-fp32-companion", action="store_true",
                    help="LeNet bf16: skip the fp32 engine measurement that follows the headline run")
    ap.add_argument("--transport", choices=["auto", "xgmi-loopback", "rccl-loopback"], default="auto",
                    help="LeNet, 1 GPU: time the data-parallel step against this rank itself (xgmi-loopback: "
                         "the bf16 two-launch exchange step; rccl-loopback: a real ncclAllReduce in the graph)")
    ap.add_argument("--seed", type=int, default=32)
    ap.add_argument("--json-out", default=None)
    return ap.parse_args()


def bench_bert(args, world, rank, dev):
    """BERT classifier training step: synthetic token ids, random-init weights, bf16 compute."""
    import torch
    import torch.distributed as dist
    from ml_trainer_amd.models.bert import BertClassifier, bert_config
    from ml_trainer_amd.ops.losses import CrossEntropyLoss
    from ml_trainer_amd.ops.optim import FusedAdamW
    from ml_trainer_amd.parallel.ddp import DistributedDataParallel

    torch.manual_seed(args.seed)
    cfg = bert_config(args.model)
    model = BertClassifier(cfg).to(dev)
    per_gpu = args.batch if args.scaling == "weak" else max(args.batch // world, 1)
    if world > 1 and args.zero:
        from ml_trainer_amd.parallel.zero import ZeroDataParallel
        ddp = ZeroDataParallel(model)  # ZeRO-1: reduce-scatter, sharded AdamW, all-gather
        opt = ddp.make_optimizer(FusedAdamW, lr=1e-4, weight_decay=0.01)
        fwd = ddp
    elif world > 1:
        ddp = DistributedDataParallel(model, bucket_cap_mb=args.bucket_mb, first_bucket_mb=args.first_bucket_mb,
                                      comm_dtype=torch.bfloat16 if args.grad_comm == "bf16" else None,
                                      timing=args.ddp_timing)
        opt = FusedAdamW(model.parameters(), lr=1e-4, weight_decay=0.01, flat=ddp.flat)
        fwd = ddp
    else:
        opt = FusedAdamW(model.parameters(), lr=1e-4, weight_decay=0.01)
        fwd = model
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    pool = 8  # rotating synthetic batches resident in HBM
    ids = torch.randint(5, cfg.vocab_size, (pool, per_gpu, args.seq_len), device=dev, generator=g)
    labels = torch.randint(0, cfg.num_labels, (pool, per_gpu), device=dev, generator=g)
    loss_acc = torch.zeros((), device=dev)

    accum = max(1, args.grad_accum)
    ce = CrossEntropyLoss()

    def run(n, start):
        for i in range(n):
            opt.zero_grad(set_to_none=False)
            for a in range(accum):  # gradient accumulation: all-reduce only on the last micro-batch
                j = (start + i * accum + a) % pool
                sync = a == accum - 1
                ctxm = ddp.no_sync() if (world > 1 and not sync) else contextlib.nullcontext()
                with ctxm:
                    loss = ce(fwd(ids[j]), labels[j])  # native fused softmax-CE (src/trainer.py:141-142)
                    (loss / accum if accum > 1 else loss).backward()
                loss_acc.add_(loss.detach())
            opt.step()

    run(args.warmup, 0)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
        if hasattr(ddp, "reset_comm_stats"):
            ddp.reset_comm_stats()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(args.steps, args.warmup)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev if dist.get_backend() == "nccl" else "cpu") \
        if world > 1 else torch.tensor([elapsed], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    total = per_gpu * world * args.steps * accum
    value = total / elapsed
    comm = None
    if world > 1 and hasattr(ddp, "comm_stats"):
        comm = ddp.comm_stats()  # bucket layout + comm backend; hipEvent timings with --ddp-timing
        if args.ddp_timing:
            vals = torch.tensor([comm.get("allreduce_ms", 0.0), comm.get("exposed_ms", 0.0)], dtype=torch.float64,
                                device=dev if dist.get_backend() == "nccl" else "cpu")
            dist.all_reduce(vals, op=dist.ReduceOp.MAX)
            comm["allreduce_ms_max_rank"], comm["exposed_ms_max_rank"] = [round(float(v), 4) for v in vals.tolist()]
    return {
        "metric": "samples/sec/node",
        "value": round(value, 1),
        "unit": "samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak" if args.scaling == "weak" else "strong",
        "vs_baseline": None,
        "dtype": "fp8" if cfg.fp8 else "bf16",
        "data": "synthetic token ids (uniform over the vocabulary) resident in HBM, random-init weights",
        "config": {"model": f"BERT classifier {args.model} ({cfg.layers}L/{cfg.hidden}H/{cfg.heads}A, "
                            f"{model.num_parameters():,} params)",
                   "global_batch": per_gpu * world * accum, "per_gpu_batch": per_gpu, "grad_accum": accum,
                   "seq_len": args.seq_len, "fp8": bool(cfg.fp8),
                   "parallelism": f"dp{world}" + ("-zero1" if (args.zero and world > 1) else ""),
                   "optimizer": "fused AdamW lr=1e-4 wd=0.01 (fp32 master, bf16 shadow)",
                   "tokens_per_s": round(value * args.seq_len, 1),
                   "model_tflops": round(model.flops_per_token(args.seq_len) * value * args.seq_len / 1e12, 1),
                   "peak_hbm_gib": round(torch.cuda.max_memory_allocated(dev) / 2**30, 1),
                   "ddp_comm": comm,
                   "comm": (comm or {}).get("comm") if world > 1 else None,
                   "loss_finite": math.isfinite(float(loss_acc.item()))},
    }


def lenet_plan(nsteps: int, st: dict, n_data: int, world: int, rank: int, per_gpu: int, spg: int, shard_fn):
    """The LeNet engine calls of the next ``nsteps`` steps, crossing epochs as needed, advancing
    the epoch state ``st`` (keys epoch/shard_len/step_in_epoch/steps_per_epoch): yields
    ("epoch", indices) and ("steps", batch, k, steps_per_graph). Every epoch ends with its
    partial batch (DistributedSampler shard length not divisible by the batch) as a 1-step call."""
    while nsteps > 0:
        if st["step_in_epoch"] >= st["steps_per_epoch"]:
            idx = shard_fn(n_data, world, rank, shuffle=True, seed=0, epoch=st["epoch"])
            st["epoch"] += 1
            st["shard_len"] = len(idx)
            st["steps_per_epoch"] = math.ceil(len(idx) / per_gpu)
            st["step_in_epoch"] = 0
            yield ("epoch", idx)
        left = st["steps_per_epoch"] - st["step_in_epoch"]
        full_left = left - (1 if st["shard_len"] % per_gpu else 0)
        if full_left > 0:
            k = min(nsteps, full_left)
            yield ("steps", per_gpu, k, spg)
        else:
            k = 1
            yield ("steps", st["shard_len"] - (st["steps_per_epoch"] - 1) * per_gpu, 1, 1)
        st["step_in_epoch"] += k
        nsteps -= k


def precapture(engine, events, use_graph: bool) -> None:
    """Capture (and upload) every hipGraph the planned steps will replay, without running one."""
    for ev in events:
        if ev[0] == "steps":
            engine.prepare(ev[1], ev[2], use_graph=use_graph, steps_per_graph=ev[3])


def _self_launch(args) -> int:
    """--gpus N > 1 without a launcher: start N fresh rank processes through torch.distributed.run
    (rendezvous on 127.0.0.1, a free port) and return its exit code. The parent never touches the
    GPU (no HIP init, no exec); rank 0 prints the JSON line."""
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def _emit(out, rank, args):
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")


def bench_cpu(args, world, rank):
    """BASELINE config 1 (tiny/default LeNet on CPU, gloo): plumbing path with stock torch ops,
    the native DDP bucket engine over gloo and the flat optimizer's CPU implementation."""
    import torch
    import torch.distributed as dist
    import torch.nn.functional as F
    from ml_trainer_amd.models.lenet import MLModel
    from ml_trainer_amd.ops.optim import build_optimizer
    from ml_trainer_amd.parallel.ddp import DistributedDataParallel

    torch.manual_seed(args.seed)
    model = MLModel(args.model)
    fwd = DistributedDataParallel(model) if world > 1 else model
    opt = build_optimizer(args.optimizer, model.parameters(), lr=1e-3, momentum=0.9, weight_decay=0.0,
                          flat=fwd.flat if world > 1 else None)
    per_gpu = args.batch if args.scaling == "weak" else max(args.batch // world, 1)
    g = torch.Generator().manual_seed(1234 + rank)
    xs = torch.randn(4, per_gpu, 3, 32, 32, generator=g)
    ys = torch.randint(0, 10, (4, per_gpu), generator=g)
    loss_acc = torch.zeros(())

    def run(n, start):
        for i in range(n):
            opt.zero_grad(set_to_none=False)
            loss = F.cross_entropy(fwd(xs[(start + i) % 4]), ys[(start + i) % 4])
            loss.backward()
            opt.step()
            loss_acc.add_(loss.detach())

    run(args.warmup, 0)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    run(args.steps, args.warmup)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    value = per_gpu * world * args.steps / elapsed
    return {
        "metric": "samples/sec/node", "value": round(value, 1), "unit": "samples/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak" if args.scaling == "weak" else "strong",
        "vs_baseline": round(value / BASELINE_SAMPLES_PER_S, 2), "dtype": "fp32",
        "data": "synthetic CIFAR-shaped float tensors, random-init weights",
        "config": {"model": f"src/model.py MLModel ({args.model})", "device": "cpu",
                   "global_batch": per_gpu * world, "per_gpu_batch": per_gpu, "seq_len": None,
                   "parallelism": f"dp{world}", "backend": dist.get_backend() if world > 1 else "none",
                   "loss_finite": math.isfinite(float(loss_acc))},
    }


def bench_lenet(args, world, rank, dev, backend, precision):
    """The LeNet headline (BASELINE.json metric): the fused step engine on an HBM-resident
    synthetic dataset, every hipGraph captured before the timed region."""
    import torch
    import torch.distributed as dist
    from ml_trainer_amd.models.lenet import MLModel
    from ml_trainer_amd.models.lenet_engine import LeNetStepEngine
    from ml_trainer_amd.ops.optim import build_optimizer
    from ml_trainer_amd.parallel.sampler import shard_indices
    from ml_trainer_amd.utils.flat import FlatParams

    torch.manual_seed(args.seed)
    model = MLModel(args.model).to(dev)
    flat = FlatParams(model.parameters())
    if world > 1:
        dist.broadcast(flat.data, src=0)  # DDP-style initial parameter broadcast
    opt = build_optimizer(args.optimizer, model.parameters(), lr=1e-3, momentum=0.9, weight_decay=0.0, flat=flat)
    per_gpu = args.batch if args.scaling == "weak" else max(args.batch // world, 1)
    engine = LeNetStepEngine(model, flat, max_batch=per_gpu, optimizer=opt, world_size=world, seed=args.seed,
                             precision=precision)
    transport = args.transport
    if os.environ.get("MLT_BENCH_FORCE_RCCL") == "1":
        transport = "rccl-loopback"
    if transport != "auto" and world == 1:
        # W=1 rehearsal of the data-parallel step: a real ncclAllReduce inside the captured graph, or
        # the xGMI exchange against this rank itself (bf16: folded into the reduction kernel)
        C = engine.C
        if transport == "rccl-loopback":
            engine.use_transport(comm=C.Communicator(C.Communicator.unique_id(), 1, 0, dev.index))
        else:
            from ml_trainer_amd.parallel.comm import create_xgmi_loopback
            engine.use_transport(xgmi=create_xgmi_loopback(flat.numel, dev))

    # Synthetic CIFAR-10-shaped dataset (uint8 HWC) resident in HBM; random labels.
    N = args.dataset_size
    g = torch.Generator(device=dev).manual_seed(1234)
    data = torch.randint(0, 256, (N, 32, 32, 3), dtype=torch.uint8, device=dev, generator=g)
    targets = torch.randint(0, 10, (N,), dtype=torch.int64, device=dev, generator=g)
    engine.set_dataset(data, targets, batch_size=per_gpu, augment=True)
    # graphs of up to 64 steps: one replay covers a short timed run, long runs amortise launches
    # steps per graph: the largest d <= 64 dividing both K and W, so that the warmup replays the very
    # graph the timed steps replay (a freshly uploaded graph's first replay costs ~40 us more, measured
    # by scripts/debug/replay_cold.py); min(64, K) when they share no useful divisor
    # With graph pre-warming (single rank, or the bf16 step's fused xGMI exchange): one graph for
    # the whole timed run when K <= 64 (else the largest divisor of K up to 64; 250-step graphs ran
    # ~1 us per step slower), its first-launch cost paid before t0 (engine.prewarm: one launch of
    # each timed graph, then every tensor it wrote restored from a snapshot -- the timed steps start
    # from bitwise the state the warmup left; profiles/r6/lenet_spg_sync_ab.jsonl: a cold graph
    # costs ~20 us on its first launch, and each extra graph launch in the timed region ~7 us)
    spg = args.steps_per_graph
    use_graph = not args.no_graph
    prewarm = use_graph and not args.no_prewarm and engine.can_prewarm()
    if not spg and prewarm:
        spg = max(d for d in range(1, min(64, args.steps) + 1) if args.steps % d == 0)
    elif not spg:
        common = [d for d in range(1, 65) if args.steps % d == 0 and args.warmup > 0 and args.warmup % d == 0]
        spg = max(common) if common and max(common) >= 4 else max(1, min(64, args.steps))

    state = {"epoch": 0, "shard_len": 0, "step_in_epoch": 0, "steps_per_epoch": 0}

    def run(nsteps: int) -> int:
        """Run nsteps training steps; return samples processed on this rank."""
        samples = 0
        for ev in lenet_plan(nsteps, state, N, world, rank, per_gpu, spg, shard_indices):
            if ev[0] == "epoch":
                engine.start_epoch(torch.as_tensor(ev[1], dtype=torch.int32))
            else:
                _, b, k, per_graph = ev
                engine.train_steps(b, k, use_graph=use_graph, steps_per_graph=per_graph)
                samples += b * k
        return samples

    # capture + upload every hipGraph the warmup AND the timed steps replay before any step runs
    # (no step runs here), so the timed region holds exactly K steps of replays and nothing else,
    # and the warmup replays end right before t0 (no capture gap lets the GPU idle down in between)
    st_w = dict(state)
    plan_w = list(lenet_plan(args.warmup, st_w, N, world, rank, per_gpu, spg, shard_indices))
    precapture(engine, plan_w, use_graph)
    precapture(engine, lenet_plan(args.steps, dict(st_w), N, world, rank, per_gpu, spg, shard_indices), use_graph)
    # no hipEvent inside the timed region: two timing-event records cost ~30 us of wall time per
    # region on this stack (21.1-21.9 vs 19.6-19.7 us/step at K=20,
    # profiles/r4/lenet_timed_region_events_ab.jsonl); per-kernel device times come from rocprofv3
    run(args.warmup)
    prewarmed = 0
    if prewarm:  # one launch of every graph the timed steps replay, state restored bitwise
        seen = set()
        for ev in lenet_plan(args.steps, dict(state), N, world, rank, per_gpu, spg, shard_indices):
            if ev[0] == "steps" and ev[1:] not in seen:
                seen.add(ev[1:])
                prewarmed += engine.prewarm(ev[1], ev[2], steps_per_graph=ev[3])
    captures_before = engine.captures
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    samples = run(args.steps)
    torch.cuda.synchronize()
    if world > 1:  # (one rank: no barrier, and nothing left for a second synchronize to wait for)
        dist.barrier()
        torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if engine.captures != captures_before:
        raise RuntimeError("a hipGraph was captured inside the timed region")

    tot = torch.tensor([elapsed, float(samples)], dtype=torch.float64,
                       device=dev if backend == "nccl" else torch.device("cpu"))
    if world > 1:
        t_max = tot[0:1].clone()
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
        s_sum = tot[1:2].clone()
        dist.all_reduce(s_sum, op=dist.ReduceOp.SUM)
        elapsed, total_samples = float(t_max.item()), float(s_sum.item())
    else:
        total_samples = float(samples)
    # sanity: training actually ran (finite loss accumulated on device); transport healthy
    loss_sum = float(engine.stats[0].item())
    engine.check_transport()
    value = total_samples / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    nodes = engine.eng.graph_nodes(engine._train_mode(), per_gpu, spg) if use_graph else 0
    tt = getattr(engine, "transport_times_ms", None)
    comm = None
    if world > 1:
        # the one 248 KB bucket is reduced inside the step's hipGraph between backward and the
        # update (latency-bound, serial by construction): its cost is the standalone per-call time
        # of the transport the engine chose, measured at set-up on every rank (max over ranks, the
        # same vote that picked the transport)
        key = {"xgmi-oneshot": "xgmi", "xgmi-twoshot": "xgmi2", "rccl": "rccl"}.get(engine.dp_transport)
        comm = {"buckets": 1, "bucket_mb": [round(flat.numel * 4 / 2 ** 20, 3)], "comm_dtype": "float32",
                "in_graph": engine.in_graph_collective, "overlap_pct": 0.0,
                "fused_into_reduction_kernel": engine.dp_transport == "xgmi-fused",
                "fused_two_phase": bool(getattr(engine, "fused_two", False)),
                "allreduce_ms": round(tt[key], 4) if (tt and key in tt) else None}
    out = {
        "metric": "samples/sec/node",
        "value": round(value, 1),
        "unit": "samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 5),
        "higher_is_better": True,
        "scaling": "weak" if args.scaling == "weak" else "strong",
        "vs_baseline": round(value / BASELINE_SAMPLES_PER_S, 2),
        "dtype": precision,
        "data": "synthetic (CIFAR-10-shaped uint8 in HBM, on-GPU RandomCrop+HFlip+Normalize), random-init weights",
        "config": {"model": f"src/model.py MLModel ({args.model} LeNet-5, 62,006 params)" if args.model == "default"
                   else f"src/model.py MLModel ({args.model})",
                   "global_batch": per_gpu * world, "per_gpu_batch": per_gpu, "seq_len": None,
                   "parallelism": f"dp{world}", "optimizer": f"{args.optimizer} lr=1e-3 momentum=0.9",
                   "hipgraph_steps": 0 if args.no_graph else spg,
                   "graph_prewarm": prewarmed,
                   "kernels_per_step": round(nodes / spg, 2) if nodes else None,
                   "update": ("pipelined: step k's batch reductions / exchange / optimizer update run in "
                              "step k+1's launch beside its sample blocks' input phase"
                              if nodes and nodes == spg else "in-step"),
                   "ddp_comm": comm,
                   "dp_transport": engine.dp_transport,
                   "comm_ranks": engine.comm.size if engine.comm is not None else None,
                   "transport_ms": getattr(engine, "transport_times_ms", None),
                   "loss_finite": math.isfinite(loss_sum)},
    }
    if world > 1:
        dist.barrier()
    return out


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_self_launch(args))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE={world}; measuring WORLD_SIZE ranks",
              file=sys.stderr)
    backend = os.environ.get("MLT_BENCH_BACKEND", "nccl")
    if args.batch is None:
        # LeNet: the reference batch (src/trainer.py / main.py: 32). Transformer configs: micro-batches
        # sized for 288 GB of HBM per GPU (per-GPU throughput keeps rising with the micro-batch:
        # BERT-base 2,552 / 2,665 / 2,710 samples/s at 128 / 256 / 512 using 21 / 40 / 77 GiB; the fp8
        # `large` config, BASELINE config 5 "sized to fill HBM": 1,013 / 1,030 samples/s at 256 / 512
        # using 126 / 245 GiB; profiles/batch_sweep_r2.jsonl; round 4, same box: BERT-base 2,921 / 2,929
        # at 512 vs 2,965 / 2,964 at 1024 (152 GiB), profiles/r4/bert_base_batch_groupm_ab.jsonl; round 5,
        # same box: 3,084 / 3,088 at 1024 vs 3,112 / 3,110 at 1536 (228 GiB),
        # profiles/r5/bert_base_batch_1024_1536.jsonl)
        args.batch = {"bert-base": 1536, "bert-large": 256, "large": 512, "bert-tiny": 32}.get(args.model, 32)

    # host waits spin instead of yield (before anything creates the device's context; MLT_SYNC_SPIN=0
    # keeps ROCm's default): the timed region ends in one synchronize
    same_dev = os.environ.get("MLT_BENCH_SAME_DEVICE") == "1"
    spin = False
    if args.device != "cpu" and torch.cuda.device_count() > 0:
        from ml_trainer_amd.parallel.dist import set_sync_spin
        spin = set_sync_spin(0 if same_dev else local_rank)
    if args.device == "cpu" or not torch.cuda.is_available():
        if world > 1:
            dist.init_process_group("gloo")
        if args.steps == 3000 and args.warmup == 300:
            args.steps, args.warmup = 50, 5
        _emit(bench_cpu(args, world, rank), rank, args)
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    # rehearsal knob for a 1-GPU box (not for real runs): all ranks on GPU 0 over gloo
    dev = torch.device("cuda", 0 if same_dev else local_rank)
    torch.cuda.set_device(dev)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
        world = dist.get_world_size()

    if args.model in ("bert-base", "bert-tiny", "bert-large", "large"):
        if args.steps == 3000 and args.warmup == 300:  # LeNet-sized defaults -> BERT-sized
            args.steps, args.warmup = 20, 5
        r = bench_bert(args, world, rank, dev)
        r["config"]["host_sync"] = "spin" if spin else "default"
        _emit(r, rank, args)
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    out = bench_lenet(args, world, rank, dev, backend, args.precision)
    out["config"]["host_sync"] = "spin" if spin else "default"
    if args.precision == "bf16" and not args.no_fp32_companion:
        # same-dtype comparison with the reference (fp32), same protocol, after the headline run
        comp = bench_lenet(args, world, rank, dev, backend, "fp32")
        out["config"]["fp32_samples_per_s"] = comp["value"]
        out["config"]["fp32_ms_per_step"] = comp["ms_per_step"]
        out["config"]["fp32_vs_baseline"] = comp["vs_baseline"]
        out["config"]["fp32_dp_transport"] = comp["config"]["dp_transport"]
    _emit(out, rank, args)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
