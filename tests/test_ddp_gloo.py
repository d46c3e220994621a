"""Native DDP over gloo with world_size 2 on CPU (fake cluster: spawned processes)."""
import copy
import os
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.helpers import TensorCifar, dist_env, free_port


def _ddp_worker(rank, world, port, mode, out_dir):
    dist_env(rank, world, port)
    dist.init_process_group("gloo")
    from ml_trainer_amd.parallel.ddp import DistributedDataParallel
    torch.manual_seed(1234 + rank)  # different init per rank: broadcast must fix it
    model = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 4))
    ddp = DistributedDataParallel(model, bucket_cap_mb=0.0005, first_bucket_mb=0.0002, mode=mode)
    assert len(ddp.bucket_sizes_bytes) >= 2
    g = torch.Generator().manual_seed(7)
    x = torch.randn(world * 6, 8, generator=g)
    y = torch.randn(world * 6, 4, generator=g)
    xs, ys = x[rank * 6:(rank + 1) * 6], y[rank * 6:(rank + 1) * 6]
    loss = ((ddp(xs) - ys) ** 2).mean()
    loss.backward()
    ddp.after_backward()
    grads = ddp.flat.grad.clone()
    torch.save({"grads": grads, "params": ddp.flat.data.clone()}, os.path.join(out_dir, f"r{rank}.pt"))
    # no_sync: local grads only
    ddp.flat.zero_grad()
    with ddp.no_sync():
        ((ddp(xs) - ys) ** 2).mean().backward()
    torch.save({"nosync": ddp.flat.grad.clone()}, os.path.join(out_dir, f"ns{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("mode,world", [("overlap", 2), ("manual", 2), ("overlap", 4)])
def test_ddp_grads_equal_full_batch(mode, world):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_ddp_worker, args=(world, free_port(), mode, d), nprocs=world, join=True)
        r = [torch.load(os.path.join(d, f"r{i}.pt"), weights_only=True) for i in range(world)]
        for k in range(1, world):
            assert torch.equal(r[0]["params"], r[k]["params"])  # broadcast from rank 0
            assert torch.equal(r[0]["grads"], r[k]["grads"])  # fixed-order reduction: bitwise equal
        # reference: full-batch gradient on one process with rank 0's params
        from ml_trainer_amd.utils.flat import FlatParams
        torch.manual_seed(1234)
        model = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 4))
        fp = FlatParams(model.parameters(), reverse=True)
        assert torch.equal(fp.data, r[0]["params"])
        g = torch.Generator().manual_seed(7)
        x = torch.randn(world * 6, 8, generator=g)
        y = torch.randn(world * 6, 4, generator=g)
        # mean of per-rank means == full mean (equal shard sizes)
        ((model(x) - y) ** 2).mean().backward()
        torch.testing.assert_close(r[0]["grads"], fp.grad, rtol=1e-5, atol=1e-6)
        ns = [torch.load(os.path.join(d, f"ns{i}.pt"), weights_only=True)["nosync"] for i in range(world)]
        assert not torch.allclose(ns[0], ns[1])


def _trainer_worker(rank, world, port, out_dir, per_device):
    dist_env(rank, world, port)
    from ml_trainer_amd.models.lenet import MLModel
    from ml_trainer_amd.trainer import Trainer
    torch.manual_seed(0)
    tr, va = TensorCifar(96, 0), TensorCifar(32, 1)
    t = Trainer(MLModel("tiny"), datasets=(tr, va), epochs=2, batch_size=32, is_parallel=True, save_history=True,
                backend="gloo", model_dir=out_dir, lr=0.02,
                options={"progress": False, "per_device_batch": per_device, "determinism_check": True})
    assert t.world_size == world and t.batch_size == (32 if per_device else 16)
    t.fit()
    torch.save({"params": t.flat.data.clone(), "losses": t.train_losses},
               os.path.join(out_dir, f"t{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("per_device", [False, True])
def test_trainer_gloo_world2(per_device):
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_trainer_worker, args=(world, free_port(), d, per_device), nprocs=world, join=True)
        r = [torch.load(os.path.join(d, f"t{i}.pt"), weights_only=True) for i in range(world)]
        assert torch.equal(r[0]["params"], r[1]["params"])  # replicas stay identical
        sd = torch.load(os.path.join(d, "model.pth"), weights_only=True)
        assert all(k.startswith("module.") for k in sd)  # DDP checkpoint keys (reference B4)
        assert os.path.exists(os.path.join(d, "history.pkl"))


def _fault_worker(rank, world, port, out_dir):
    dist_env(rank, world, port)
    from ml_trainer_amd.models.lenet import MLModel
    from ml_trainer_amd.trainer import Trainer
    tr, va = TensorCifar(256, 0), TensorCifar(32, 1)
    t = Trainer(MLModel("tiny"), datasets=(tr, va), epochs=1, batch_size=16, is_parallel=True, backend="gloo",
                model_dir=out_dir, options={"progress": False, "fault_inject_step": 3, "fault_inject_rank": 1,
                                            "dist_timeout_s": 20})
    try:
        t.fit()
        status = "completed"
    except Exception as e:  # noqa: BLE001
        status = f"error: {type(e).__name__}"
    with open(os.path.join(out_dir, f"s{rank}.txt"), "w") as f:
        f.write(status)


def test_fault_injection_surfaces_on_all_ranks():
    world = 2
    with tempfile.TemporaryDirectory() as d:
        ctx = mp.start_processes(_fault_worker, args=(world, free_port(), d), nprocs=world, join=False,
                                 start_method="spawn")
        ctx.join(timeout=120) or None
        while not ctx.join(timeout=120):
            pass
        s = [open(os.path.join(d, f"s{i}.txt")).read() for i in range(world)]
        assert s[1].startswith("error") and "completed" not in s[0], s


def _bf16_comm_worker(rank, world, port, out_dir):
    dist_env(rank, world, port)
    dist.init_process_group("gloo")
    from ml_trainer_amd.parallel.ddp import DistributedDataParallel
    out = {}
    for tag, cd in (("fp32", None), ("bf16", torch.bfloat16)):
        torch.manual_seed(1234)
        model = torch.nn.Sequential(torch.nn.Linear(32, 64), torch.nn.ReLU(), torch.nn.Linear(64, 8))
        ddp = DistributedDataParallel(model, bucket_cap_mb=0.004, first_bucket_mb=0.002, comm_dtype=cd)
        g = torch.Generator().manual_seed(11 + rank)
        x, y = torch.randn(16, 32, generator=g), torch.randn(16, 8, generator=g)
        ((ddp(x) - y) ** 2).mean().backward()
        ddp.after_backward()
        out[tag] = ddp.flat.grad.clone()
        out[tag + "_buckets"] = len(ddp.bucket_sizes_bytes)
        out[tag + "_dtype"] = ddp.comm_stats()["comm_dtype"]
    torch.save(out, os.path.join(out_dir, f"b{rank}.pt"))
    dist.destroy_process_group()


def test_bf16_gradient_comm_close_to_fp32():
    """comm_dtype=bf16: buckets are cast to bf16, reduced, cast back -- within bf16 rounding
    of the fp32 all-reduce, identical on every rank."""
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_bf16_comm_worker, args=(world, free_port(), d), nprocs=world, join=True)
        r = [torch.load(os.path.join(d, f"b{i}.pt"), weights_only=True) for i in range(world)]
        assert r[0]["bf16_buckets"] >= 2 and r[0]["bf16_dtype"] == "bfloat16" and r[0]["fp32_dtype"] == "float32"
        assert torch.equal(r[0]["bf16"], r[1]["bf16"])
        a, b = r[0]["fp32"], r[0]["bf16"]
        rel = (a - b).norm() / a.norm()
        assert rel < 1e-2, rel
        assert not torch.equal(a, b)  # the wire dtype really was bf16


_EVENTS = []


class _DirectLinear(torch.autograd.Function):
    """A fused-block stand-in: y = x W^T + b whose backward accumulates dW / db straight into the
    flat gradient buffer, notifies the owner, and returns None for the parameters (as
    ops/transformer.py's blocks do)."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x)
        ctx.p = (w, b)
        return x @ w.detach().t() + b.detach()

    @staticmethod
    def backward(ctx, dy):
        from ml_trainer_amd.utils.flat import FlatParams
        (x,) = ctx.saved_tensors
        w, b = ctx.p
        fp = FlatParams.owner(w)
        fp.grad_sink(w).add_(dy.t() @ x)
        fp.grad_sink(b).add_(dy.sum(0))
        _EVENTS.append("bwd")  # before the notifications: the last one launches the bucket
        fp.notify_grad_ready(w)
        fp.notify_grad_ready(b)
        return dy @ w.detach(), None, None


class _TwoBlocks(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.l1 = torch.nn.Linear(8, 16)
        self.l2 = torch.nn.Linear(16, 4)

    def forward(self, x):
        return _DirectLinear.apply(torch.relu(_DirectLinear.apply(x, self.l1.weight, self.l1.bias)), self.l2.weight,
                                   self.l2.bias)


def _direct_worker(rank, world, port, out_dir):
    dist_env(rank, world, port)
    dist.init_process_group("gloo")
    from ml_trainer_amd.parallel.ddp import DistributedDataParallel
    torch.manual_seed(5)
    model = _TwoBlocks()
    ddp = DistributedDataParallel(model, bucket_cap_mb=1.0, first_bucket_mb=1.0)  # ONE bucket over both blocks
    assert len(ddp.bucket_sizes_bytes) == 1
    red = ddp._reduce_bucket

    def traced(bi, async_op=True):
        _EVENTS.append("launch")
        return red(bi, async_op)
    ddp._reduce_bucket = traced
    g = torch.Generator().manual_seed(21 + rank)
    x, y = torch.randn(6, 8, generator=g), torch.randn(6, 4, generator=g)
    ((ddp(x) - y) ** 2).mean().backward()
    assert _EVENTS == ["bwd", "bwd", "launch"], _EVENTS  # the bucket waits for BOTH blocks
    torch.save({"g": ddp.flat.grad.clone()}, os.path.join(out_dir, f"d{rank}.pt"))
    dist.destroy_process_group()


def test_ddp_bucket_spanning_two_direct_write_blocks():
    """Regression: a parameter whose gradient is written by a fused backward is reported twice
    (direct notification + the AccumulateGrad post hook, which fires even for a None gradient).
    Counted twice, a bucket spanning two such blocks was all-reduced after the FIRST block, and
    the second block's gradients stayed rank-local. The averaged gradient must equal the
    full-batch gradient on every rank."""
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_direct_worker, args=(world, free_port(), d), nprocs=world, join=True)
        r = [torch.load(os.path.join(d, f"d{i}.pt"), weights_only=True)["g"] for i in range(world)]
        assert torch.equal(r[0], r[1])
        from ml_trainer_amd.utils.flat import FlatParams
        torch.manual_seed(5)
        model = _TwoBlocks()
        fp = FlatParams(model.parameters(), reverse=True)
        xs, ys = [], []
        for rank in range(world):
            g = torch.Generator().manual_seed(21 + rank)
            xs.append(torch.randn(6, 8, generator=g))
            ys.append(torch.randn(6, 4, generator=g))
        sum(((model(x) - y) ** 2).mean() for x, y in zip(xs, ys)).div(world).backward()
        torch.testing.assert_close(r[0], fp.grad, rtol=1e-5, atol=1e-6)


def test_bucket_plan_alpha_beta():
    """The alpha-beta bucket planner: defaults without a backward-time estimate; a comm-bound step
    gets the largest cap; a compute-bound one the smallest cap that keeps the comm stream up."""
    from ml_trainer_amd.parallel.ddp import (DEFAULT_BUCKET_MB, MAX_BUCKET_MB, MIN_BUCKET_MB, allreduce_us,
                                             plan_buckets)
    mb = 2 ** 20
    assert plan_buckets(440 * mb, 8) == (DEFAULT_BUCKET_MB, 4.0)
    assert plan_buckets(440 * mb, 1, bwd_ms=100.0)[0] == DEFAULT_BUCKET_MB
    # BERT-base fp32 grads on 8 ranks: beta*M ~ 2.6 ms << 130 ms of backward -> small buckets
    cap, first = plan_buckets(440 * mb, 8, bwd_ms=130.0)
    assert cap == MIN_BUCKET_MB and first <= cap
    # comm-bound: backward shorter than the bandwidth term -> fewest collectives
    assert plan_buckets(440 * mb, 8, bwd_ms=1.0)[0] == MAX_BUCKET_MB
    # in between: C = M * alpha / (T - beta M), and the model's pieces add up
    t = allreduce_us(440 * mb, 8, alpha_us=25.0, bus_gbps=300.0)
    assert abs(t - (25.0 + 1.75 * 440 * mb / 300e3)) < 1e-6
    cap, _ = plan_buckets(440 * mb, 8, bwd_ms=2.9, alpha_us=25.0, bus_gbps=300.0)
    beta_m = t - 25.0
    assert abs(cap - min(MAX_BUCKET_MB, max(MIN_BUCKET_MB, 440 * 25.0 / (2900.0 - beta_m)))) < 1e-9


def _autoplan_worker(rank, world, port, out_dir, auto, cap, first):
    dist_env(rank, world, port)
    # a cheap wire and a tiny minimum bucket: the planned layout differs from the 32 / 4 MB default
    os.environ["MLT_DDP_MIN_BUCKET_MB"] = "0.0001"
    os.environ["MLT_DDP_ALPHA_US"] = "0.05"
    os.environ["MLT_DDP_BUS_GBPS"] = "1000"
    dist.init_process_group("gloo")
    from ml_trainer_amd.parallel.ddp import DistributedDataParallel
    torch.manual_seed(5)
    model = torch.nn.Sequential(*[torch.nn.Linear(64, 64) for _ in range(6)])
    ddp = (DistributedDataParallel(model) if auto else
           DistributedDataParallel(model, bucket_cap_mb=cap, first_bucket_mb=first))
    opt = torch.optim.SGD(model.parameters(), lr=0.05)
    g = torch.Generator().manual_seed(11 + rank)
    layouts = []
    for _ in range(5):
        x = torch.randn(16, 64, generator=g)
        opt.zero_grad(set_to_none=False)
        ddp(x).pow(2).mean().backward()
        opt.step()
        layouts.append(list(ddp._buckets))
    torch.save({"params": ddp.flat.data.clone(), "plan": ddp.bucket_plan, "layouts": layouts},
               os.path.join(out_dir, f"{'a' if auto else 'f'}{rank}.pt"))
    dist.destroy_process_group()


def test_ddp_autoplan_rebuckets_once_bitwise():
    """DDP without explicit caps times its second synchronised backward, agrees the MAX over ranks at
    the end of that backward (collective, after its buckets were waited for) and rebuilds its buckets
    ONCE from the alpha-beta model (bucket_plan source 'alpha-beta'); training is bitwise equal to
    fixed caps of the same layout, on every rank."""
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_autoplan_worker, args=(world, free_port(), d, True, None, None), nprocs=world, join=True)
        a = [torch.load(os.path.join(d, f"a{r}.pt"), weights_only=True) for r in range(world)]
        plan = a[0]["plan"]
        assert plan["source"] == "alpha-beta" and plan["replans"] == 1 and plan["bwd_ms"] > 0
        assert a[1]["plan"] == plan  # agreed: the same plan on every rank
        lay = a[0]["layouts"]
        assert lay[1] == lay[2] == lay[3] == lay[4]  # rebuilt once, at the end of the 2nd backward
        assert lay[1] != lay[0] and len(lay[1]) > 1
        mp.spawn(_autoplan_worker, args=(world, free_port(), d, False, plan["cap_mb"], plan["first_mb"]),
                 nprocs=world, join=True)
        f = [torch.load(os.path.join(d, f"f{r}.pt"), weights_only=True) for r in range(world)]
        assert f[0]["layouts"][0] == lay[1]
        for r in range(world):
            assert torch.equal(a[r]["params"], f[r]["params"])


def _ab_worker(rank, world, port, out_dir):
    dist_env(rank, world, port)
    for k in ("MLT_DDP_ALPHA_US", "MLT_DDP_BUS_GBPS", "MLT_DDP_MEASURE_AB"):
        os.environ.pop(k, None)
    dist.init_process_group("gloo")
    from ml_trainer_amd.parallel.ddp import DistributedDataParallel
    torch.manual_seed(5)
    model = torch.nn.Sequential(*[torch.nn.Linear(64, 64) for _ in range(4)])
    ddp = DistributedDataParallel(model)
    g = torch.Generator().manual_seed(3 + rank)
    for _ in range(3):
        ddp(torch.randn(8, 64, generator=g)).pow(2).mean().backward()
    torch.save({"plan": ddp.bucket_plan, "grad_bytes": ddp._grad_bytes}, os.path.join(out_dir, f"ab{rank}.pt"))
    dist.destroy_process_group()


def test_ddp_replan_fits_alpha_beta_on_the_live_group():
    """With no MLT_DDP_ALPHA_US / MLT_DDP_BUS_GBPS, the one-time re-plan fits the alpha-beta model on
    the group's own wire (timed all-reduces of two sizes, MAX over ranks): every rank records the same
    measured alpha / bus bandwidth, and the caps are the planner's for exactly those values."""
    from ml_trainer_amd.parallel.ddp import plan_buckets
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_ab_worker, args=(world, free_port(), d), nprocs=world, join=True)
        r = [torch.load(os.path.join(d, f"ab{k}.pt"), weights_only=True) for k in range(world)]
    plan = r[0]["plan"]
    assert r[1]["plan"] == plan
    assert plan["source"] == "alpha-beta" and plan["replans"] == 1
    if plan["ab"] == "measured":  # (a noisy host can give a non-positive slope: then the priors stay)
        assert plan["alpha_us"] > 0 and plan["bus_gbps"] > 0
        cap, first = plan_buckets(r[0]["grad_bytes"], world, plan["bwd_ms"], alpha_us=plan["alpha_us"],
                                  bus_gbps=plan["bus_gbps"])
        assert abs(cap - plan["cap_mb"]) <= 1e-6 * max(1.0, cap) + 1e-3 and first <= cap
    else:
        assert plan["ab"] == "model"
