"""Two ranks sharing the one GPU of the test box (gloo process group; RCCL needs one GPU per
rank): the data-parallel paths that are not the in-graph RCCL one -- the LeNet engine's
torch.distributed fallback step and the native DDP wrapper around the BERT blocks with direct
flat-gradient writes (grad_ready notifications) -- must keep the ranks bit-identical."""
import os
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.helpers import dist_env, free_port

pytestmark = pytest.mark.gpu


def _lenet_worker(rank, world, port, out_dir):
    dist_env(rank, world, port)
    dist.init_process_group("gloo")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    from ml_trainer_amd.models.lenet import MLModel
    from ml_trainer_amd.models.lenet_engine import LeNetStepEngine
    from ml_trainer_amd.ops.optim import build_optimizer
    from ml_trainer_amd.parallel.sampler import shard_indices
    from ml_trainer_amd.utils.flat import FlatParams
    torch.manual_seed(rank)  # different init per rank: broadcast must fix it
    m = MLModel().to(dev)
    flat = FlatParams(m.parameters())
    dist.broadcast(flat.data, src=0)
    opt = build_optimizer("sgd", m.parameters(), lr=1e-2, momentum=0.9, flat=flat)
    eng = LeNetStepEngine(m, flat, max_batch=16, optimizer=opt, world_size=world)
    assert eng.comm is None  # gloo: torch.distributed fallback
    g = torch.Generator().manual_seed(3)
    N = 256
    data = torch.randint(0, 256, (N, 32, 32, 3), dtype=torch.uint8, generator=g)
    targets = torch.randint(0, 10, (N,), generator=g)
    eng.set_dataset(data, targets, batch_size=16)
    idx = shard_indices(N, world, rank, shuffle=True, seed=0, epoch=0)
    eng.start_epoch(torch.as_tensor(idx, dtype=torch.int32))
    eng.train_steps(16, 6, use_graph=True)
    torch.cuda.synchronize()
    torch.save({"p": flat.data.cpu(), "ctrl": eng.ctrl.cpu()}, os.path.join(out_dir, f"l{rank}.pt"))
    dist.destroy_process_group()


def _bert_worker(rank, world, port, out_dir):
    dist_env(rank, world, port)
    dist.init_process_group("gloo")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    import torch.nn.functional as F
    from ml_trainer_amd.models.bert import BertClassifier, bert_config
    from ml_trainer_amd.ops.optim import FusedAdamW
    from ml_trainer_amd.parallel.ddp import DistributedDataParallel
    torch.manual_seed(rank)
    m = BertClassifier(bert_config("bert-tiny")).to(dev)
    ddp = DistributedDataParallel(m, bucket_cap_mb=1.0, first_bucket_mb=0.5)
    opt = FusedAdamW(m.parameters(), lr=1e-3, flat=ddp.flat)
    g = torch.Generator().manual_seed(11 + rank)
    ids = torch.randint(5, 1000, (2, 128), generator=g).to(dev)
    y = torch.randint(0, 2, (2,), generator=g).to(dev)
    for _ in range(3):
        opt.zero_grad(set_to_none=False)
        F.cross_entropy(ddp(ids), y).backward()
        opt.step()
    torch.cuda.synchronize()
    torch.save({"p": ddp.flat.data.cpu(), "g": ddp.flat.grad.cpu()}, os.path.join(out_dir, f"b{rank}.pt"))
    dist.destroy_process_group()


def _bert_autoplan_worker(rank, world, port, out_dir):
    dist_env(rank, world, port)
    for k in ("MLT_DDP_ALPHA_US", "MLT_DDP_BUS_GBPS", "MLT_DDP_MEASURE_AB", "MLT_DDP_AUTOPLAN"):
        os.environ.pop(k, None)
    dist.init_process_group("gloo")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    import torch.nn.functional as F
    from ml_trainer_amd.models.bert import BertClassifier, bert_config
    from ml_trainer_amd.ops.optim import FusedAdamW
    from ml_trainer_amd.parallel.ddp import DistributedDataParallel
    torch.manual_seed(rank)
    m = BertClassifier(bert_config("bert-tiny")).to(dev)
    ddp = DistributedDataParallel(m)  # no caps: timed backward + alpha-beta fit on the live group
    opt = FusedAdamW(m.parameters(), lr=1e-3, flat=ddp.flat)
    g = torch.Generator().manual_seed(11 + rank)
    ids = torch.randint(5, 1000, (2, 128), generator=g).to(dev)
    y = torch.randint(0, 2, (2,), generator=g).to(dev)
    for _ in range(4):
        opt.zero_grad(set_to_none=False)
        F.cross_entropy(ddp(ids), y).backward()
        opt.step()
    torch.cuda.synchronize()
    torch.save({"p": ddp.flat.data.cpu(), "plan": ddp.bucket_plan}, os.path.join(out_dir, f"b{rank}.pt"))
    dist.destroy_process_group()


def _run(fn, world=2, *extra):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(fn, args=(world, free_port(), d, *extra), nprocs=world, join=True)
        return [torch.load(os.path.join(d, f), weights_only=True) for f in sorted(os.listdir(d))]


def test_lenet_engine_two_ranks_stay_in_sync():
    r = _run(_lenet_worker)
    assert torch.equal(r[0]["p"], r[1]["p"])
    assert r[0]["ctrl"].tolist() == [6, 6]


def test_bert_ddp_autoplan_fits_alpha_beta_on_gpu():
    """DDP on device gradients with no caps: the one-time re-plan times the backward, fits alpha /
    bus bandwidth with all-reduces of device buffers through the bucket path, and every rank ends
    with the same plan and identical weights."""
    r = _run(_bert_autoplan_worker)
    assert r[0]["plan"] == r[1]["plan"]
    assert r[0]["plan"]["source"] == "alpha-beta" and r[0]["plan"]["ab"] in ("measured", "model")
    assert torch.equal(r[0]["p"], r[1]["p"])


def test_bert_ddp_direct_grads_two_ranks():
    r = _run(_bert_worker)
    assert torch.equal(r[0]["p"], r[1]["p"])  # all-reduced grads -> identical updates
    assert torch.equal(r[0]["g"], r[1]["g"])
    assert r[0]["g"].abs().sum() > 0


def _xgmi_worker(rank, world, port, out_dir, algo=0):
    dist_env(rank, world, port)
    dist.init_process_group("gloo")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    from ml_trainer_amd.parallel.comm import create_xgmi_allreduce
    x = create_xgmi_allreduce(None, 70000, dev, allow_gloo=True)  # includes the self-test of both algorithms
    assert x is not None and x.two_shot_ok  # both algorithms passed the self-test on every rank
    x.algo = algo
    res = []
    g = torch.Generator().manual_seed(100 + rank)
    for it in range(5):  # odd/even parities, sizes with a float4 tail
        n = [62006, 70000, 13, 4096, 62006][it]
        t = torch.randn(n, generator=g).to(dev)
        ref = t.cpu().clone()
        dist.all_reduce(ref)  # gloo SUM on the host copy
        x.all_reduce(t, average=True)
        torch.cuda.synchronize()
        res.append(bool(torch.equal(t.cpu(), ref * 0.5)))
    # the LeNet data-parallel step with the one-shot kernel inside 2-step hipGraphs
    from ml_trainer_amd.models.lenet import MLModel
    from ml_trainer_amd.models.lenet_engine import LeNetStepEngine
    from ml_trainer_amd.ops.optim import build_optimizer
    from ml_trainer_amd.parallel.sampler import shard_indices
    from ml_trainer_amd.utils.flat import FlatParams
    torch.manual_seed(0)
    m = MLModel().to(dev)
    flat = FlatParams(m.parameters())
    opt = build_optimizer("sgd", m.parameters(), lr=1e-2, momentum=0.9, flat=flat)
    eng = LeNetStepEngine(m, flat, max_batch=16, optimizer=opt, world_size=world)
    xe = create_xgmi_allreduce(None, flat.numel, dev, allow_gloo=True)
    xe.algo = algo
    eng.use_transport(xgmi=xe)
    assert eng.dp_transport == ("xgmi-twoshot" if algo else "xgmi-oneshot")
    gd = torch.Generator().manual_seed(3)
    N = 256
    data = torch.randint(0, 256, (N, 32, 32, 3), dtype=torch.uint8, generator=gd)
    targets = torch.randint(0, 10, (N,), generator=gd)
    eng.set_dataset(data, targets, batch_size=16)
    eng.start_epoch(torch.as_tensor(shard_indices(N, world, rank, shuffle=True, seed=0, epoch=0), dtype=torch.int32))
    eng.train_steps(16, 6, use_graph=True, steps_per_graph=2)
    torch.cuda.synchronize()
    torch.save({"ok": torch.tensor(res), "err": torch.tensor([x.error(), xe.error()]), "p": flat.data.cpu()},
               os.path.join(out_dir, f"x{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("algo", [0, 1])
def test_xgmi_oneshot_allreduce_two_ranks_one_gpu(algo):
    """IPC-shared uncached regions + flag barrier + rank-ordered sums; two processes on the one
    GPU of the box stand in for two xGMI peers (same code path, the peer is just local).
    algo 0: one-shot (pull), 1: two-shot (push reduce-scatter + push all-gather)."""
    r = _run(_xgmi_worker, 2, algo)
    for d in r:
        assert d["ok"].all(), d["ok"]
        assert d["err"].tolist() == [0, 0]
    assert torch.equal(r[0]["p"], r[1]["p"])
    # same updates as the torch.distributed fallback path (AVG of two = exact)
    ref = _run(_lenet_worker)
    assert torch.equal(r[0]["p"], ref[0]["p"])


def _xgmi_sizes_worker(rank, world, port, out_dir, algo):
    dist_env(rank, world, port)
    dist.init_process_group("gloo")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    from ml_trainer_amd.parallel.comm import create_xgmi_allreduce
    os.environ["MLT_XGMI_TIMEOUT_MS"] = "20000"
    x = create_xgmi_allreduce(None, 70000, dev, allow_gloo=True)
    assert x is not None and x.two_shot_ok
    x.algo = algo
    res = []
    g = torch.Generator().manual_seed(200 + rank)
    inv = torch.tensor(1.0 / world, dtype=torch.float32)
    # odd lengths, lengths below 4 * world (empty / partial slices of the two-shot split), a float4
    # tail, and the LeNet bucket; small-integer values keep every sum exact in any order
    for n in (1, 3, 4 * world - 1, 4 * world + 1, 13, 4099, 62006, 69999):
        t = torch.randint(-64, 64, (n,), generator=g).float()
        ref = t.clone()
        dist.all_reduce(ref)  # gloo SUM on the host copy (exact)
        td = t.to(dev)
        x.all_reduce(td, average=True)
        torch.cuda.synchronize()
        res.append(bool(torch.equal(td.cpu(), ref * inv)))
    torch.save({"ok": torch.tensor(res), "err": torch.tensor([x.error()])}, os.path.join(out_dir, f"s{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [3, 4, 8])
@pytest.mark.parametrize("algo", [0, 1])
def test_xgmi_allreduce_three_four_eight_ranks_one_gpu(world, algo):
    """The one-shot / two-shot kernels at W = 3, 4, 8 (the 4- and 8-GPU node's code paths: slice and
    flag indexing, partial and empty slices; W = 8 is what the node's vote runs) rehearsed as W
    processes on the box's one GPU; every result bit-exact against the host sum."""
    r = _run(_xgmi_sizes_worker, world, algo)
    assert len(r) == world
    for d in r:
        assert d["ok"].all(), d["ok"]
        assert d["err"].tolist() == [0]


def _fused_dp_worker(rank, world, port, out_dir):
    """bf16 LeNet data-parallel step over xGMI: the two-launch step (exchange folded into the batch-
    reduction kernel) and its two-phase form vs the four-launch step (reduction, one-shot all-reduce,
    apply)."""
    dist_env(rank, world, port)
    dist.init_process_group("gloo")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    os.environ["MLT_XGMI_TIMEOUT_MS"] = "20000"
    from ml_trainer_amd.models.lenet import MLModel
    from ml_trainer_amd.models.lenet_engine import LeNetStepEngine
    from ml_trainer_amd.ops.optim import build_optimizer
    from ml_trainer_amd.parallel.comm import create_xgmi_allreduce
    from ml_trainer_amd.parallel.sampler import shard_indices
    from ml_trainer_amd.utils.flat import FlatParams
    out = {}
    gd = torch.Generator().manual_seed(3)
    N = 64 * world
    data = torch.randint(0, 256, (N, 32, 32, 3), dtype=torch.uint8, generator=gd)
    targets = torch.randint(0, 10, (N,), generator=gd)
    for variant, fused in (("1", True), ("0", False), ("two", True)):
        torch.manual_seed(0)
        m = MLModel().to(dev)
        flat = FlatParams(m.parameters())
        opt = build_optimizer("adamw", m.parameters(), lr=1e-3, weight_decay=0.01, flat=flat)
        eng = LeNetStepEngine(m, flat, max_batch=8, optimizer=opt, world_size=world, precision="bf16")
        xe = create_xgmi_allreduce(None, flat.numel, dev, allow_gloo=True)
        assert xe is not None
        xe.algo = 0
        xe.fused_two = variant == "two"  # the exchange's two-phase form (chunk owners publish the sums)
        eng.use_transport(xgmi=xe, fused=fused)
        assert eng.dp_transport == ("xgmi-fused" if fused else "xgmi-oneshot")
        eng.set_dataset(data, targets, batch_size=8)
        eng.start_epoch(torch.as_tensor(shard_indices(N, world, rank, shuffle=True, seed=0, epoch=0),
                                        dtype=torch.int32))
        if fused:  # a dry launch of the step graph first (bench.py's pre-warm): must change nothing
            assert eng.prewarm(8, 6, steps_per_graph=3) == 1
        eng.train_steps(8, 6, use_graph=True, steps_per_graph=3)
        eng.check_transport()
        torch.cuda.synchronize()
        out[f"p{variant}"] = flat.data.cpu()
        out[f"g{variant}"] = flat.grad.cpu()
        out[f"nodes{variant}"] = eng.eng.graph_nodes(eng._train_mode(), 8, 3)
        out[f"err{variant}"] = xe.error()
        dist.barrier()
    torch.save(out, os.path.join(out_dir, f"f{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_lenet_bf16_fused_dp_matches_four_launch(world):
    """Two launches per data-parallel step (and the exchange's two-phase form), bitwise equal to the four-launch step and identical on every rank (W = 8: the
    node's size, as 8 processes on the box's one GPU) -- the fused runs after a dry pre-warm launch
    of their graph (no exchange published, no launch counter advanced)."""
    r = _run(_fused_dp_worker, world)
    assert len(r) == world
    for d in r:
        assert d["err1"] == 0 and d["err0"] == 0 and d["errtwo"] == 0
        assert torch.equal(d["p1"], d["p0"]) and torch.equal(d["g1"], d["g0"])
        assert torch.equal(d["ptwo"], d["p0"]) and torch.equal(d["gtwo"], d["g0"])
        assert d["nodestwo"] == 6
        assert (d["nodes1"], d["nodes0"]) == (6, 12)  # 2 / 4 kernels per step
        assert torch.equal(d["p1"], r[0]["p1"])


def _selftest_worker(rank, world, port, out_dir, inject, two=False):
    """Transport bring-up of the bf16 engine at W = 2 (both ranks on the box's GPU): the fused
    exchange's own self-test runs before it may carry a step; MLT_XGMI_INJECT_FAULT="0:2" makes
    rank 0 publish corrupted values, which rank 1's check catches -- then EVERY rank rejects the
    fused step (MIN vote) and trains on the four-launch step, replicas still identical."""
    dist_env(rank, world, port)
    os.environ["MLT_XGMI_ALLOW_GLOO"] = "1"
    os.environ["MLT_XGMI_TIMEOUT_MS"] = "20000"
    if inject:
        os.environ["MLT_XGMI_INJECT_FAULT"] = "0:2"
    if two:
        os.environ["MLT_XGMI_FUSED_TWO"] = "1"
    dist.init_process_group("gloo")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    from ml_trainer_amd.models.lenet import MLModel
    from ml_trainer_amd.models.lenet_engine import LeNetStepEngine
    from ml_trainer_amd.ops.optim import build_optimizer
    from ml_trainer_amd.parallel.sampler import shard_indices
    from ml_trainer_amd.utils.flat import FlatParams
    torch.manual_seed(0)
    m = MLModel().to(dev)
    flat = FlatParams(m.parameters())
    opt = build_optimizer("sgd", m.parameters(), lr=1e-2, momentum=0.9, flat=flat)
    eng = LeNetStepEngine(m, flat, max_batch=8, optimizer=opt, world_size=world, precision="bf16")
    gd = torch.Generator().manual_seed(3)
    N = 64 * world
    data = torch.randint(0, 256, (N, 32, 32, 3), dtype=torch.uint8, generator=gd)
    targets = torch.randint(0, 10, (N,), generator=gd)
    eng.set_dataset(data, targets, batch_size=8)
    eng.start_epoch(torch.as_tensor(shard_indices(N, world, rank, shuffle=True, seed=0, epoch=0), dtype=torch.int32))
    eng.train_steps(8, 4, use_graph=True, steps_per_graph=2)
    eng.check_transport()
    torch.cuda.synchronize()
    out = {"ok": getattr(eng, "fused_selftest_ok", None), "ok2": getattr(eng, "fused2_selftest_ok", None),
           "two": eng.fused_two, "transport": eng.dp_transport, "times": eng.transport_times_ms, "p": flat.data.cpu()}
    torch.save(out, os.path.join(out_dir, f"s{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("inject,two", [(False, False), (True, False), (False, True)])
def test_fused_exchange_selftest_and_fallback(inject, two):
    """two: MLT_XGMI_FUSED_TWO=1 -- the two-phase form runs its own self-test and, when the fused
    step is taken, carries it."""
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_selftest_worker, args=(2, free_port(), d, inject, two), nprocs=2, join=True)
        r = [torch.load(os.path.join(d, f"s{i}.pt"), weights_only=True) for i in range(2)]
    for x in r:
        assert x["ok"] is (not inject), x
        if two:
            assert x["ok2"] is True and "xgmi-fused2" in x["times"], x
            assert x["two"] is (x["transport"] == "xgmi-fused"), x
        if inject:
            assert x["transport"] in ("xgmi-oneshot", "xgmi-twoshot"), x["transport"]
        else:
            assert x["transport"] in ("xgmi-fused", "xgmi-oneshot", "xgmi-twoshot"), x["transport"]
            assert "xgmi-fused" in x["times"] and "reduce" in x["times"]
    assert r[0]["transport"] == r[1]["transport"]
    assert torch.equal(r[0]["p"], r[1]["p"])


def _bert_zero_worker(rank, world, port, out_dir):
    """ZeRO-1 around the fused BERT blocks (direct flat-gradient writes -> reduce-scatter, sharded
    fused AdamW on the GPU, all-gather + bf16 shadow re-cast) against replicated DDP."""
    dist_env(rank, world, port)
    dist.init_process_group("gloo")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    import torch.nn.functional as F
    from ml_trainer_amd.models.bert import BertClassifier, bert_config
    from ml_trainer_amd.ops.optim import FusedAdamW
    from ml_trainer_amd.parallel.ddp import DistributedDataParallel
    from ml_trainer_amd.parallel.zero import ZeroDataParallel
    out = {}
    for kind in ("ddp", "zero"):
        torch.manual_seed(rank)
        m = BertClassifier(bert_config("bert-tiny")).to(dev)
        if kind == "zero":
            w = ZeroDataParallel(m, bucket_cap_mb=1.0, first_bucket_mb=0.5)
            opt = w.make_optimizer(FusedAdamW, lr=1e-3)
        else:
            w = DistributedDataParallel(m, bucket_cap_mb=1.0, first_bucket_mb=0.5)
            opt = FusedAdamW(m.parameters(), lr=1e-3, flat=w.flat)
        g = torch.Generator().manual_seed(11 + rank)
        ids = torch.randint(5, 1000, (2, 128), generator=g).to(dev)
        y = torch.randint(0, 2, (2,), generator=g).to(dev)
        for _ in range(3):
            opt.zero_grad(set_to_none=False)
            F.cross_entropy(w(ids), y).backward()
            opt.step()
        w.wait_parameters() if kind == "zero" else None
        torch.cuda.synchronize()
        out[kind] = {k: v.float().cpu() for k, v in w.state_dict().items()}
    torch.save(out, os.path.join(out_dir, f"z{rank}.pt"))
    dist.destroy_process_group()


def test_bert_zero1_two_ranks_matches_ddp():
    r = _run(_bert_zero_worker)
    for k, v in r[0]["ddp"].items():
        assert torch.equal(r[0]["zero"][k], r[1]["zero"][k])
        torch.testing.assert_close(r[0]["zero"][k], v, rtol=2e-3, atol=2e-4)


def _bert_comm_worker(rank, world, port, out_dir):
    """The DDP side-stream path (timing events + bf16 wire dtype) around the fused BERT blocks."""
    dist_env(rank, world, port)
    dist.init_process_group("gloo")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    import torch.nn.functional as F
    from ml_trainer_amd.models.bert import BertClassifier, bert_config
    from ml_trainer_amd.parallel.ddp import DistributedDataParallel
    out = {}
    for tag, cd in (("fp32", None), ("bf16", torch.bfloat16)):
        torch.manual_seed(rank)
        m = BertClassifier(bert_config("bert-tiny")).to(dev)
        ddp = DistributedDataParallel(m, bucket_cap_mb=1.0, first_bucket_mb=0.5, comm_dtype=cd, timing=True)
        g = torch.Generator().manual_seed(11 + rank)
        ids = torch.randint(5, 1000, (2, 128), generator=g).to(dev)
        y = torch.randint(0, 2, (2,), generator=g).to(dev)
        for _ in range(3):
            ddp.flat.zero_grad()
            F.cross_entropy(ddp(ids), y).backward()
        torch.cuda.synchronize()
        out[tag] = ddp.flat.grad.cpu()
        st = ddp.comm_stats()
        out[tag + "_stats"] = torch.tensor([st["steps_timed"], st["buckets"], st["allreduce_ms"], st["overlap_pct"],
                                            st["fwd_bwd_ms"]], dtype=torch.float64)
    torch.save(out, os.path.join(out_dir, f"c{rank}.pt"))
    dist.destroy_process_group()


def test_bert_ddp_timing_and_bf16_comm_two_ranks():
    r = _run(_bert_comm_worker)
    for tag in ("fp32", "bf16"):
        assert torch.equal(r[0][tag], r[1][tag])
        steps, buckets, ar_ms, ov, fb = r[0][tag + "_stats"].tolist()
        assert steps == 3 and buckets >= 2 and ar_ms > 0 and 0.0 <= ov <= 100.0 and fb > 0
    a, b = r[0]["fp32"], r[0]["bf16"]
    assert (a - b).norm() / a.norm() < 2e-2
