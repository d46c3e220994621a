"""The native collectives on hardware (reference src/trainer.py:59,98):

* the RCCL ``Communicator`` at world size 1 on the box's GPU -- every collective against its
  torch-computed expectation, plus the health query;
* the LeNet data-parallel step with a real ``ncclAllReduce`` captured inside multi-step
  hipGraphs (W=1 rehearsal of the 8-GPU path) against the fused single-rank step;
* the one-shot xGMI all-reduce failing loudly and fail-stop when a peer never arrives
  (two processes on the one GPU, gloo rendezvous).
"""
import os
import tempfile
import time

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.helpers import dist_env, free_port

pytestmark = pytest.mark.gpu


def _comm(dev):
    from ml_trainer_amd.ops._ext import require_native
    C = require_native()
    return C.Communicator(C.Communicator.unique_id(), 1, 0, dev.index)


def test_rccl_world1_collectives(dev):
    c = _comm(dev)
    assert c.size == 1 and c.rank == 0 and c.async_error() == ""
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(1 << 20, device=dev, generator=g)
    for op in ("sum", "avg", "max", "min"):
        t = x.clone()
        c.all_reduce(t, op)
        torch.testing.assert_close(t, x, rtol=0, atol=0)
    xb = x.to(torch.bfloat16)
    tb = xb.clone()
    c.all_reduce(tb, "sum")
    assert torch.equal(tb, xb)
    out = torch.empty_like(x)
    c.reduce_scatter(x, out, "sum")
    assert torch.equal(out, x)
    out.zero_()
    c.all_gather(x, out)
    assert torch.equal(out, x)
    t = x.clone()
    c.broadcast(t, 0)
    assert torch.equal(t, x)
    out.zero_()
    c.all_to_all(x, out)
    assert torch.equal(out, x)
    i64 = torch.arange(1000, device=dev)
    c.all_reduce(i64, "sum")
    assert torch.equal(i64, torch.arange(1000, device=dev))
    torch.cuda.synchronize()
    assert c.async_error() == ""


def _lenet_engine(dev, seed=0):
    from ml_trainer_amd.models.lenet import MLModel
    from ml_trainer_amd.models.lenet_engine import LeNetStepEngine
    from ml_trainer_amd.ops.optim import build_optimizer
    from ml_trainer_amd.utils.flat import FlatParams
    torch.manual_seed(seed)
    m = MLModel().to(dev)
    flat = FlatParams(m.parameters())
    opt = build_optimizer("sgd", m.parameters(), lr=1e-2, momentum=0.9, flat=flat)
    eng = LeNetStepEngine(m, flat, max_batch=32, optimizer=opt)
    g = torch.Generator().manual_seed(3)
    N = 512
    data = torch.randint(0, 256, (N, 32, 32, 3), dtype=torch.uint8, generator=g)
    targets = torch.randint(0, 10, (N,), generator=g)
    eng.set_dataset(data, targets, batch_size=32)
    eng.start_epoch(torch.randperm(N, generator=torch.Generator().manual_seed(1)).to(torch.int32))
    return eng, flat


def test_lenet_step_with_rccl_allreduce_in_graph(dev):
    """W=1 data-parallel step: backward -> ncclAllReduce(AVG) -> flat optimizer, 4-step graphs."""
    ref, fref = _lenet_engine(dev)
    ref.train_steps(32, 8, use_graph=True, steps_per_graph=4)
    eng, flat = _lenet_engine(dev)
    eng.use_transport(comm=_comm(dev))
    assert eng.dp_transport == "rccl" and not eng.fused
    eng.train_steps(32, 8, use_graph=True, steps_per_graph=4)
    eng.check_transport()
    assert eng.ctrl.tolist() == [8, 8]
    assert eng.captures == 1
    torch.testing.assert_close(flat.data, fref.data, rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(eng.stats, ref.stats, rtol=1e-6, atol=1e-6)


def _late_peer_worker(rank, world, port, out_dir):
    dist_env(rank, world, port)
    dist.init_process_group("gloo")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    os.environ["MLT_XGMI_TIMEOUT_MS"] = "300"
    from ml_trainer_amd.models.lenet_engine import TransportError
    from ml_trainer_amd.parallel.comm import create_xgmi_allreduce
    eng, flat = _lenet_engine(dev)
    xe = create_xgmi_allreduce(None, flat.numel, dev, allow_gloo=True)
    assert xe is not None and xe.timeout_ms == 300
    eng.use_transport(xgmi=xe)
    eng.train_steps(32, 2, use_graph=True, steps_per_graph=1)  # both ranks: healthy steps
    eng.check_transport()
    dist.barrier()
    res = {}
    if rank == 0:  # rank 1 is now "dead": it never launches again
        before = flat.data.clone()
        t0 = time.time()
        raised = False
        try:
            eng.train_steps(32, 1, use_graph=True, steps_per_graph=1)
            eng.check_transport()
        except TransportError:
            raised = True
        res["raised"] = raised
        res["secs"] = time.time() - t0
        res["unchanged"] = bool(torch.equal(flat.data, before))  # the failed step was not applied
        t1 = time.time()
        try:  # sticky: the kernels return at once and the poll raises again
            eng.train_steps(32, 3, use_graph=True, steps_per_graph=1)
            res["sticky_raised"] = False
        except TransportError:
            res["sticky_raised"] = True
        torch.cuda.synchronize()
        res["sticky_secs"] = time.time() - t1
        res["still_unchanged"] = bool(torch.equal(flat.data, before))
        torch.save(res, os.path.join(out_dir, "late.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_xgmi_late_peer_fails_within_one_step():
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_late_peer_worker, args=(2, free_port(), d), nprocs=2, join=True)
        r = torch.load(os.path.join(d, "late.pt"), weights_only=True)
    assert r["raised"], r
    assert r["secs"] < 5.0, r
    assert r["unchanged"] and r["still_unchanged"], r
    assert r["sticky_raised"] and r["sticky_secs"] < 1.0, r


def _partial_peer_worker(rank, world, port, out_dir, algo):
    """Rank r withholds the flags of slices b % 4 == r (fault injection): on each rank half of the
    blocks see their peers and reduce, the other half time out. The step must be applied NOWHERE --
    neither on the slices that reduced nor on the ones that did not (all-or-nothing)."""
    dist_env(rank, world, port)
    dist.init_process_group("gloo")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    os.environ["MLT_XGMI_TIMEOUT_MS"] = "300"
    from ml_trainer_amd.models.lenet_engine import TransportError
    from ml_trainer_amd.parallel.comm import create_xgmi_allreduce
    eng, flat = _lenet_engine(dev)
    xe = create_xgmi_allreduce(None, flat.numel, dev, allow_gloo=True)
    assert xe is not None
    xe.algo = algo
    eng.use_transport(xgmi=xe)
    eng.train_steps(32, 2, use_graph=True, steps_per_graph=1)  # healthy steps
    eng.check_transport()
    dist.barrier()
    before = flat.data.clone()
    xe.fault = 1  # graphs are captured afresh below (use_transport clears them): the fault is live
    eng.use_transport(xgmi=xe)
    raised = False
    try:
        eng.train_steps(32, 1, use_graph=True, steps_per_graph=1)
        eng.check_transport()
    except TransportError:
        raised = True
    torch.cuda.synchronize()
    torch.save({"raised": raised, "unchanged": bool(torch.equal(flat.data, before))},
               os.path.join(out_dir, f"p{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("algo", [0, 1])
def test_xgmi_partial_peer_step_all_or_nothing(algo):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_partial_peer_worker, args=(2, free_port(), d, algo), nprocs=2, join=True)
        r = [torch.load(os.path.join(d, f"p{i}.pt"), weights_only=True) for i in range(2)]
    for i in range(2):
        assert r[i]["raised"], (i, r)
        assert r[i]["unchanged"], (i, r)


def _ddp_avg_worker(rank, world, port, out_dir):
    """Native DDP on the GPU must AVERAGE: the synced gradient equals the mean of the ranks'
    local gradients (no_sync backward of the same batch), not their sum."""
    dist_env(rank, world, port)
    dist.init_process_group("gloo")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    import torch.nn.functional as F
    from ml_trainer_amd.models.bert import BertClassifier, bert_config
    from ml_trainer_amd.parallel.ddp import DistributedDataParallel
    torch.manual_seed(rank)
    m = BertClassifier(bert_config("bert-tiny")).to(dev)
    ddp = DistributedDataParallel(m, bucket_cap_mb=1.0, first_bucket_mb=0.5)
    g = torch.Generator().manual_seed(11 + rank)
    ids = torch.randint(5, 1000, (2, 128), generator=g).to(dev)
    y = torch.randint(0, 2, (2,), generator=g).to(dev)
    ddp.flat.grad.zero_()
    with ddp.no_sync():
        F.cross_entropy(ddp(ids), y).backward()
    local = ddp.flat.grad.clone()
    ddp.flat.grad.zero_()
    F.cross_entropy(ddp(ids), y).backward()
    torch.cuda.synchronize()
    torch.save({"local": local.cpu(), "synced": ddp.flat.grad.cpu()}, os.path.join(out_dir, f"a{rank}.pt"))
    dist.destroy_process_group()


def test_ddp_gpu_averages_not_sums():
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_ddp_avg_worker, args=(2, free_port(), d), nprocs=2, join=True)
        r = [torch.load(os.path.join(d, f"a{i}.pt"), weights_only=True) for i in range(2)]
    mean = (r[0]["local"] + r[1]["local"]) / 2
    assert not torch.equal(r[0]["local"], r[1]["local"])
    for i in range(2):
        torch.testing.assert_close(r[i]["synced"], mean, rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("zero", [False, True])
def test_ddp_native_comm_single_rank_bit_equal(dev, zero):
    """BERT-tiny DDP (and ZeRO-1) with its buckets reduced by the native RCCL communicator (size-1
    rehearsal of the W > 1 path: dedicated high-priority comm stream, hipEvent edges, AVG) gives
    gradients / weights bit-equal to the same model without any communication."""
    import torch.nn.functional as F
    from ml_trainer_amd.models.bert import BertClassifier, bert_config
    from ml_trainer_amd.ops._ext import require_native
    from ml_trainer_amd.ops.optim import FusedAdamW
    from ml_trainer_amd.parallel.ddp import DistributedDataParallel
    from ml_trainer_amd.parallel.zero import ZeroDataParallel
    C = require_native()
    g = torch.Generator().manual_seed(3)
    ids = torch.randint(5, 1000, (2, 128), generator=g).to(dev)
    y = torch.randint(0, 2, (2,), generator=g).to(dev)
    out = []
    for native in (False, True):
        torch.manual_seed(0)
        m = BertClassifier(bert_config("bert-tiny")).to(dev)
        comm = C.Communicator(C.Communicator.unique_id(), 1, 0, dev.index) if native else False
        cls = ZeroDataParallel if zero else DistributedDataParallel
        ddp = cls(m, bucket_cap_mb=1.0, first_bucket_mb=0.5, comm=comm)
        assert ddp.comm_backend == ("native-rccl" if native else "torch.distributed-none")
        opt = ddp.make_optimizer(FusedAdamW, lr=1e-3) if zero else FusedAdamW(m.parameters(), lr=1e-3, flat=ddp.flat)
        for _ in range(3):
            opt.zero_grad(set_to_none=False)
            F.cross_entropy(ddp(ids), y).backward()
            opt.step()
        if zero:
            ddp.wait_parameters()
        torch.cuda.synchronize()
        out.append((ddp.flat.data.clone(), ddp.flat.grad.clone()))
    assert torch.equal(out[0][1], out[1][1])
    assert torch.equal(out[0][0], out[1][0])
