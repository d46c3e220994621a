"""The exact path ``main.py`` takes on the 8-GPU node, rehearsed with 2 ranks on the one GPU of
the test box (gloo group, MLT_SAME_DEVICE=1, xGMI kernels allowed over gloo):
``Trainer(MLModel(), datasets, is_parallel=True).fit()`` -> native DDP wrap -> fused LeNet step
engine with ``world_size=2`` -> transport vote (xGMI one-/two-shot) -> in-graph all-reduce ->
rank-0 ``module.``-prefixed checkpoint (reference src/trainer.py:57-64,97-101,252-256).

Checks: the ranks end bit-identical; model.pth keys carry ``module.``; the global history equals
a one-rank run at the same global batch (32 = 2 x 16, reference batch semantics) within 1e-4."""
import os
import tempfile

import pytest
import torch
import torch.multiprocessing as mp

from tests.helpers import dist_env, free_port

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, out_dir, precision):
    dist_env(rank, world, port)
    os.environ["MLT_SAME_DEVICE"] = "1"
    os.environ["MLT_XGMI_ALLOW_GLOO"] = "1"
    os.environ["MLT_LENET_FUSED_DP"] = "2"  # the fused step once it passed its self-test (no timed vote)
    from ml_trainer_amd.data.cifar10 import SyntheticCIFAR10
    from ml_trainer_amd.data.transforms import Compose, Normalize, ToTensor
    from ml_trainer_amd.models.lenet import MLModel
    from ml_trainer_amd.trainer import Trainer
    tf = Compose([ToTensor(), Normalize((0.4914, 0.4822, 0.4465), (0.2023, 0.1994, 0.2010))])
    train = SyntheticCIFAR10(512, True, transform=tf, seed=3, learnable=True)
    val = SyntheticCIFAR10(128, False, transform=tf, seed=3, learnable=True)
    mdir = os.path.join(out_dir, "model")
    os.makedirs(mdir, exist_ok=True)
    torch.manual_seed(5)
    tr = Trainer(MLModel(), datasets=(train, val), epochs=2, batch_size=32, is_parallel=True, save_history=True,
                 options={"global_metrics": True, "progress": False, "use_engine": True, "precision": precision,
                          "steps_per_graph": 4},
                 backend="gloo", metric="accuracy", lr=1e-2, model_dir=mdir)
    tr.fit()
    eng = tr._engine
    res = {"p": tr.flat.data.detach().cpu().clone(), "history": tr.history, "world": tr.world_size,
           "transport": eng.dp_transport if eng is not None else None}
    if rank == 0:
        sd = torch.load(os.path.join(mdir, "model.pth"), weights_only=True)
        res["keys"] = sorted(sd.keys())
    torch.save(res, os.path.join(out_dir, f"r{rank}.pt"))
    import torch.distributed as dist
    dist.barrier()
    dist.destroy_process_group()


def _run(world, precision):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, free_port(), d, precision), nprocs=world, join=True)
        return [torch.load(os.path.join(d, f"r{i}.pt"), weights_only=False) for i in range(world)]


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_trainer_is_parallel_two_ranks_matches_one(precision):
    two = _run(2, precision)
    one = _run(1, precision)[0]
    assert two[0]["world"] == 2 and one["world"] == 1
    expect = ("xgmi-fused",) if precision == "bf16" else ("xgmi-oneshot", "xgmi-twoshot")
    assert two[0]["transport"] in expect, two[0]["transport"]
    assert torch.equal(two[0]["p"], two[1]["p"])  # replicas bit-identical
    assert all(k.startswith("module.") for k in two[0]["keys"]), two[0]["keys"]
    assert "module.conv1.weight" in two[0]["keys"]
    h2, h1 = two[0]["history"], one["history"]
    assert h2["epochs"] == h1["epochs"] == [1, 2]
    for k in ("train_loss", "val_loss", "train_metric", "val_metric"):
        for a, b in zip(h2[k], h1[k]):
            assert abs(a - b) <= 1e-4 * max(1.0, abs(b)), (k, h2[k], h1[k])
    rel = (two[0]["p"] - one["p"]).norm() / one["p"].norm()
    assert rel < 1e-4, rel.item()


def _fault_resume_worker(rank, world, port, out_dir, asym=False):
    """Epoch 1 healthy (checkpointed: model.pth + trainer_state.pt), then the xGMI transport's fault
    injection makes epoch 2 fail with TransportError on EVERY rank -- after some gradient slices
    were applied on one rank and not the other (the fused exchange applies per slice). A fresh
    Trainer(resume=True) must restore bit-identical replicas from the checkpoint and train on.
    asym: only rank 0 withholds its granules (its peers' polls time out while its own succeed, so
    rank 0 applies that step whole and rank 1 only partly -- the replicas silently diverge -- and
    rank 1's sticky error then starves rank 0 on the next step): both must still raise."""
    dist_env(rank, world, port)
    os.environ["MLT_SAME_DEVICE"] = "1"
    os.environ["MLT_XGMI_ALLOW_GLOO"] = "1"
    os.environ["MLT_LENET_FUSED_DP"] = "2"  # the fused step once it passed its self-test (no timed vote)
    os.environ["MLT_XGMI_TIMEOUT_MS"] = "300"
    from ml_trainer_amd.data.cifar10 import SyntheticCIFAR10
    from ml_trainer_amd.data.transforms import Compose, Normalize, ToTensor
    from ml_trainer_amd.models.lenet import MLModel
    from ml_trainer_amd.models.lenet_engine import TransportError
    from ml_trainer_amd.trainer import Trainer
    tf = Compose([ToTensor(), Normalize((0.4914, 0.4822, 0.4465), (0.2023, 0.1994, 0.2010))])
    train = SyntheticCIFAR10(512, True, transform=tf, seed=3, learnable=True)
    val = SyntheticCIFAR10(128, False, transform=tf, seed=3, learnable=True)
    mdir = os.path.join(out_dir, "model")
    os.makedirs(mdir, exist_ok=True)
    opts = {"progress": False, "use_engine": True, "precision": "bf16", "steps_per_graph": 4,
            "save_trainer_state": True}

    def mk(resume):
        torch.manual_seed(5)
        return Trainer(MLModel(), datasets=(train, val), epochs=2, batch_size=32, is_parallel=True,
                       options=dict(opts, resume=resume), backend="gloo", metric="accuracy", lr=1e-2,
                       model_dir=mdir)
    tr = mk(False)
    tr.epochs = 1
    tr.fit()
    ck = tr.flat.data.detach().cpu().clone()
    eng = tr._engine
    res = {"transport": eng.dp_transport}
    if rank == 0 or not asym:
        eng.xgmi.fault = 1
    eng.use_transport(xgmi=eng.xgmi)  # recapture with the fault live
    tr.epochs, tr.start_epoch = 2, 2
    try:
        tr.fit()
        res["raised"] = False
    except TransportError:
        res["raised"] = True
    import torch.distributed as dist
    res["diverged_from_ckpt"] = not torch.equal(tr.flat.data.detach().cpu(), ck)
    res["failed_p"] = tr.flat.data.detach().cpu().clone()
    dist.barrier()
    tr2 = mk(True)
    res["resumed_p"] = tr2.flat.data.detach().cpu().clone()
    res["ckpt_p"] = ck
    res["start_epoch"] = tr2.start_epoch
    tr2.fit()  # epoch 2 again, healthy transport
    res["final_p"] = tr2.flat.data.detach().cpu().clone()
    res["final_err"] = tr2._engine.xgmi.error()
    torch.save(res, os.path.join(out_dir, f"q{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("asym", [False, True])
def test_fused_dp_transport_error_then_resume_restores_replicas(asym):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_fault_resume_worker, args=(2, free_port(), d, asym), nprocs=2, join=True)
        r = [torch.load(os.path.join(d, f"q{i}.pt"), weights_only=False) for i in range(2)]
    assert r[0]["transport"] == "xgmi-fused"
    assert r[0]["raised"] and r[1]["raised"]
    assert r[0]["start_epoch"] == 2
    if asym:
        assert not torch.equal(r[0]["failed_p"], r[1]["failed_p"])  # diverged before the error surfaced
    for i in range(2):
        assert r[i]["diverged_from_ckpt"]  # the failed step was applied on the slices whose peers arrived
        assert torch.equal(r[i]["resumed_p"], r[i]["ckpt_p"])  # restored from model.pth exactly
        assert r[i]["final_err"] == 0
    assert torch.equal(r[0]["resumed_p"], r[1]["resumed_p"])
    assert torch.equal(r[0]["final_p"], r[1]["final_p"])  # and in lock-step again after training on
