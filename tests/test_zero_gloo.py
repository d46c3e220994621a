"""ZeRO-1 (parallel/zero.py) over gloo, world_size 2 on CPU: sharded AdamW must track replicated DDP."""
import os
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.helpers import TensorCifar, dist_env, free_port


def _model():
    return torch.nn.Sequential(torch.nn.Linear(8, 33), torch.nn.ReLU(), torch.nn.Linear(33, 17),
                               torch.nn.ReLU(), torch.nn.Linear(17, 4))


def _zero_worker(rank, world, port, out_dir):
    dist_env(rank, world, port)
    dist.init_process_group("gloo")
    from ml_trainer_amd.ops.optim import FusedAdamW
    from ml_trainer_amd.parallel.ddp import DistributedDataParallel
    from ml_trainer_amd.parallel.zero import ZeroDataParallel
    g = torch.Generator().manual_seed(7)
    x = torch.randn(world * 6, 8, generator=g)
    y = torch.randn(world * 6, 4, generator=g)
    xs, ys = x[rank * 6:(rank + 1) * 6], y[rank * 6:(rank + 1) * 6]
    out = {}
    for kind in ("ddp", "zero"):
        torch.manual_seed(1234 + rank)  # different per rank: the initial broadcast must fix it
        m = _model()
        if kind == "zero":
            w = ZeroDataParallel(m, bucket_cap_mb=0.002, first_bucket_mb=0.001)
            assert len(w.shard.chunks) >= 2 and w.shard.numel * world == w.flat.numel
            opt = w.make_optimizer(FusedAdamW, lr=1e-2, weight_decay=0.01)
            out["state_bytes"] = w.optimizer_state_bytes(opt)
        else:
            w = DistributedDataParallel(m, bucket_cap_mb=0.002, first_bucket_mb=0.001)
            opt = FusedAdamW(m.parameters(), lr=1e-2, weight_decay=0.01, flat=w.flat)
            out["ddp_state_bytes"] = sum(b.numel() * b.element_size() for b in opt.state_buffers(0))
        for it in range(4):
            opt.zero_grad()
            if it == 1:  # gradient accumulation: local micro-batch without communication
                with w.no_sync():
                    ((w(xs) - ys) ** 2).mean().backward()
            ((w(xs) - ys) ** 2).mean().backward()
            opt.step()
        sd = w.state_dict()
        out[kind] = {k: v.clone() for k, v in sd.items()}
        if kind == "zero":
            osd = opt.state_dict()  # collective gather of the sharded state
            out["zero_s1"] = osd["flat_state"][0]["s1"]
            # round trip: reload the gathered state, the shard must be unchanged
            before = opt.state_buffers(0)[0].clone()
            opt.load_state_dict(osd)
            assert torch.equal(before, opt.state_buffers(0)[0])
            out["zero_full_numel"] = w.flat.numel
    torch.save(out, os.path.join(out_dir, f"z{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_zero1_matches_ddp(world):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_zero_worker, args=(world, free_port(), d), nprocs=world, join=True)
        r = [torch.load(os.path.join(d, f"z{i}.pt"), weights_only=True) for i in range(world)]
        for k in r[0]["ddp"]:
            assert k.startswith("module.")
            for q in range(1, world):  # replicas identical after all-gather
                assert torch.equal(r[0]["zero"][k], r[q]["zero"][k])
            torch.testing.assert_close(r[0]["zero"][k], r[0]["ddp"][k], rtol=1e-5, atol=1e-6)
        # optimizer state is sharded: each rank holds 1/world of the (padded) replicated state
        assert r[0]["state_bytes"] * world == 2 * 4 * r[0]["zero_full_numel"]
        assert r[0]["state_bytes"] < r[0]["ddp_state_bytes"]
        assert all(torch.equal(r[0]["zero_s1"], r[q]["zero_s1"]) for q in range(1, world))


def _trainer_worker(rank, world, port, out_dir, zero):
    dist_env(rank, world, port)
    from ml_trainer_amd.models.lenet import MLModel
    from ml_trainer_amd.trainer import Trainer
    torch.manual_seed(0)
    tr, va = TensorCifar(64, 0), TensorCifar(32, 1)
    sub = os.path.join(out_dir, f"zero{zero}")
    os.makedirs(sub, exist_ok=True)
    t = Trainer(MLModel("tiny"), datasets=(tr, va), epochs=2, batch_size=32, is_parallel=True, backend="gloo",
                model_dir=sub, optimizer="adamw", lr=0.01,
                options={"progress": False, "zero_stage": zero, "grad_clip": 1.0})
    t.fit()
    torch.save({"params": t.flat.data.clone(), "losses": t.train_losses},
               os.path.join(sub, f"t{rank}.pt"))
    dist.destroy_process_group()


def test_trainer_zero1_tracks_ddp():
    world = 2
    with tempfile.TemporaryDirectory() as d:
        for zero in (0, 1):
            mp.spawn(_trainer_worker, args=(world, free_port(), d, zero), nprocs=world, join=True)
        r0 = torch.load(os.path.join(d, "zero0", "t0.pt"), weights_only=True)
        z = [torch.load(os.path.join(d, "zero1", f"t{i}.pt"), weights_only=True) for i in range(world)]
        assert torch.equal(z[0]["params"], z[1]["params"])
        torch.testing.assert_close(z[0]["losses"], r0["losses"], rtol=1e-4, atol=1e-5)
        sd0 = torch.load(os.path.join(d, "zero0", "model.pth"), weights_only=True)
        sd1 = torch.load(os.path.join(d, "zero1", "model.pth"), weights_only=True)
        assert sd0.keys() == sd1.keys()
        for k in sd0:
            torch.testing.assert_close(sd1[k], sd0[k], rtol=1e-4, atol=1e-5)
        assert os.path.exists(os.path.join(d, "zero1", "trainer_state.pt"))


def _zero_default_caps_worker(rank, world, port, out_dir):
    """ZeroDataParallel(module) with NO bucket caps (as bench.py builds it) next to plain DDP with no
    caps: DDP re-plans its buckets after the second backward (a cheap-wire model that changes the
    layout), ZeRO must not -- its shard chunks and sharded optimizer state follow its construction-time
    buckets."""
    dist_env(rank, world, port)
    os.environ["MLT_DDP_MIN_BUCKET_MB"] = "0.0001"
    os.environ["MLT_DDP_ALPHA_US"] = "0.05"
    os.environ["MLT_DDP_BUS_GBPS"] = "1000"
    dist.init_process_group("gloo")
    from ml_trainer_amd.ops.optim import FusedAdamW
    from ml_trainer_amd.parallel.ddp import DistributedDataParallel
    from ml_trainer_amd.parallel.zero import ZeroDataParallel
    out = {}
    for kind in ("ddp", "zero"):
        torch.manual_seed(5)
        m = torch.nn.Sequential(*[torch.nn.Linear(64, 64) for _ in range(6)])
        if kind == "zero":
            w = ZeroDataParallel(m)
            opt = w.make_optimizer(FusedAdamW, lr=1e-2, weight_decay=0.01)
            chunks0 = list(w.shard.chunks)
        else:
            w = DistributedDataParallel(m)
            opt = FusedAdamW(m.parameters(), lr=1e-2, weight_decay=0.01, flat=w.flat)
        layouts = []
        g = torch.Generator().manual_seed(11 + rank)
        for _ in range(5):
            opt.zero_grad()
            w(torch.randn(16, 64, generator=g)).pow(2).mean().backward()
            opt.step()
            layouts.append(list(w._buckets))
        if kind == "zero":
            w.wait_parameters()
            out["zero_chunks_same"] = list(w.shard.chunks) == chunks0
        out[kind] = w.flat.data.clone() if kind == "zero" else None
        out[kind + "_layouts"] = layouts
        out[kind + "_plan"] = dict(w.bucket_plan)
        if kind == "ddp":
            out["ddp_params"] = {n: p.detach().clone() for n, p in m.named_parameters()}
        else:
            out["zero_params"] = {n: p.detach().clone() for n, p in m.named_parameters()}
    torch.save(out, os.path.join(out_dir, f"d{rank}.pt"))
    dist.destroy_process_group()


def test_zero1_default_caps_never_replans():
    """ZeroDataParallel without caps inherited DDP's one-time bucket re-plan, which
    rebuilt the buckets under a fixed shard layout. It must keep its buckets, and train like DDP."""
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_zero_default_caps_worker, args=(world, free_port(), d), nprocs=world, join=True)
        r = [torch.load(os.path.join(d, f"d{i}.pt"), weights_only=True) for i in range(world)]
    for q in range(world):
        lay = r[q]["ddp_layouts"]
        assert r[q]["ddp_plan"]["replans"] == 1 and lay[1] != lay[0]  # DDP did re-plan (the test bites)
        zl = r[q]["zero_layouts"]
        assert all(x == zl[0] for x in zl) and r[q]["zero_chunks_same"]
        assert r[q]["zero_plan"]["replans"] == 0
        for n, p in r[q]["ddp_params"].items():
            torch.testing.assert_close(r[q]["zero_params"][n], p, rtol=1e-5, atol=1e-6)
    assert torch.equal(r[0]["zero"], r[1]["zero"])
