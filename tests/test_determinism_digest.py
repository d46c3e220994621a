"""Cross-rank determinism check: a bitwise digest of the parameter words, not a sum."""
import os
import tempfile

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.helpers import TensorCifar, dist_env, free_port
from ml_trainer_amd.utils.flat import bitwise_digest


def test_digest_sees_bit_flips_and_swaps_a_sum_misses():
    g = torch.Generator().manual_seed(0)
    x = torch.randn(62006, generator=g)
    d0 = bitwise_digest(x)
    assert d0 == bitwise_digest(x.clone())  # deterministic
    y = x.clone()
    y[[10, 20000]] = y[[20000, 10]]  # a permutation: the float64 sum is the same
    assert float(y.double().sum()) == float(x.double().sum())
    assert bitwise_digest(y)[0] != d0[0] and bitwise_digest(y)[1] != d0[1]
    for i in (0, 777, 62005):
        z = x.clone()
        z.view(torch.int32)[i] ^= 1  # last mantissa bit
        assert bitwise_digest(z) != d0
    # -0.0 vs +0.0: equal as floats, different words
    a, b = torch.zeros(8), torch.zeros(8)
    b[3] = -0.0
    assert torch.equal(a, b) and bitwise_digest(a) != bitwise_digest(b)
    # chunking does not change the value
    assert bitwise_digest(x, chunk=1000) == d0


def _worker(rank, world, port, out_dir):
    dist_env(rank, world, port)
    from ml_trainer_amd.models.lenet import MLModel
    from ml_trainer_amd.trainer import Trainer
    torch.manual_seed(0)
    tr, va = TensorCifar(64, 0), TensorCifar(32, 1)
    t = Trainer(MLModel("tiny"), datasets=(tr, va), epochs=1, batch_size=32, is_parallel=True, backend="gloo",
                model_dir=out_dir, options={"progress": False, "determinism_check": True})
    res = {}
    t._determinism_check()  # replicas identical after the initial broadcast
    res["clean"] = True
    with torch.no_grad():
        saved = t.flat.data.clone()
        if rank == 1:  # swap two different values on one rank: the sum is unchanged
            i, j = 3, 500
            assert t.flat.data[i] != t.flat.data[j]
            t.flat.data[[i, j]] = t.flat.data[[j, i]]
        try:
            t._determinism_check()
            res["swap"] = False
        except RuntimeError:
            res["swap"] = True
        t.flat.data.copy_(saved)
        if rank == 1:  # one parameter's last bit
            t.flat.data.view(torch.int32)[7] ^= 1
        try:
            t._determinism_check()
            res["flip"] = False
        except RuntimeError:
            res["flip"] = True
    torch.save(res, os.path.join(out_dir, f"d{rank}.pt"))
    dist.destroy_process_group()


def test_determinism_check_raises_on_one_flipped_bit_world2():
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, free_port(), d), nprocs=world, join=True)
        r = [torch.load(os.path.join(d, f"d{k}.pt"), weights_only=True) for k in range(world)]
    for x in r:  # every rank raises (the check is collective)
        assert x == {"clean": True, "swap": True, "flip": True}
