"""Property-based tests (hypothesis) of the CPU-side contracts: the data sharder reproduces
torch's DistributedSampler partition for any (n, world, rank, seed, epoch, drop_last), and the
regression criteria / mcrmse keep torch semantics on CPU tensors."""
import torch
import torch.nn.functional as F
from hypothesis import given, settings
from hypothesis import strategies as st
from torch.utils.data.distributed import DistributedSampler

from ml_trainer_amd.ops.losses import L1Loss, MSELoss, NLLLoss, mcrmse
from ml_trainer_amd.parallel.sampler import shard_indices


class _DS(torch.utils.data.Dataset):
    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        return i


@settings(max_examples=60, deadline=None)
@given(n=st.integers(1, 300), world=st.integers(1, 8), data=st.data(), seed=st.integers(0, 1000),
       epoch=st.integers(0, 5), shuffle=st.booleans(), drop_last=st.booleans())
def test_shard_matches_distributed_sampler(n, world, data, seed, epoch, shuffle, drop_last):
    rank = data.draw(st.integers(0, world - 1))
    s = DistributedSampler(_DS(n), num_replicas=world, rank=rank, shuffle=shuffle, seed=seed, drop_last=drop_last)
    s.set_epoch(epoch)
    assert shard_indices(n, world, rank, shuffle=shuffle, seed=seed, epoch=epoch, drop_last=drop_last) == list(s)


@settings(max_examples=40, deadline=None)
@given(B=st.integers(1, 64), C=st.integers(1, 12), seed=st.integers(0, 10_000))
def test_cpu_criteria_match_torch(B, C, seed):
    g = torch.Generator().manual_seed(seed)
    p, t = torch.randn(B, C, generator=g), torch.randn(B, C, generator=g)
    torch.testing.assert_close(L1Loss()(p, t), F.l1_loss(p, t))
    torch.testing.assert_close(MSELoss()(p, t), F.mse_loss(p, t))
    lp, y = F.log_softmax(p, -1), torch.randint(0, C, (B,), generator=g)
    torch.testing.assert_close(NLLLoss()(lp, y), F.nll_loss(lp, y))
    torch.testing.assert_close(mcrmse(p, t), torch.mean(torch.sqrt(torch.mean(torch.square(t - p), dim=0))))
