"""Flat fused optimizers (CPU math path) vs torch.optim, multi-step, all five kinds."""
import copy

import pytest
import torch

from ml_trainer_amd.ops.optim import FusedAdagrad, FusedAdam, FusedAdamax, FusedAdamW, FusedSGD, clip_grad_norm_flat
from ml_trainer_amd.utils.flat import FlatParams

CASES = [
    (lambda p: FusedSGD(p, lr=0.1, momentum=0.9, weight_decay=0.01), lambda p: torch.optim.SGD(p, lr=0.1, momentum=0.9, weight_decay=0.01)),
    (lambda p: FusedSGD(p, lr=0.1, momentum=0.9, nesterov=True), lambda p: torch.optim.SGD(p, lr=0.1, momentum=0.9, nesterov=True)),
    (lambda p: FusedSGD(p, lr=0.1), lambda p: torch.optim.SGD(p, lr=0.1)),
    (lambda p: FusedAdam(p, lr=0.01, weight_decay=0.01), lambda p: torch.optim.Adam(p, lr=0.01, weight_decay=0.01)),
    (lambda p: FusedAdamW(p, lr=0.01, weight_decay=0.05), lambda p: torch.optim.AdamW(p, lr=0.01, weight_decay=0.05)),
    (lambda p: FusedAdagrad(p, lr=0.05, lr_decay=0.01, weight_decay=0.01), lambda p: torch.optim.Adagrad(p, lr=0.05, lr_decay=0.01, weight_decay=0.01)),
    (lambda p: FusedAdamax(p, lr=0.01, weight_decay=0.01), lambda p: torch.optim.Adamax(p, lr=0.01, weight_decay=0.01)),
]


@pytest.mark.parametrize("mk", CASES, ids=["sgd_m_wd", "sgd_nesterov", "sgd_plain", "adam", "adamw", "adagrad", "adamax"])
def test_matches_torch(mk):
    torch.manual_seed(0)
    m1 = torch.nn.Sequential(torch.nn.Linear(7, 5), torch.nn.Linear(5, 3))
    m2 = copy.deepcopy(m1)
    o1, o2 = mk[0](m1.parameters()), mk[1](m2.parameters())
    for _ in range(5):
        x = torch.randn(4, 7)
        for m, o in ((m1, o1), (m2, o2)):
            o.zero_grad()
            m(x).square().sum().backward()
            o.step()
    for p, q in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(p, q, rtol=1e-5, atol=1e-6)


def test_params_are_flat_views_and_state_roundtrip():
    m = torch.nn.Linear(6, 3)
    o = FusedAdam(m.parameters(), lr=0.01)
    fp = o.flats[0]
    assert m.weight.data_ptr() == fp.data.data_ptr() + fp.offsets[0] * 4
    m(torch.randn(2, 6)).sum().backward()
    assert m.weight.grad.data_ptr() == fp.grad.data_ptr() + fp.offsets[0] * 4
    o.step()
    sd = o.state_dict()
    o2 = FusedAdam(torch.nn.Linear(6, 3).parameters(), lr=0.5)
    o2.load_state_dict(sd)
    assert o2._steps == [1] and o2.param_groups[0]["lr"] == 0.01
    torch.testing.assert_close(o2._s1[0], o._s1[0])


def test_zero_grad_set_to_none_rebinds():
    m = torch.nn.Linear(4, 2)
    o = FusedSGD(m.parameters(), lr=0.1)
    m.zero_grad(set_to_none=True)  # user code detaching the views
    m(torch.randn(3, 4)).sum().backward()
    g = m.weight.grad.clone()
    w0 = m.weight.detach().clone()
    o.step()
    torch.testing.assert_close(m.weight.detach(), w0 - 0.1 * g)


def test_works_with_lr_schedulers():
    m = torch.nn.Linear(4, 2)
    o = FusedSGD(m.parameters(), lr=1.0)
    s = torch.optim.lr_scheduler.StepLR(o, step_size=1, gamma=0.5)
    for _ in range(3):
        o.step()
        s.step()
    assert o.param_groups[0]["lr"] == pytest.approx(0.125)


def test_clip_grad_norm_flat_cpu():
    m = torch.nn.Linear(10, 10)
    fp = FlatParams(m.parameters())
    fp.grad.fill_(1.0)
    ref = torch.tensor([1.0]).expand(fp.numel).norm()
    total = clip_grad_norm_flat(fp, 1.0)
    assert total.item() == pytest.approx(ref.item(), rel=1e-6)
    assert fp.grad.norm().item() == pytest.approx(1.0, rel=1e-4)
