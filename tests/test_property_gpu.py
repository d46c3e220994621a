"""Property-based numerics (hypothesis) of the native gfx950 kernels vs plain torch fp32 over
randomly drawn shapes: LeNet forward/backward at any batch size, fused
softmax-CE and the regression criteria."""
import copy

import pytest
import torch
import torch.nn.functional as F
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

pytestmark = pytest.mark.gpu
_S = settings(max_examples=12, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])


def _exact_lenet(config, seed):
    from ml_trainer_amd.models.lenet import MLModel
    torch.manual_seed(seed)
    m = MLModel(config)
    g = torch.Generator().manual_seed(seed + 100)
    with torch.no_grad():  # dyadic weights + inputs: every sum exact, arg-max decisions identical
        for name, p in m.named_parameters():
            p.copy_(torch.randint(-2, 3, p.shape, generator=g).float() / (16.0 if name.startswith("conv") else 64.0))
    return m


@_S
@given(B=st.integers(1, 70), config=st.sampled_from(["default", "tiny"]), seed=st.integers(0, 1000))
def test_lenet_fwd_bwd_any_batch(dev, B, config, seed):
    m = _exact_lenet(config, seed).to(dev)
    ref = copy.deepcopy(m)
    g = torch.Generator().manual_seed(seed)
    x = (torch.randint(-2, 3, (B, 3, 32, 32), generator=g).float() / 4).to(dev)
    y = torch.randint(0, 10, (B,), generator=g).to(dev)
    out, ref_out = m(x), ref.forward_reference(x)
    torch.testing.assert_close(out, ref_out, rtol=1e-5, atol=1e-5)
    F.cross_entropy(out, y).backward()
    F.cross_entropy(ref_out, y).backward()
    for (n, p), q in zip(m.named_parameters(), ref.parameters()):
        torch.testing.assert_close(p.grad, q.grad, rtol=2e-3, atol=2e-5, msg=lambda s: f"{n}: {s}")


@_S
@given(B=st.integers(1, 300), C=st.integers(2, 200), ls=st.sampled_from([0.0, 0.1]), seed=st.integers(0, 1000))
def test_ce_any_shape(dev, B, C, ls, seed):
    from ml_trainer_amd.ops.losses import CrossEntropyLoss
    g = torch.Generator().manual_seed(seed)
    z = (torch.randn(B, C, generator=g) * 3).to(dev).requires_grad_(True)
    y = torch.randint(0, C, (B,), generator=g).to(dev)
    z2 = z.detach().clone().requires_grad_(True)
    loss, ref = CrossEntropyLoss(label_smoothing=ls)(z, y), F.cross_entropy(z2, y, label_smoothing=ls)
    torch.testing.assert_close(loss, ref, rtol=1e-5, atol=1e-5)
    loss.backward()
    ref.backward()
    torch.testing.assert_close(z.grad, z2.grad, rtol=1e-5, atol=1e-7)


@_S
@given(n=st.integers(1, 200_000), kind=st.sampled_from(["l1", "mse"]), seed=st.integers(0, 1000))
def test_pointwise_any_size(dev, n, kind, seed):
    from ml_trainer_amd.ops.losses import L1Loss, MSELoss
    g = torch.Generator().manual_seed(seed)
    p = torch.randn(n, generator=g).to(dev).requires_grad_(True)
    t = torch.randn(n, generator=g).to(dev)
    p2 = p.detach().clone().requires_grad_(True)
    crit, fn = (L1Loss(), F.l1_loss) if kind == "l1" else (MSELoss(), F.mse_loss)
    loss, ref = crit(p, t), fn(p2, t)
    torch.testing.assert_close(loss, ref, rtol=1e-5, atol=1e-6)
    loss.backward()
    ref.backward()
    torch.testing.assert_close(p.grad, p2.grad, rtol=1e-6, atol=1e-9)
