"""Native softmax-CE / accuracy kernels vs the plain torch fp32 reference."""
import pytest
import torch
import torch.nn.functional as F

from ml_trainer_amd.ops.losses import CrossEntropyLoss, accuracy

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,C", [(1, 10), (33, 10), (256, 2), (64, 1000), (7, 130)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("ls", [0.0, 0.1])
def test_ce_forward_backward(dev, B, C, dtype, ls):
    z = (torch.randn(B, C, device=dev) * 3).to(dtype).requires_grad_(True)
    y = torch.randint(0, C, (B,), device=dev)
    if B > 3:
        y[1] = -100  # ignore_index row
    z2 = z.detach().float().requires_grad_(True)
    loss = CrossEntropyLoss(label_smoothing=ls)(z, y)
    ref = F.cross_entropy(z2, y, label_smoothing=ls)
    torch.testing.assert_close(loss.float(), ref, rtol=1e-5, atol=1e-5)
    (loss * 1.7).backward()
    (ref * 1.7).backward()
    tol = 1e-6 if dtype == torch.float32 else 1e-2
    torch.testing.assert_close(z.grad.float(), z2.grad, rtol=tol, atol=tol)


def test_accuracy(dev):
    z = torch.randn(1000, 10, device=dev)
    y = torch.randint(0, 10, (1000,), device=dev)
    ref = (z.argmax(-1) == y).float().mean()
    torch.testing.assert_close(accuracy(z, y), ref)


@pytest.mark.parametrize("shape", [(1,), (37, 3), (4096, 5), (300001,)])
@pytest.mark.parametrize("kind", ["l1", "mse"])
def test_pointwise_losses(dev, shape, kind):
    from ml_trainer_amd.ops.losses import L1Loss, MSELoss
    p = torch.randn(*shape, device=dev, requires_grad=True)
    t = torch.randn(*shape, device=dev)
    if kind == "l1":
        t.view(-1)[0] = p.detach().view(-1)[0]  # sign(0) = 0 gradient
    p2 = p.detach().clone().requires_grad_(True)
    crit, ref_fn = (L1Loss(), F.l1_loss) if kind == "l1" else (MSELoss(), F.mse_loss)
    loss, ref = crit(p, t), ref_fn(p2, t)
    torch.testing.assert_close(loss, ref, rtol=1e-5, atol=1e-6)
    (loss * 3.0).backward()
    (ref * 3.0).backward()
    torch.testing.assert_close(p.grad, p2.grad, rtol=1e-6, atol=1e-9)
    # fixed-order reductions: bitwise reproducible
    assert torch.equal(crit(p, t), loss)


@pytest.mark.parametrize("B,C", [(1, 10), (513, 7), (64, 1000)])
def test_nll_loss(dev, B, C):
    from ml_trainer_amd.ops.losses import NLLLoss
    z = torch.randn(B, C, device=dev)
    lp = F.log_softmax(z, -1).requires_grad_(True)
    y = torch.randint(0, C, (B,), device=dev)
    if B > 3:
        y[2] = -100
    lp2 = lp.detach().clone().requires_grad_(True)
    loss, ref = NLLLoss()(lp, y), F.nll_loss(lp2, y)
    torch.testing.assert_close(loss, ref, rtol=1e-5, atol=1e-6)
    (loss * 0.5).backward()
    (ref * 0.5).backward()
    torch.testing.assert_close(lp.grad, lp2.grad, rtol=1e-6, atol=1e-9)


@pytest.mark.parametrize("B,C", [(1, 3), (100, 6), (5000, 2)])
def test_mcrmse(dev, B, C):
    from ml_trainer_amd.ops.losses import mcrmse
    p, t = torch.randn(B, C, device=dev), torch.randn(B, C, device=dev)
    ref = torch.mean(torch.sqrt(torch.mean(torch.square(t - p), dim=0)), dim=0)
    torch.testing.assert_close(mcrmse(p, t), ref, rtol=1e-5, atol=1e-6)


def test_custom_loss_native(dev):
    from ml_trainer_amd.utils.functions import custom_loss_function
    p, t = torch.randn(32, 10, device=dev), torch.randn(32, 10, device=dev)
    torch.testing.assert_close(custom_loss_function(p, t), torch.mean((p - t) ** 2), rtol=1e-5, atol=1e-6)
