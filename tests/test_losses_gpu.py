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
