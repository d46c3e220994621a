"""Debug: bf16 vs fp32 LeNet engine over several epochs at two learning rates (loss per epoch,
non-finite checks), and the bf16 engine vs the bf16 torch reference over 12 SGD steps."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from ml_trainer_amd.models.lenet import MLModel  # noqa: E402
from ml_trainer_amd.models.lenet_bf16_ref import lenet_bf16_grads  # noqa: E402
from ml_trainer_amd.models.lenet_engine import LeNetStepEngine  # noqa: E402
from ml_trainer_amd.ops.optim import build_optimizer  # noqa: E402
from ml_trainer_amd.utils.flat import FlatParams  # noqa: E402

dev = torch.device("cuda", 0)


def toy(N, seed=0):
    g = torch.Generator().manual_seed(seed)
    t = torch.randint(0, 10, (N,), generator=g)
    base = (t.view(N, 1, 1, 1).float() * 25).expand(N, 32, 32, 3)
    d = (base + torch.randint(0, 30, (N, 32, 32, 3), generator=g).float()).clamp(0, 255).to(torch.uint8)
    return d, t


def engine(prec, lr, B=64, seed=12):
    torch.manual_seed(seed)
    m = MLModel().to(dev)
    flat = FlatParams(m.parameters())
    o = build_optimizer("sgd", m.parameters(), lr=lr, momentum=0.9, flat=flat)
    return LeNetStepEngine(m, flat, max_batch=B, optimizer=o, precision=prec), flat, m


data, targets = toy(2048, 11)
for lr in (5e-2, 1e-2):
    for prec in ("fp32", "bf16"):
        eng, flat, m = engine(prec, lr)
        eng.set_dataset(data, targets, batch_size=64)
        losses = []
        for ep in range(4):
            eng.start_epoch(torch.randperm(2048, generator=torch.Generator().manual_seed(ep)))
            eng.reset_stats()
            eng.train_steps(64, 32, use_graph=True, steps_per_graph=16)
            losses.append(round(eng.read_stats(32)[0], 4))
        print(f"lr {lr} {prec}: losses {losses} finite params {bool(torch.isfinite(flat.data).all())} "
              f"max|p| {flat.data.abs().max().item():.3g}", flush=True)

# engine vs reference, 12 SGD steps on the same batches
eng, flat, m = engine("bf16", 2e-2, B=32)
p = {n: q.detach().clone() for n, q in m.named_parameters()}
buf = {n: None for n in p}
for i in range(12):
    x = torch.randn(32, 3, 32, 32, device=dev) + 0.5 * (torch.arange(32, device=dev) % 10).view(32, 1, 1, 1) / 10
    y = (torch.arange(32, device=dev) % 10)
    eng.step_from_tensors(x, y, train=True)
    _, _, g = lenet_bf16_grads(p, x, y)
    for n in p:
        gg = g[n].float().to(dev)
        buf[n] = gg if buf[n] is None else 0.9 * buf[n] + gg
        p[n] = p[n] - 2e-2 * buf[n]
    rel = max(((q.detach() - p[n]).norm() / p[n].norm()).item() for n, q in m.named_parameters())
    print(f"step {i}: max rel param diff engine vs reference {rel:.2e}", flush=True)
