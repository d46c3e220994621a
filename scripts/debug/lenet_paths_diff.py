"""Diff every intermediate buffer of the LeNet engine path vs the autograd path (same inputs)."""
import os, sys; sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import copy
import torch
import torch.nn.functional as F
from ml_trainer_amd.models.lenet import MLModel
from ml_trainer_amd.models.lenet_engine import LeNetStepEngine
from ml_trainer_amd.ops.optim import build_optimizer
from ml_trainer_amd.utils.flat import FlatParams

dev = torch.device("cuda", 0)
torch.manual_seed(2)
m = MLModel().to(dev)
ref = copy.deepcopy(m)
x = torch.randn(32, 3, 32, 32, device=dev)
y = torch.randint(0, 10, (32,), device=dev)
F.cross_entropy(ref(x), y).backward()  # autograd path over native kernels
ref_grads = {n: p.grad.clone() for n, p in ref.named_parameters()}
ref2 = copy.deepcopy(m)
F.cross_entropy(ref2.forward_reference(x), y).backward()
for mode_opt in ["none", "sgd"]:
    mm = copy.deepcopy(m)
    flat = FlatParams(mm.parameters())
    o = build_optimizer("sgd", mm.parameters(), lr=0.0, momentum=0.0, flat=flat)
    eng = LeNetStepEngine(mm, flat, max_batch=32, optimizer=o)
    eng.step_from_tensors(x, y, train=True)
    torch.cuda.synchronize()
    print("=== engine fused-opt(lr=0)")
    for (n, p), (_, q) in zip(mm.named_parameters(), ref2.named_parameters()):
        o_, k = flat.segment(p)
        g = flat.grad[o_:o_ + k].view_as(q)
        print(f"{n:12s} engine-vs-torch {(g - q.grad).abs().max().item():.3e}  autograd-native-vs-torch "
              f"{(ref_grads[n] - q.grad).abs().max().item():.3e}  |g| {q.grad.abs().max().item():.3e}")
    break
