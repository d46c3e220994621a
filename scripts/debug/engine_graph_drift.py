"""Engine training with hipGraph replay vs eager launches (same init / data / order): the
weights must agree bitwise; also each vs a torch autograd replay of the augmented batches."""
import os, sys; sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import copy
import torch
import torch.nn.functional as F
from ml_trainer_amd.models.lenet import MLModel
from ml_trainer_amd.models.lenet_engine import LeNetStepEngine
from ml_trainer_amd.ops.optim import build_optimizer
from ml_trainer_amd.utils.flat import FlatParams

dev = torch.device("cuda", 0)
B, STEPS = 64, 8
N = 640
g = torch.Generator().manual_seed(1)
if os.environ.get("DRIFT_LEARNABLE") == "1":  # the Trainer test's class-coloured synthetic set
    from ml_trainer_amd.data.cifar10 import SyntheticCIFAR10
    ds = SyntheticCIFAR10(N, train=True, seed=0, learnable=True)
    data, targets = torch.from_numpy(ds.data), torch.tensor(ds.targets)
else:
    data = torch.randint(0, 256, (N, 32, 32, 3), dtype=torch.uint8, generator=g)
    targets = torch.randint(0, 10, (N,), generator=g)
perm = torch.randperm(N, generator=g)
torch.manual_seed(3)
base = MLModel().to(dev)
out = {}
for tag, graph in (("eager", False), ("graph", True)):
    m = copy.deepcopy(base)
    flat = FlatParams(m.parameters())
    opt = build_optimizer("sgd", m.parameters(), lr=0.01, momentum=0.9, flat=flat)
    eng = LeNetStepEngine(m, flat, max_batch=B, optimizer=opt)
    eng.set_dataset(data, targets, batch_size=B)
    eng.start_epoch(perm)
    if graph:
        eng.train_steps(B, STEPS, use_graph=True, steps_per_graph=4)
    else:
        for _ in range(STEPS):
            eng.train_steps(B, 1, use_graph=False)
    torch.cuda.synchronize()
    out[tag] = flat.data.clone()
    print(tag, "ctrl", eng.ctrl.tolist())
d = (out["eager"] - out["graph"]).abs().max().item()
print(f"eager vs graph max|dW| {d:.3e}")

# eager engine steps vs a torch autograd + torch.optim.SGD replay of the same augmented batches
m = copy.deepcopy(base)
ref = copy.deepcopy(base)
flat = FlatParams(m.parameters())
opt = build_optimizer("sgd", m.parameters(), lr=0.01, momentum=0.9, flat=flat)
ro = torch.optim.SGD(ref.parameters(), lr=0.01, momentum=0.9)
eng = LeNetStepEngine(m, flat, max_batch=B, optimizer=opt)
eng.set_dataset(data, targets, batch_size=B)
eng.start_epoch(perm)
for s in range(STEPS):
    eng.train_steps(B, 1, use_graph=False)
    torch.cuda.synchronize()
    x = eng.bufs["x"][:B * 3072].view(B, 3, 32, 32).clone()
    y = eng.bufs["targets"][:B].clone()
    ro.zero_grad()
    F.cross_entropy(ref.forward_reference(x), y).backward()
    ro.step()
    d = max((p.detach() - q.detach()).abs().max().item() for p, q in zip(m.parameters(), ref.parameters()))
    print(f"step {s}: engine vs torch max|dW| {d:.3e}")
