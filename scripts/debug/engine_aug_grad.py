"""One fused engine step on the device-augmented dataset path vs torch autograd on the
augmented batch the engine wrote (bufs['x'], bufs['targets']): gradient and loss agreement."""
import os, sys; sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import copy
import torch
import torch.nn.functional as F
from ml_trainer_amd.models.lenet import MLModel
from ml_trainer_amd.models.lenet_engine import LeNetStepEngine
from ml_trainer_amd.ops.optim import build_optimizer
from ml_trainer_amd.utils.flat import FlatParams

dev = torch.device("cuda", 0)
torch.manual_seed(3)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
m = MLModel().to(dev)
ref = copy.deepcopy(m)
flat = FlatParams(m.parameters())
opt = build_optimizer("sgd", m.parameters(), lr=0.0, momentum=0.0, flat=flat)
eng = LeNetStepEngine(m, flat, max_batch=B, optimizer=opt)
N = 640
data = torch.randint(0, 256, (N, 32, 32, 3), dtype=torch.uint8)
targets = torch.randint(0, 10, (N,))
eng.set_dataset(data, targets, batch_size=B)
eng.start_epoch(torch.randperm(N))
for step in range(3):
    eng.reset_stats()
    eng.train_steps(B, 1, use_graph=False)
    torch.cuda.synchronize()
    x = eng.bufs["x"][:B * 3072].view(B, 3, 32, 32).clone()
    y = eng.bufs["targets"][:B].clone()
    ref.zero_grad()
    loss = F.cross_entropy(ref.forward_reference(x), y)
    loss.backward()
    print(f"step {step}: loss engine {eng.read_stats(1)[0]:.8f} torch {loss.item():.8f}")
    for (n, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
        o, k = flat.segment(p)
        g = flat.grad[o:o + k].view_as(q)
        print(f"   {n:12s} max|g-gref| {(g - q.grad).abs().max().item():.3e}  |gref| {q.grad.abs().max().item():.3e}")
    for nm in ("p1", "p2", "h1", "h2", "logits", "dlogits", "dh2", "dh1", "dflat", "g1"):
        pass
