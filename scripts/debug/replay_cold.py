"""First (cold) vs later replays of a freshly captured + uploaded hipGraph of k LeNet bf16 steps:
python scripts/debug/replay_cold.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from ml_trainer_amd.models.lenet import MLModel  # noqa: E402
from ml_trainer_amd.models.lenet_engine import LeNetStepEngine  # noqa: E402
from ml_trainer_amd.ops.optim import build_optimizer  # noqa: E402
from ml_trainer_amd.utils.flat import FlatParams  # noqa: E402

dev = torch.device("cuda", 0)
m = MLModel().to(dev)
flat = FlatParams(m.parameters())
opt = build_optimizer("sgd", m.parameters(), lr=1e-3, momentum=0.9, flat=flat)
eng = LeNetStepEngine(m, flat, max_batch=32, optimizer=opt, precision="bf16")
N = 50000
data = torch.randint(0, 256, (N, 32, 32, 3), dtype=torch.uint8, device=dev)
targets = torch.randint(0, 10, (N,), device=dev)
eng.set_dataset(data, targets, batch_size=32)
eng.start_epoch(torch.randperm(N, dtype=torch.int32))
eng.train_steps(32, 5, use_graph=True, steps_per_graph=5)
for k in (20, 7, 33):
    eng.prepare(32, k, use_graph=True, steps_per_graph=k)
    for rep in range(4):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        eng.train_steps(32, k, use_graph=True, steps_per_graph=k)
        e1.record()
        torch.cuda.synchronize()
        w = (time.perf_counter() - t0) * 1e6
        d = e0.elapsed_time(e1) * 1e3
        print(f"k={k} replay {rep}: wall {w:8.1f} us device {d:8.1f} us  per step {w / k:6.2f} / {d / k:6.2f}", flush=True)
