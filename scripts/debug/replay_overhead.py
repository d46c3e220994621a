"""Wall vs device time of one hipGraph replay of k LeNet bf16 steps from an idle GPU (the driver
protocol's fixed cost): python scripts/debug/replay_overhead.py"""
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
for k in (1, 5, 20, 64):
    eng.train_steps(32, k, use_graph=True, steps_per_graph=k)  # capture + warm
    for idle_us in (0, 200):
        walls, devs = [], []
        for rep in range(15):
            eng.train_steps(32, k, use_graph=True, steps_per_graph=k)
            torch.cuda.synchronize()
            if idle_us:
                time.sleep(idle_us * 1e-6)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e0.record()
            eng.train_steps(32, k, use_graph=True, steps_per_graph=k)
            e1.record()
            torch.cuda.synchronize()
            walls.append((time.perf_counter() - t0) * 1e6)
            devs.append(e0.elapsed_time(e1) * 1e3)
        walls.sort()
        devs.sort()
        print(f"k={k:3d} idle={idle_us:4d}us: wall {walls[7]:8.1f} us  device {devs[7]:8.1f} us  "
              f"fixed {walls[7] - devs[7]:6.1f} us  per-step wall {walls[7] / k:6.2f} dev {devs[7] / k:6.2f}", flush=True)
