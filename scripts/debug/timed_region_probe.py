"""Where the fixed ~30 us of a driver-protocol LeNet timed region goes (bf16, B32, K=20 one graph):
host time to the first hipGraphLaunch, launch call time, synchronize wait; the Python path alone
(replay stubbed out). python scripts/debug/timed_region_probe.py"""
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
K = 20
eng.prepare(32, K, use_graph=True, steps_per_graph=K)
eng.train_steps(32, 2 * K, use_graph=True, steps_per_graph=K, flush=False)
torch.cuda.synchronize()


class Stub:
    def __init__(self, inner):
        self.inner = inner

    def replay(self, *a):
        pass

    def __getattr__(self, k):
        return getattr(self.inner, k)


eng.prepare(32, K, use_graph=True, steps_per_graph=5)
eng.train_steps(32, K, use_graph=True, steps_per_graph=5, flush=False)
for spg in (5, 20):
    rows = []
    for rep in range(12):
        torch.cuda.synchronize()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.train_steps(32, K, use_graph=True, steps_per_graph=spg, flush=False)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        rows.append(((t1 - t0) * 1e6, (t2 - t1) * 1e6, (t3 - t2) * 1e6, (t3 - t0) * 1e6))
    rows.sort(key=lambda r: r[3])
    med = rows[len(rows) // 2]
    print(f"K={K} spg={spg}: launch calls {med[0]:.1f} us, first sync {med[1]:.1f} us, second sync {med[2]:.1f} us, "
          f"region {med[3]:.1f} us = {med[3] / K:.2f} us/step")
real = eng.eng
eng.eng = Stub(real)
py = []
for rep in range(200):
    t0 = time.perf_counter()
    eng.train_steps(32, K, use_graph=True, steps_per_graph=K, flush=False)
    py.append((time.perf_counter() - t0) * 1e6)
eng.eng = real
idle = []
for rep in range(50):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    torch.cuda.synchronize()
    idle.append((time.perf_counter() - t0) * 1e6)
py.sort()
idle.sort()
print(f"python path with replay stubbed: median {py[len(py) // 2]:.2f} us; idle synchronize median {idle[len(idle) // 2]:.2f} us")
