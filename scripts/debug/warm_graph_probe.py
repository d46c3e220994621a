"""Does a limited replay (device step limit, ab/pkg_steplimit build) warm a k-step hipGraph like a
full replay does? Fresh engine per variant; after a 5-step warmup graph, time one replay of the
20-step graph (wall, region-style) under: A cold, B limited(5) first, C full replay first.
PYTHONPATH=ab/pkg_steplimit python scripts/debug/warm_graph_probe.py"""
import sys
import time

import torch

from ml_trainer_amd.models.lenet import MLModel
from ml_trainer_amd.models.lenet_engine import LeNetStepEngine
from ml_trainer_amd.ops.optim import build_optimizer
from ml_trainer_amd.utils.flat import FlatParams

dev = torch.device("cuda", 0)
N = 50000
data = torch.randint(0, 256, (N, 32, 32, 3), dtype=torch.uint8, device=dev)
targets = torch.randint(0, 10, (N,), device=dev)
perm = torch.randperm(N, dtype=torch.int32)


def fresh():
    m = MLModel().to(dev)
    flat = FlatParams(m.parameters())
    opt = build_optimizer("sgd", m.parameters(), lr=1e-3, momentum=0.9, flat=flat)
    eng = LeNetStepEngine(m, flat, max_batch=32, optimizer=opt, precision="bf16")
    eng.set_dataset(data, targets, batch_size=32)
    eng.start_epoch(perm)
    eng.prepare(32, 5, use_graph=True, steps_per_graph=5)
    eng.prepare(32, 20, use_graph=True, steps_per_graph=20)
    return eng


def region(eng):
    torch.cuda.synchronize()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.train_steps(32, 20, use_graph=True, steps_per_graph=20, flush=False)
    torch.cuda.synchronize()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e6 / 20


res = {}
for rep in range(3):
    for v in ("A_cold", "B_limited5", "C_full", "D_limited5_then_5step", "E_spg5"):
        eng = fresh()
        eng.train_steps(32, 5, use_graph=True, steps_per_graph=5, flush=False)  # the warmup
        if v == "B_limited5":
            eng.replay_limited(32, 20, 5)
        elif v == "C_full":
            eng.train_steps(32, 20, use_graph=True, steps_per_graph=20, flush=False)
        elif v == "D_limited5_then_5step":
            eng.replay_limited(32, 20, 5)
            eng.train_steps(32, 5, use_graph=True, steps_per_graph=5, flush=False)
        if v == "E_spg5":
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.train_steps(32, 20, use_graph=True, steps_per_graph=5, flush=False)
            torch.cuda.synchronize()
            torch.cuda.synchronize()
            us = (time.perf_counter() - t0) * 1e6 / 20
        else:
            us = region(eng)
        res.setdefault(v, []).append(round(us, 2))
        del eng
        torch.cuda.synchronize()
for k, v in res.items():
    print(k, v, flush=True)
