"""Tiny driver for rocprofv3 --pmc passes over the GEMM layouts: one forward-layout GEMM (A, B
k-contiguous) and one weight-gradient-layout GEMM (both mn-contiguous) of the same FLOP count,
a few launches each, planner configs. Usage:
    rocprofv3 --pmc SQ_WAVE_CYCLES ... -d gpurun_out/pmc -o run --output-format csv -- \
        python3 benchmarks/gemm_pmc_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_trainer_amd.ops._ext import require_native  # noqa: E402

C = require_native()
dev = torch.device("cuda", 0)
T = 65536
M, N = 2304, 768
A_f = torch.randn(T, N, device=dev).to(torch.bfloat16)      # fwd-layout: [T, 768] x [2304, 768]^T
W = torch.randn(M, N, device=dev).to(torch.bfloat16)
Y = torch.empty(T, M, dtype=torch.bfloat16, device=dev)
dY = torch.randn(T, M, device=dev).to(torch.bfloat16)       # wgrad-layout: dY^T [2304, T] x X [T, 768]
G = torch.zeros(M, N, dtype=torch.float32, device=dev)
for _ in range(int(os.environ.get("PROBE_ITERS", 3))):
    C.gemm(A_f, W, Y, False, False)
    C.gemm(dY, A_f, G, True, True, accumulate=True)
torch.cuda.synchronize()
print("probe done", flush=True)
