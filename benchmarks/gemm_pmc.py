"""Run the 256x256 GEMM variants (config 1 two-phase, config 5 ping-pong) a few times each on
one shape, for rocprofv3 --pmc / --kernel-trace A/B runs:

    rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY ... --output-format csv -d out -- \\
        python benchmarks/gemm_pmc.py --M 8192 --N 8192 --K 8192
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_trainer_amd.ops._ext import require_native  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--M", type=int, default=8192)
p.add_argument("--N", type=int, default=8192)
p.add_argument("--K", type=int, default=8192)
p.add_argument("--a_mn", type=int, default=0)
p.add_argument("--b_mn", type=int, default=0)
p.add_argument("--cfgs", default="1,5")
p.add_argument("--reps", type=int, default=5)
p.add_argument("--torch", type=int, default=0, help="also run torch.matmul (hipBLASLt) this many times")
a = p.parse_args()
C = require_native()
dev = torch.device("cuda", 0)
A = torch.rand((a.K, a.M) if a.a_mn else (a.M, a.K), device=dev).sub_(0.5).to(torch.bfloat16)
B = torch.rand((a.K, a.N) if a.b_mn else (a.N, a.K), device=dev).sub_(0.5).to(torch.bfloat16)
out = torch.empty(a.M, a.N, dtype=torch.bfloat16, device=dev)
for cfg in [int(c) for c in a.cfgs.split(",")]:
    for _ in range(a.reps):
        C.gemm(A, B, out, bool(a.a_mn), bool(a.b_mn), cfg=cfg)
At = A.t() if a.a_mn else A
Bt = B if a.b_mn else B.t()
for _ in range(a.torch):
    torch.matmul(At, Bt, out=out)
torch.cuda.synchronize()
print("done")
