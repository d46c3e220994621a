"""Fixed vs per-K-step cost of the tile GEMMs: time M x N x K for a K sweep and fit
t(K) = a + b*K per config (a = prologue + epilogue per launch, b = main-loop cost), next to
torch.matmul (hipBLASLt). Random bf16 operands, interleaved rounds in one process."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_trainer_amd.ops._ext import require_native  # noqa: E402

C = require_native()
dev = torch.device("cuda", 0)
M = int(os.environ.get("SWEEP_M", 16384))
Ns = [int(v) for v in os.environ.get("SWEEP_N", "3072,768").split(",")]
Ks = [256, 512, 768, 1536, 3072]
cfgs = {"t256": 1, "t192": 4, "pp": 5}
if os.environ.get("SWEEP_CFGS"):
    cfgs = {f"c{c}": int(c) for c in os.environ["SWEEP_CFGS"].split(",")}


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


for N in Ns:
    rows = {}
    for K in Ks:
        A = torch.randn(M, K, device=dev).to(torch.bfloat16)
        B = torch.randn(N, K, device=dev).to(torch.bfloat16)
        out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        best = {}
        for _ in range(3):
            for k, c in cfgs.items():
                best[k] = min(best.get(k, 1e9), timeit(lambda: C.gemm(A, B, out, False, False, cfg=c)))
            best["torch"] = min(best.get("torch", 1e9), timeit(lambda: torch.matmul(A, B.t(), out=out)))
        rows[K] = best
        print(json.dumps({"M": M, "N": N, "K": K, **{k: round(v, 2) for k, v in best.items()},
                          **{k + "_tf": round(2.0 * M * N * K / v / 1e6, 1) for k, v in best.items()}}), flush=True)
    for k in list(cfgs) + ["torch"]:
        xs = torch.tensor([float(K) for K in Ks], dtype=torch.float64)
        ys = torch.tensor([rows[K][k] for K in Ks], dtype=torch.float64)
        b = ((xs - xs.mean()) * (ys - ys.mean())).sum() / ((xs - xs.mean()) ** 2).sum()
        a = ys.mean() - b * xs.mean()
        print(json.dumps({"fit": k, "N": N, "fixed_us": round(float(a), 2), "us_per_64k": round(float(b) * 64, 3),
                          "mainloop_tf": round(2.0 * M * N * 64 / (float(b) * 64) / 1e6, 1)}), flush=True)
