"""cfg 7 (gemm_w4.hip) K / raster sweep at 64K tokens against torch.matmul (hipBLASLt): per-tile
overhead (intercept of time vs K) and the grouped-raster width (MLT_GEMM_GROUP_M is read once per
process, so run once per width). One JSON line per (N, K)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_trainer_amd.ops._ext import require_native  # noqa: E402

C = require_native()
dev = torch.device("cuda", 0)
M = int(os.environ.get("GEMM_BENCH_TOKENS", 65536))
gm = os.environ.get("MLT_GEMM_GROUP_M", "4")


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
    return s.elapsed_time(e) / iters


for N in (768, 2304, 3072):
    for K in (256, 768, 1536, 3072):
        A = (torch.rand(M, K, device=dev) - 0.5).to(torch.bfloat16)
        B = (torch.rand(N, K, device=dev) - 0.5).to(torch.bfloat16)
        out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        t7 = min(timeit(lambda: C.gemm(A, B, out, False, False, cfg=7)) for _ in range(2))
        tt = min(timeit(lambda: torch.matmul(A, B.t(), out=out)) for _ in range(2))
        fl = 2.0 * M * N * K
        print(json.dumps({"group_m": int(gm), "M": M, "N": N, "K": K, "cfg7_ms": round(t7, 4), "torch_ms": round(tt, 4),
                          "cfg7_tflops": round(fl / t7 / 1e9, 1), "torch_tflops": round(fl / tt / 1e9, 1)}), flush=True)
