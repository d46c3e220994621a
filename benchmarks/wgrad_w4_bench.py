"""Weight-gradient GEMMs (BERT-base shapes at GEMM_BENCH_TOKENS tokens, A [K][M], B [K][N], fp32
accumulate into the gradient) through the planner (cfg 7 split-K by default; MLT_GEMM_W4=0: the
8-wave split-K tiles) and torch.matmul (hipBLASLt, bf16 out). One JSON line per shape."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_trainer_amd.ops._ext import require_native  # noqa: E402

C = require_native()
dev = torch.device("cuda", 0)
T = int(os.environ.get("GEMM_BENCH_TOKENS", 262144))


def timeit(fn, iters=10):
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


for name, M, N in [("qkv_wgrad", 2304, 768), ("out_wgrad", 768, 768), ("ffn1_wgrad", 3072, 768), ("ffn2_wgrad", 768, 3072)]:
    A = (torch.rand(T, M, device=dev) - 0.5).to(torch.bfloat16)
    B = (torch.rand(T, N, device=dev) - 0.5).to(torch.bfloat16)
    out = torch.zeros(M, N, device=dev)
    fl = 2.0 * M * N * T
    t = min(timeit(lambda: C.gemm(A, B, out, True, True, accumulate=True)) for _ in range(2))
    ob = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    tt = min(timeit(lambda: torch.matmul(A.t(), B, out=ob)) for _ in range(2))
    print(json.dumps({"shape": name, "M": M, "N": N, "K": T, "w4_env": os.environ.get("MLT_GEMM_W4", "1"),
                      "plan": list(C.gemm_plan(True, True, M, N, T)), "ms": round(t, 4), "tflops": round(fl / t / 1e9, 1),
                      "torch_tflops": round(fl / tt / 1e9, 1)}), flush=True)
