"""Config 7 (4-wave asm main loop, gemm_w4.hip) vs config 5 (8-wave ping-pong) vs torch.matmul
(hipBLASLt) on the forward-layout BERT shapes at 64K tokens and two squares; interleaved rounds,
random operands, one JSON line per shape."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_trainer_amd.ops._ext import require_native  # noqa: E402

C = require_native()
dev = torch.device("cuda", 0)
T = int(os.environ.get("GEMM_BENCH_TOKENS", 65536))
shapes = [("qkv_fwd", T, 2304, 768, 0), ("out_fwd", T, 768, 768, 0), ("ffn1_fwd", T, 3072, 768, 0),
          ("ffn2_fwd", T, 768, 3072, 0), ("qkv_dgrad", T, 768, 2304, 1), ("out_dgrad", T, 768, 768, 1),
          ("ffn1_dgrad", T, 768, 3072, 1), ("ffn2_dgrad", T, 3072, 768, 1),
          ("sq4096", 4096, 4096, 4096, 0), ("sq8192", 8192, 8192, 8192, 0)]


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


for name, M, N, K, bmn in shapes:
    A = (torch.rand(M, K, device=dev) - 0.5).to(torch.bfloat16)
    B = (torch.rand((K, N) if bmn else (N, K), device=dev) - 0.5).to(torch.bfloat16)
    Bt = B if bmn else B.t()
    out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    fns = {"cfg5": lambda: C.gemm(A, B, out, False, bool(bmn), cfg=5),
           "cfg7": lambda: C.gemm(A, B, out, False, bool(bmn), cfg=7),
           "torch": lambda: torch.matmul(A, Bt, out=out)}
    best = {k: 1e9 for k in fns}
    for _ in range(3):
        for k, f in fns.items():
            best[k] = min(best[k], timeit(f))
    fl = 2.0 * M * N * K
    r = {"shape": name, "M": M, "N": N, "K": K, "b_mn": bmn}
    for k, v in best.items():
        r[k + "_ms"] = round(v, 4)
        r[k + "_tflops"] = round(fl / v / 1e9, 1)
    r["cfg7_vs_torch"] = round(best["torch"] / best["cfg7"], 3)
    print(json.dumps(r), flush=True)
