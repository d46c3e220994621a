"""Weight-gradient GEMM exploration (BERT-base shapes at 16384 tokens, both operands
mn-contiguous): tile config x split count x split-combine mode, plus a full-grid (1,1) square
as the layout's throughput ceiling. One JSON line per shape."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_trainer_amd.ops._ext import require_native  # noqa: E402

C = require_native()
dev = torch.device("cuda", 0)
T = 16384


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


shapes = [("qkv_wgrad", 2304, 768, T), ("out_wgrad", 768, 768, T), ("ffn1_wgrad", 3072, 768, T),
          ("ffn2_wgrad", 768, 3072, T), ("sq4096_k16k", 4096, 4096, T)]
for name, M, N, K in shapes:
    A = torch.randn(K, M, device=dev).to(torch.bfloat16)
    B = torch.randn(K, N, device=dev).to(torch.bfloat16)
    out = torch.zeros(M, N, device=dev)
    fl = 2.0 * M * N * K
    r = {"shape": name, "M": M, "N": N, "K": K, "plan": list(C.gemm_plan(True, True, M, N, K))}
    r["auto_tflops"] = round(fl / timeit(lambda: C.gemm(A, B, out, True, True, accumulate=True)) / 1e9, 1)
    for cfg in (1, 2, 4, 5):
        for splits in (1, 2, 3, 4, 6, 8, 12):
            for mode in (0, 1):
                if splits == 1 and mode == 1:
                    continue
                C.set_gemm_split_mode(mode)
                t = timeit(lambda: C.gemm(A, B, out, True, True, accumulate=True, cfg=cfg, splits=splits))
                r[f"c{cfg}s{splits}m{mode}"] = round(fl / t / 1e9, 1)
    C.set_gemm_split_mode(-1)
    best = max((v, k) for k, v in r.items() if k.startswith("c"))
    r["best"] = best[1]
    r["best_tflops"] = best[0]
    print(json.dumps(r), flush=True)
