"""Weight-gradient GEMMs (dW += dY^T X, both operands mn-contiguous, fp32 accumulate) at BERT-base
64K tokens: the planner's tile + split-K choice vs the ping-pong kernel (cfg 5) at several split
counts. Interleaved rounds in one process; one JSON line per shape."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_trainer_amd.ops._ext import require_native  # noqa: E402

C = require_native()
dev = torch.device("cuda", 0)
T = int(os.environ.get("GEMM_BENCH_TOKENS", 65536))
shapes = [("qkv_wgrad", 2304, 768), ("out_wgrad", 768, 768), ("ffn1_wgrad", 3072, 768), ("ffn2_wgrad", 768, 3072)]


def timeit(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


for name, M, N in shapes:
    A = torch.randn(T, M, device=dev).to(torch.bfloat16)  # dY [tokens, M]: A^T is mn-contiguous
    B = torch.randn(T, N, device=dev).to(torch.bfloat16)  # X  [tokens, N]
    out = torch.zeros(M, N, dtype=torch.float32, device=dev)
    plan = list(C.gemm_plan(True, True, M, N, T))
    variants = {"planner": {}}
    for s in (4, 6, 8, 9, 12, 16):
        variants[f"pp_s{s}"] = {"cfg": 5, "splits": s}
        variants[f"t256_s{s}"] = {"cfg": 1, "splits": s}
    best = {k: 1e9 for k in variants}
    for _ in range(3):
        for k, kw in variants.items():
            best[k] = min(best[k], timeit(lambda: C.gemm(A, B, out, True, True, accumulate=True, **kw)))
    ref = (A.float().t() @ B.float())
    out.zero_()
    C.gemm(A, B, out, True, True, accumulate=True, cfg=5, splits=9)
    err = ((out - ref).abs().max() / ref.abs().max()).item()
    fl = 2.0 * M * N * T
    r = {"shape": name, "M": M, "N": N, "K": T, "plan": plan, "pp_s9_rel_err": err}
    r.update({k + "_tflops": round(fl / v / 1e9, 1) for k, v in best.items()})
    print(json.dumps(r), flush=True)
