"""bf16 GEMM throughput: native MFMA kernel vs torch.matmul (hipBLASLt) on BERT shapes.
Interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24), random operands."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_trainer_amd.ops._ext import require_native  # noqa: E402

C = require_native()
dev = torch.device("cuda", 0)
T = 32 * 512  # tokens of BERT-base at batch 32, seq 512
T = int(os.environ.get("GEMM_BENCH_TOKENS", T))
shapes = [  # (name, M, N, K, a_mn, b_mn)
    ("qkv_fwd", T, 2304, 768, 0, 0), ("out_fwd", T, 768, 768, 0, 0), ("ffn1_fwd", T, 3072, 768, 0, 0),
    ("ffn2_fwd", T, 768, 3072, 0, 0), ("qkv_dgrad", T, 768, 2304, 0, 1), ("ffn1_dgrad", T, 768, 3072, 0, 1),
    ("ffn2_dgrad", T, 3072, 768, 0, 1), ("qkv_wgrad", 2304, 768, T, 1, 1), ("out_wgrad", 768, 768, T, 1, 1),
    ("ffn1_wgrad", 3072, 768, T, 1, 1), ("ffn2_wgrad", 768, 3072, T, 1, 1),
    ("sq4096", 4096, 4096, 4096, 0, 0), ("sq8192", 8192, 8192, 8192, 0, 0),
]


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


res = []
for name, M, N, K, a_mn, b_mn in shapes:
    A = torch.randn((K, M) if a_mn else (M, K), device=dev).to(torch.bfloat16)
    B = torch.randn((K, N) if b_mn else (N, K), device=dev).to(torch.bfloat16)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    At = A.t() if a_mn else A
    Bt = B if b_mn else B.t()
    plan = C.gemm_plan(bool(a_mn), bool(b_mn), M, N, K)
    variants = {"native": {}, "legacy128": {"cfg": 0}, "t256x256": {"cfg": 1}, "t256x128": {"cfg": 2}, "t256x192": {"cfg": 4},
                "t128x256": {"cfg": 3}, "pp256": {"cfg": 5}}
    if not a_mn:
        variants["persist256"] = {"cfg": 6}
    best = {k: 1e9 for k in list(variants) + ["torch"]}
    for _ in range(3):
        for k, kw in variants.items():
            best[k] = min(best[k], timeit(lambda: C.gemm(A, B, out, bool(a_mn), bool(b_mn), **kw)))
        best["torch"] = min(best["torch"], timeit(lambda: torch.matmul(At, Bt, out=out)))
    fl = 2.0 * M * N * K
    r = {"shape": name, "M": M, "N": N, "K": K, "plan": list(plan), "native_ms": round(best["native"], 4),
         "torch_ms": round(best["torch"], 4), "native_tflops": round(fl / best["native"] / 1e9, 1),
         "torch_tflops": round(fl / best["torch"] / 1e9, 1)}
    r.update({k + "_tflops": round(fl / best[k] / 1e9, 1) for k in variants if k != "native"})
    if not a_mn and not b_mn and K % 128 == 0:  # fp8 e4m3 x e4m3 (MX-scaled MFMA) on the same shape
        A8 = A.to(torch.float8_e4m3fn)
        B8 = B.to(torch.float8_e4m3fn)
        one = torch.ones(1, device=dev)
        t8 = min(timeit(lambda: C.gemm_f8(A8, B8, out, 0, 0, one, one)) for _ in range(3))
        r["fp8_tflops"] = round(fl / t8 / 1e9, 1)
        t8p = min(timeit(lambda: C.gemm_f8(A8, B8, out, 0, 0, one, one, cfg=5)) for _ in range(3))
        r["fp8_pp256_tflops"] = round(fl / t8p / 1e9, 1)
        t8q = min(timeit(lambda: C.gemm_f8(A8, B8, out, 0, 0, one, one, cfg=6)) for _ in range(3))
        r["fp8_persist256_tflops"] = round(fl / t8q / 1e9, 1)
        r["fp8_plan"] = list(C.gemm_f8_plan(M, N, K))
    res.append(r)
    print(json.dumps(r), flush=True)
