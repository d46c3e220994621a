"""fp8 FFN intermediate: quantising GEMM epilogue (C.gemm_f8_q) vs bf16 GEMM output + the
cast-transpose pass it replaces, on the large config's FFN shapes (H 1024, F 4096).
Interleaved rounds in one process, random operands. One JSON line per (direction, tokens)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_trainer_amd.ops._ext import require_native  # noqa: E402

C = require_native()
dev = torch.device("cuda", 0)
H, F = 1024, 4096


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


one = torch.ones(1, device=dev)
amax = torch.zeros(C.FP8_AMAX_SLOTS, device=dev)
for T in [int(t) for t in os.environ.get("FFN_BENCH_TOKENS", "32768,131072").split(",")]:
    x8 = torch.randn(T, H, device=dev).to(torch.float8_e4m3fn)
    w1 = torch.randn(F, H, device=dev).mul_(0.05).to(torch.float8_e4m3fn)
    w2t = torch.randn(F, H, device=dev).mul_(0.05).to(torch.float8_e4m3fn)  # W2^T [F, H]
    dy8 = torch.randn(T, H, device=dev).to(torch.float8_e5m2)
    b1 = torch.randn(F, device=dev)
    pre = torch.empty(T, F, dtype=torch.bfloat16, device=dev)
    a16 = torch.empty(T, F, dtype=torch.bfloat16, device=dev)
    a8 = torch.empty(T, F, dtype=torch.float8_e4m3fn, device=dev)
    a8t = torch.empty(F, T, dtype=torch.float8_e4m3fn, device=dev)
    d8 = torch.empty(T, F, dtype=torch.float8_e5m2, device=dev)
    d8t = torch.empty(F, T, dtype=torch.float8_e5m2, device=dev)
    db = torch.empty(F, device=dev)

    def fwd_unfused():
        C.gemm_f8(x8, w1, a16, 0, 0, one, one, bias=b1, aux=pre, mode=1)
        C.fp8_cast_transpose(a16, a8, a8t, one, amax, 0)

    def fwd_fused():
        C.gemm_f8_q(x8, w1, a8, a8t, 0, 0, one, one, 0, one, amax, bias=b1, aux=pre, mode=1)

    def bwd_unfused():
        C.gemm_f8(dy8, w2t, a16, 1, 0, one, one, aux=pre, mode=2)
        C.fp8_cast_transpose(a16, d8, d8t, one, amax, 1, colsum_out=db)

    def bwd_fused():
        C.gemm_f8_q(dy8, w2t, d8, d8t, 1, 0, one, one, 1, one, amax, aux=pre, mode=2, colsum_out=db)

    def gemm_only():
        C.gemm_f8(x8, w1, a16, 0, 0, one, one, bias=b1, aux=pre, mode=1)

    r = {k: [] for k in ("fwd_unfused", "fwd_fused", "bwd_unfused", "bwd_fused", "fwd_gemm_only")}
    for _ in range(3):
        r["fwd_unfused"].append(timeit(fwd_unfused))
        r["fwd_fused"].append(timeit(fwd_fused))
        r["bwd_unfused"].append(timeit(bwd_unfused))
        r["bwd_fused"].append(timeit(bwd_fused))
        r["fwd_gemm_only"].append(timeit(gemm_only))
    out = {"tokens": T, "H": H, "F": F}
    out.update({k + "_ms": round(min(v), 4) for k, v in r.items()})
    out["fwd_fused_tflops"] = round(2.0 * T * H * F / (out["fwd_fused_ms"] * 1e9), 1)
    print(json.dumps(out), flush=True)
