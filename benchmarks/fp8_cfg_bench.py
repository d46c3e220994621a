"""fp8 (MX-scaled MFMA) GEMM configs on the `large` model's shapes (24L/1024H/4096 FFN) at the
bench's 131,072 tokens: the planner's pick vs every runnable 256-wide config, interleaved in one
process; one JSON line per shape. Operands k-contiguous (forward / dgrad layouts after the casts)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_trainer_amd.ops._ext import require_native  # noqa: E402

C = require_native()
dev = torch.device("cuda", 0)
T = int(os.environ.get("GEMM_BENCH_TOKENS", 131072))
H, F = 1024, 4096
shapes = [("qkv_fwd", T, 3 * H, H), ("out_fwd", T, H, H), ("ffn1_fwd", T, F, H), ("ffn2_fwd", T, H, F),
          ("qkv_dgrad", T, H, 3 * H), ("ffn1_dgrad", T, H, F), ("ffn2_dgrad", T, F, H),
          ("qkv_wgrad", 3 * H, H, T), ("ffn1_wgrad", F, H, T)]


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
for name, M, N, K in shapes:
    A = torch.randn(M, K, device=dev).to(torch.float8_e4m3fn)
    B = torch.randn(N, K, device=dev).to(torch.float8_e4m3fn)
    wg = name.endswith("wgrad")
    out = torch.zeros(M, N, dtype=torch.float32 if wg else torch.bfloat16, device=dev)
    variants = {"planner": {}, "cfg1": {"cfg": 1}, "cfg5": {"cfg": 5}, "cfg6": {"cfg": 6}}
    best = {k: 1e9 for k in variants}
    for _ in range(3):
        for k, kw in variants.items():
            best[k] = min(best[k], timeit(lambda: C.gemm_f8(A, B, out, 0, 0, one, one, accumulate=wg, **kw)))
    fl = 2.0 * M * N * K
    r = {"shape": name, "M": M, "N": N, "K": K, "plan": list(C.gemm_f8_plan(M, N, K))}
    r.update({k + "_tflops": round(fl / v / 1e9, 1) for k, v in best.items()})
    print(json.dumps(r), flush=True)
