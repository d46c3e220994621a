"""Where the fp8 quantising FFN1 GEMM's time goes (large config shape: M tokens x 4096, K = 1024):
the plain GEMM on the 4-wave kernel (cfg 7) and on the ping-pong kernel (cfg 5), each with the
bf16 bias + GELU epilogue (pre-activation saved), and the quantising (q8) epilogues of gemm_f8_q
(fp8 Y + Y^T + amax): FFN1's GELU and FFN2-dgrad's dGELU (+ column sums). MLT_GEMM_W4Q8=0 puts the
q8 forms on the ping-pong kernel instead of the 4-wave one. One JSON line. FFN_TOKENS (default 262144)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_trainer_amd.ops._ext import require_native  # noqa: E402

C = require_native()
dev = torch.device("cuda", 0)
T, H, F = int(os.environ.get("FFN_TOKENS", 262144)), 1024, 4096


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
x8 = torch.randn(T, H, device=dev).to(torch.float8_e4m3fn)
w1 = torch.randn(F, H, device=dev).mul_(0.05).to(torch.float8_e4m3fn)
b1 = torch.randn(F, device=dev)
y = torch.empty(T, F, dtype=torch.bfloat16, device=dev)
pre = torch.empty(T, F, dtype=torch.bfloat16, device=dev)
a8 = torch.empty(T, F, dtype=torch.float8_e4m3fn, device=dev)
a8t = torch.empty(F, T, dtype=torch.float8_e4m3fn, device=dev)
r = {"tokens": T}
for cfg in (7, 5):
    r[f"cfg{cfg}_plain_ms"] = round(timeit(lambda: C.gemm_f8(x8, w1, y, 0, 0, one, one, cfg=cfg)), 4)
    r[f"cfg{cfg}_gelu_ms"] = round(timeit(lambda: C.gemm_f8(x8, w1, y, 0, 0, one, one, bias=b1, aux=pre, mode=1,
                                                          cfg=cfg)), 4)
r["q8_gelu_ms"] = round(timeit(lambda: C.gemm_f8_q(x8, w1, a8, a8t, 0, 0, one, one, 0, one, amax, bias=b1, aux=pre,
                                                   mode=1)), 4)
# FFN2-dgrad's quantising dGELU form: e5m2 dY (T x H) x W2 (stored [F][H]) -> e5m2 dA + its transpose,
# times gelu'(pre-activation), column sums (the FFN1 bias gradient)
dy8 = torch.randn(T, H, device=dev).to(torch.float8_e5m2)
g8 = torch.empty(T, F, dtype=torch.float8_e5m2, device=dev)
g8t = torch.empty(F, T, dtype=torch.float8_e5m2, device=dev)
cs = torch.zeros(F, device=dev)
r["q8_dgelu_ms"] = round(timeit(lambda: C.gemm_f8_q(dy8, w1, g8, g8t, 1, 0, one, one, 1, one, amax, aux=pre, mode=2,
                                                    colsum_out=cs, colsum_accumulate=True)), 4)
fl = 2.0 * T * F * H
for k in list(r):
    if k.endswith("_ms"):
        r[k.replace("_ms", "_tflops")] = round(fl / r[k] / 1e9, 1)
print(json.dumps(r), flush=True)
