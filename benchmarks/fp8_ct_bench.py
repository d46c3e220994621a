"""Activation / gradient fp8 cast-transpose (bf16 [tokens, C] -> e4m3 / e5m2 + transpose, the wide
128x128 kernel) at the `large` config's shapes; one JSON line: microseconds and effective TB/s."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_trainer_amd.ops._ext import require_native  # noqa: E402

C = require_native()
dev = torch.device("cuda", 0)
T = int(os.environ.get("CT_TOKENS", 131072))


def timeit(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3


scale = torch.ones(1, device=dev)
amax = torch.zeros(C.FP8_AMAX_SLOTS, device=dev)
rec = {"tokens": T}
for cols in (1024, 3072):
    x = torch.randn(T, cols, device=dev).to(torch.bfloat16)
    y = torch.empty(T, cols, dtype=torch.float8_e5m2, device=dev)
    yt = torch.empty(cols, T, dtype=torch.float8_e5m2, device=dev)
    cs = torch.empty(cols, dtype=torch.float32, device=dev)
    t = timeit(lambda: C.fp8_cast_transpose(x, y, yt, scale, amax, 1))
    tc = timeit(lambda: C.fp8_cast_transpose(x, y, yt, scale, amax, 1, colsum_out=cs))
    rec[f"c{cols}_us"] = round(t, 2)
    rec[f"c{cols}_colsum_us"] = round(tc, 2)
    rec[f"c{cols}_TBps"] = round(4 * T * cols / t / 1e6, 2)
print(json.dumps(rec), flush=True)
