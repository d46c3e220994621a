"""fp8 quantisation kernel throughput (cast with / without amax, amax alone, cast-transpose)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_trainer_amd.ops._ext import require_native  # noqa: E402

C = require_native()
dev = torch.device("cuda", 0)


def timeit(fn, iters=50):
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
for shape in [(8192, 1024), (8192, 4096), (16384, 3072), (262144, 1024)]:
    x = torch.randn(*shape, device=dev).to(torch.bfloat16)
    y = torch.empty(shape, dtype=torch.float8_e4m3fn, device=dev)
    n = x.numel()
    t_amax = timeit(lambda: C.fp8_cast(x, y, scale, amax, 0))
    t_noamax = timeit(lambda: C.fp8_cast(x, y, scale, None, 0))
    t_amax_only = timeit(lambda: C.fp8_amax(x, amax))
    t_copy = timeit(lambda: y.view(torch.uint8).copy_(x.view(torch.uint8).view(-1)[:n].view(shape)))
    print(json.dumps({"shape": shape, "cast_amax_us": round(t_amax, 2), "cast_us": round(t_noamax, 2),
                      "GBps": round(3 * n / t_noamax / 1e3, 1),
                      "amax_us": round(t_amax_only, 2), "amax_GBps": round(2 * n / t_amax_only / 1e3, 1), "torch_u8_copy_us": round(t_copy, 2)}), flush=True)
w = torch.randn(4096, 1024, device=dev)
w8 = torch.empty(4096, 1024, dtype=torch.float8_e4m3fn, device=dev)
wt = torch.empty(1024, 4096, dtype=torch.float8_e4m3fn, device=dev)
print(json.dumps({"cast_transpose_4096x1024_us": round(timeit(lambda: C.fp8_cast_transpose(w, w8, wt, scale, amax, 0)), 2)}))
