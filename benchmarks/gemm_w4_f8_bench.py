"""fp8 GEMM: config 7 (4-wave asm loop on the block-scaled MFMA) vs configs 5 / 6 (ping-pong /
persistent ping-pong) and the bf16 config 7, on the `large` (24L / 1024H / FFN 4096) shapes at 128K
tokens and a square; interleaved rounds, random operands, one JSON line per shape."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_trainer_amd.ops._ext import require_native  # noqa: E402

C = require_native()
dev = torch.device("cuda", 0)
T = int(os.environ.get("GEMM_BENCH_TOKENS", 131072))
shapes = [("qkv", T, 3072, 1024), ("out", T, 1024, 1024), ("ffn1", T, 4096, 1024), ("ffn2", T, 1024, 4096),
          ("sq8192", 8192, 8192, 8192)]


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


one = torch.ones(1, device=dev)
for name, M, N, K in shapes:
    A8 = (torch.rand(M, K, device=dev) - 0.5).to(torch.float8_e4m3fn)
    B8 = (torch.rand(N, K, device=dev) - 0.5).to(torch.float8_e4m3fn)
    A16 = (torch.rand(M, K, device=dev) - 0.5).to(torch.bfloat16)
    B16 = (torch.rand(N, K, device=dev) - 0.5).to(torch.bfloat16)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    fns = {"f8_cfg7": lambda: C.gemm_f8(A8, B8, out, 0, 0, one, one, cfg=7),
           "f8_cfg5": lambda: C.gemm_f8(A8, B8, out, 0, 0, one, one, cfg=5),
           "f8_cfg6": lambda: C.gemm_f8(A8, B8, out, 0, 0, one, one, cfg=6),
           "bf16_cfg7": lambda: C.gemm(A16, B16, out, False, False, cfg=7),
           "bf16_torch": lambda: torch.matmul(A16, B16.t(), out=out)}
    best = {k: 1e9 for k in fns}
    for _ in range(3):
        for k, f in fns.items():
            best[k] = min(best[k], timeit(f))
    fl = 2.0 * M * N * K
    r = {"shape": name, "M": M, "N": N, "K": K}
    for k, v in best.items():
        r[k + "_tflops"] = round(fl / v / 1e9, 1)
    r["f8_cfg7_vs_bf16_cfg7"] = round(best["bf16_cfg7"] / best["f8_cfg7"], 3)
    print(json.dumps(r), flush=True)
