"""Fused attention throughput (fwd / bwd) vs torch SDPA on BERT shapes; one JSON line per case."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.environ.get("ATTN_BENCH_PKG") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_trainer_amd.ops._ext import require_native  # noqa: E402

C = require_native()
dev = torch.device("cuda", 0)
B, S, H = int(os.environ.get("ATTN_B", 32)), int(os.environ.get("ATTN_S", 512)), 12
D = H * 64


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


qkv = torch.randn(B * S, 3 * D, device=dev).to(torch.bfloat16)
out = torch.empty(B * S, D, dtype=torch.bfloat16, device=dev)
lse = torch.empty(B * H * S, device=dev)
dout = torch.randn(B * S, D, device=dev).to(torch.bfloat16)
dqkv = torch.empty_like(qkv)
delta = torch.empty(B * S * H, device=dev)
C.attn_fwd(qkv, out, lse, None, B, S, H, 0.125)
q, k, v = qkv.view(B, S, 3, H, 64).permute(2, 0, 3, 1, 4)
q, k, v = [t.contiguous().requires_grad_() for t in (q, k, v)]
o = F.scaled_dot_product_attention(q, k, v)
go = dout.view(B, S, H, 64).transpose(1, 2).contiguous()
fl_f = 4.0 * B * H * S * S * 64

t = {
    "native_fwd": timeit(lambda: C.attn_fwd(qkv, out, lse, None, B, S, H, 0.125)),
    "native_bwd": timeit(lambda: C.attn_bwd(qkv, out, dout, lse, delta, None, dqkv, B, S, H, 0.125)),
    "sdpa_fwd": timeit(lambda: F.scaled_dot_product_attention(q, k, v)),
    "sdpa_bwd": timeit(lambda: torch.autograd.grad(o, (q, k, v), go, retain_graph=True)),
}
rec = {"B": B, "S": S, "H": H, **{k_: round(v_, 4) for k_, v_ in t.items()},
       "native_fwd_tflops": round(fl_f / t["native_fwd"] / 1e9, 1),
       "native_bwd_tflops": round(2.5 * fl_f / t["native_bwd"] / 1e9, 1),
       "sdpa_fwd_tflops": round(fl_f / t["sdpa_fwd"] / 1e9, 1),
       "sdpa_bwd_tflops": round(2.5 * fl_f / t["sdpa_bwd"] / 1e9, 1),
       "env": {k_: v_ for k_, v_ in os.environ.items() if k_.startswith("MLT_ATTN")}}
print(json.dumps(rec), flush=True)
