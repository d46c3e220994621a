"""Attention backward with / without the fused QKV bias-gradient partials (colsum_out), and the
plain colsum pass it replaces; BERT-base shape (S 512, H 12), interleaved in one process."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_trainer_amd.ops._ext import require_native  # noqa: E402

C = require_native()
dev = torch.device("cuda", 0)
B, S, H = int(os.environ.get("ATTN_B", 128)), 512, 12
D = H * 64
g = torch.Generator().manual_seed(0)
qkv = (torch.randn(B * S, 3 * D, generator=g) * 0.5).to(torch.bfloat16).to(dev)
out = torch.empty(B * S, D, dtype=torch.bfloat16, device=dev)
lse = torch.empty(B * H * S, device=dev)
C.attn_fwd(qkv, out, lse, None, B, S, H, 0.125)
dout = (torch.randn(B * S, D, generator=g) * 0.5).to(torch.bfloat16).to(dev)
dqkv = torch.empty_like(qkv)
delta = torch.empty(B * S * H, device=dev)
cs = torch.empty(3 * D, device=dev)


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


fns = {
    "bwd": lambda: C.attn_bwd(qkv, out, dout, lse, delta, None, dqkv, B, S, H, 0.125),
    "bwd_fused_colsum": lambda: C.attn_bwd(qkv, out, dout, lse, delta, None, dqkv, B, S, H, 0.125, colsum_out=cs),
    "colsum_pass": lambda: C.colsum(dqkv, cs, False),
}
r = {k: [] for k in fns}
for _ in range(3):
    for k, f in fns.items():
        r[k].append(timeit(f))
print(json.dumps({"B": B, "S": S, "H": H, **{k + "_ms": round(min(v), 4) for k, v in r.items()}}), flush=True)
