"""BERT-base GEMMs with their fused epilogues (GEMM_BENCH_TOKENS, default 16384): FFN1 forward with bias + GELU
(writes the pre-activation too), FFN2 dgrad with the dGELU epilogue (reads it back), the
out-projection forward with bias + residual, and the plain forms for comparison."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_trainer_amd.ops._ext import require_native  # noqa: E402

C = require_native()
dev = torch.device("cuda", 0)
T = int(os.environ.get("GEMM_BENCH_TOKENS", 16384))


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def bf(*shape):
    return torch.randn(*shape, device=dev).to(torch.bfloat16)


x, w1, w2, wo = bf(T, 768), bf(3072, 768), bf(768, 3072), bf(768, 768)
b1, bo = torch.randn(3072, device=dev), torch.randn(768, device=dev)
h, aux = torch.empty(T, 3072, dtype=torch.bfloat16, device=dev), bf(T, 3072)
dy, dh = bf(T, 768), torch.empty(T, 3072, dtype=torch.bfloat16, device=dev)
db1 = torch.empty(3072, device=dev)
y, res = torch.empty(T, 768, dtype=torch.bfloat16, device=dev), bf(T, 768)
cases = {
    "ffn1_fwd_plain": (lambda: C.gemm(x, w1, h, False, False), 2.0 * T * 3072 * 768),
    "ffn1_fwd_bias_gelu": (lambda: C.gemm(x, w1, h, False, False, bias=b1, aux=aux, mode=1), 2.0 * T * 3072 * 768),
    "ffn2_dgrad_plain": (lambda: C.gemm(dy, w2, dh, False, True), 2.0 * T * 3072 * 768),
    "ffn2_dgrad_dgelu": (lambda: C.gemm(dy, w2, dh, False, True, aux=aux, mode=2), 2.0 * T * 3072 * 768),
    "ffn2_dgrad_dgelu_colsum": (lambda: C.gemm(dy, w2, dh, False, True, aux=aux, mode=2, colsum_out=db1),
                                2.0 * T * 3072 * 768),
    "out_fwd_plain": (lambda: C.gemm(x, wo, y, False, False), 2.0 * T * 768 * 768),
    "out_fwd_bias_res": (lambda: C.gemm(x, wo, y, False, False, bias=bo, res=res), 2.0 * T * 768 * 768),
}
r = {"tokens": T}
for k, (fn, fl) in cases.items():
    t = min(timeit(fn) for _ in range(3))
    r[k + "_us"] = round(t * 1e3, 1)
    r[k + "_tflops"] = round(fl / t / 1e9, 1)
print(json.dumps(r), flush=True)
