"""Print which hipBLASLt kernels torch.matmul picks for the BERT GEMM shapes (run under rocprofv3)."""
import torch
dev = torch.device("cuda", 0)
import os
T = int(os.environ.get("GEMM_BENCH_TOKENS", 16384))
for M, N, K in [(T, 3072, 768), (T, 768, 3072), (T, 2304, 768), (T, 768, 768), (8192, 8192, 8192)]:
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    B = torch.randn(N, K, device=dev).to(torch.bfloat16)
    for _ in range(5):
        torch.matmul(A, B.t())
    torch.cuda.synchronize()
