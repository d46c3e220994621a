#!/bin/bash
# Round 4 final build: cfg 7 vs cfg 5 vs hipBLASLt (torch.matmul) at 64 K tokens, and the epilogue GEMMs at 256 K.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4z11
mkdir -p $O
timeout -k 10 400 python -u benchmarks/gemm_w4_bench.py > $O/gemm_w4_vs_hipblaslt.jsonl 2>$O/err.log || { tail $O/err.log; exit 1; }
python3 -c "
import json
for l in open('$O/gemm_w4_vs_hipblaslt.jsonl'):
    d=json.loads(l); print(d['shape'], d['cfg7_tflops'], d['torch_tflops'], d['cfg7_vs_torch'])"
GEMM_BENCH_TOKENS=262144 timeout -k 10 300 python -u benchmarks/gemm_epi_bench.py > $O/epi.jsonl 2>>$O/err.log || { tail $O/err.log; exit 1; }
cat $O/epi.jsonl
