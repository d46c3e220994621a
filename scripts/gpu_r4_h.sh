#!/bin/bash
# Round 4: cfg 7 with the peeled C = 0 first tile and the LDS-staged 16-byte epilogue.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4h
mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gemm_gpu.py -k "w4" \
  > $O/t_w4.log 2>&1 || { tail -30 $O/t_w4.log; exit 1; }
tail -1 $O/t_w4.log
timeout -k 10 300 python -u benchmarks/gemm_w4_bench.py > $O/w4_bench.jsonl 2>$O/w4_bench.err || { tail $O/w4_bench.err; exit 1; }
python3 -c "import sys,json; [print(d['shape'], d['cfg5_tflops'], d['cfg7_tflops'], d['torch_tflops'], d['cfg7_vs_torch']) for d in map(json.loads, open('$O/w4_bench.jsonl'))]"
