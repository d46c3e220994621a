#!/bin/bash
# Round 4: cfg 7 main-loop variants (MLT_W4_VARIANT 0 glds / 1 spread glds / 2 register staging):
# correctness for each, then the shape bench for each, one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4g
mkdir -p $O
for v in 2 1 0; do
  MLT_W4_VARIANT=$v timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gemm_gpu.py -k "w4" \
    > $O/t_w4_v$v.log 2>&1 || { tail -30 $O/t_w4_v$v.log; exit 1; }
  echo "v$v: $(tail -1 $O/t_w4_v$v.log)"
done
for v in 0 1 2; do
  MLT_W4_VARIANT=$v timeout -k 10 300 python -u benchmarks/gemm_w4_bench.py > $O/w4_bench_v$v.jsonl 2>$O/w4_bench.err || { tail $O/w4_bench.err; exit 1; }
  echo "== v$v"; cat $O/w4_bench_v$v.jsonl | python3 -c "import sys,json; [print(d['shape'], d['cfg5_tflops'], d['cfg7_tflops'], d['torch_tflops'], d['cfg7_vs_torch']) for d in map(json.loads, sys.stdin)]"
done
