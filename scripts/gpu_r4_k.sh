#!/bin/bash
# Round 4: cfg 7 forward + input-gradient layouts: tests, shape bench, full GEMM test file with the
# planner default, then BERT-base b512 MLT_GEMM_W4=1/0 alternated on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4k
mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gemm_gpu.py -k "w4" \
  > $O/t_w4.log 2>&1 || { tail -30 $O/t_w4.log; exit 1; }
tail -1 $O/t_w4.log
timeout -k 10 300 python -u benchmarks/gemm_w4_bench.py > $O/w4_bench.jsonl 2>$O/w4_bench.err || { tail $O/w4_bench.err; exit 1; }
python3 -c "import sys,json; [print(d['shape'], d['cfg5_tflops'], d['cfg7_tflops'], d['torch_tflops'], d['cfg7_vs_torch']) for d in map(json.loads, open('$O/w4_bench.jsonl'))]"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py \
  > $O/t_gemm.log 2>&1 || { tail -30 $O/t_gemm.log; exit 1; }
tail -1 $O/t_gemm.log
for w in 1 0 1 0; do
  MLT_GEMM_W4=$w timeout -k 10 300 python -u bench.py --model bert-base --steps 10 --warmup 3 > $O/_b.json 2>$O/bert.err || { tail $O/bert.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/_b.json').read().strip().splitlines()[-1]); d['w4']=$w; print(json.dumps(d))" >> $O/bert_ab.jsonl
  tail -1 $O/bert_ab.jsonl | cut -c1-120
done
