#!/bin/bash
# Round 4: cfg 7 weight gradients (split-K) + tile gate: tests, wgrad bench, fp8 large + BERT-base A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4p
mkdir -p $O
true \
  || exit 1

GEMM_BENCH_TOKENS=262144 timeout -k 10 300 python -u benchmarks/wgrad_w4_bench.py > $O/wgrad_w4.jsonl 2>$O/wg.err || { tail $O/wg.err; exit 1; }
cut -c1-220 $O/wgrad_w4.jsonl
MLT_GEMM_W4=0 GEMM_BENCH_TOKENS=262144 timeout -k 10 300 python -u benchmarks/wgrad_w4_bench.py > $O/wgrad_pp.jsonl 2>$O/wg.err || { tail $O/wg.err; exit 1; }
cut -c1-220 $O/wgrad_pp.jsonl
for m in bert-base large; do
  for w in 1 0 1 0; do
    MLT_GEMM_W4=$w timeout -k 10 400 python -u bench.py --model $m --steps 6 --warmup 2 > $O/_b.json 2>$O/bench.err || { tail $O/bench.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/_b.json').read().strip().splitlines()[-1]); d['w4']=$w; print(json.dumps(d))" >> $O/ab_$m.jsonl
    tail -1 $O/ab_$m.jsonl | cut -c1-110
  done
done
