#!/bin/bash
# Round 4: cfg 7 tile-count gate: GEMM / fp8 tests, fp8 large + BERT-base A/B (MLT_GEMM_W4 1/0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4o
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_fp8_gpu.py tests/test_gemm_gpu.py \
  > $O/t_gemm.log 2>&1 || { tail -30 $O/t_gemm.log; exit 1; }
tail -1 $O/t_gemm.log
for m in large bert-base; do
  for w in 1 0 1 0; do
    MLT_GEMM_W4=$w timeout -k 10 400 python -u bench.py --model $m --steps 6 --warmup 2 > $O/_b.json 2>$O/bench.err || { tail $O/bench.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/_b.json').read().strip().splitlines()[-1]); d['w4']=$w; print(json.dumps(d))" >> $O/ab_$m.jsonl
    tail -1 $O/ab_$m.jsonl | cut -c1-110
  done
done
timeout -k 10 400 python -u bench.py --model bert-large --steps 6 --warmup 2 --batch 256 > $O/bl.json 2>$O/bench.err || { tail $O/bench.err; exit 1; }
tail -1 $O/bl.json | cut -c1-150
timeout -k 10 400 python -u bench.py --model large --steps 6 --warmup 2 --batch 256 > $O/l256.json 2>$O/bench.err || { tail $O/bench.err; exit 1; }
tail -1 $O/l256.json | cut -c1-150
