#!/bin/bash
# Round 4: cfg 7 persistent with per-XCD contiguous tile runs (MLT_W4_PERSIST=1) vs one tile per
# workgroup: GEMM tests under persist, shape bench both ways, BERT-base A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4t
mkdir -p $O
MLT_W4_PERSIST=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gemm_gpu.py -k "w4 or dgelu" \
  > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for p in 1 0 1 0; do
  MLT_W4_PERSIST=$p timeout -k 10 300 python -u benchmarks/gemm_w4_bench.py > $O/b_p$p.jsonl 2>$O/b.err || { tail $O/b.err; exit 1; }
  echo "== persist=$p"; python3 -c "import json; [print(d['shape'], d['cfg7_tflops'], d['torch_tflops'], d['cfg7_vs_torch']) for d in map(json.loads, open('$O/b_p$p.jsonl'))]"
done
for p in 1 0 1 0; do
  MLT_W4_PERSIST=$p timeout -k 10 400 python -u bench.py --model bert-base --steps 6 --warmup 2 > $O/_b.json 2>$O/bench.err || { tail $O/bench.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/_b.json').read().strip().splitlines()[-1]); d['persist']=$p; print(json.dumps(d))" >> $O/ab_bert.jsonl
  tail -1 $O/ab_bert.jsonl | cut -c1-100
done
