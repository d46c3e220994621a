#!/bin/bash
# Round 4: attention -delta fold (tests + B512 timing), cfg 7 side-operand prefetch (tests), BERT-base
# b512 MLT_GEMM_W4=1/0 alternated.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4m
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests -k "attn or attention or w4" \
  > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for b in 512 512; do ATTN_B=$b timeout -k 10 120 python3 -u benchmarks/attn_bench.py >> $O/attn_bench.jsonl 2>$O/attn.err || exit 1; done
cut -c1-140 $O/attn_bench.jsonl
for w in 1 0 1 0; do
  MLT_GEMM_W4=$w timeout -k 10 300 python -u bench.py --model bert-base --steps 10 --warmup 3 > $O/_b.json 2>$O/bert.err || { tail $O/bert.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/_b.json').read().strip().splitlines()[-1]); d['w4']=$w; print(json.dumps(d))" >> $O/bert_ab.jsonl
  tail -1 $O/bert_ab.jsonl | cut -c1-110
done
