#!/bin/bash
# Round 4: tile-raster group width for cfg 7 on BERT-base b512 (MLT_GEMM_GROUP_M 4 / 8 / 16, alternated).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4w
mkdir -p $O
for rep in 1 2; do
  for g in 4 8 16 2; do
    MLT_GEMM_GROUP_M=$g timeout -k 10 300 python -u bench.py --model bert-base --steps 10 --warmup 3 > $O/_b.json 2>$O/b.err || { tail $O/b.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/_b.json').read().strip().splitlines()[-1]); d['group_m']=$g; print(json.dumps(d))" >> $O/ab_groupm.jsonl
    tail -1 $O/ab_groupm.jsonl | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['group_m'], d['value'])"
  done
done
for b in 1024 512 1024 512; do
  timeout -k 10 400 python -u bench.py --model bert-base --steps 10 --warmup 3 --batch $b > $O/_b.json 2>$O/b.err || { tail $O/b.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/_b.json').read().strip().splitlines()[-1]); print(json.dumps(d))" >> $O/ab_batch.jsonl
  tail -1 $O/ab_batch.jsonl | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('batch', d['config']['global_batch'], d['value'])"
done
