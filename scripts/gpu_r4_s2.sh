#!/bin/bash
# Round 4 (packed-epilogue build): BERT-base b512 driver-protocol bench + kernel stats at b512, fp8 large kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4s2
mkdir -p $O
timeout -k 10 300 python -u bench.py --model bert-base --batch 512 --steps 20 --warmup 5 > $O/bert_b512.json 2>$O/b.err || { tail $O/b.err; exit 1; }
tail -1 $O/bert_b512.json | cut -c1-200
for spec in "bert-base 512" "large 512"; do
  set -- $spec
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$1 -o run -- \
    python3 -u bench.py --model $1 --batch $2 --steps 4 --warmup 2 > $O/$1.log 2>&1 || { tail $O/$1.log; exit 1; }
  f=$(find $O/$1 -name "*kernel_stats.csv" | head -1)
  cp $f $O/${1}_b$2_stats.csv
  python3 scripts/kstats.py $O/${1}_b$2_stats.csv 6 18 | cut -c1-150
done
# LeNet driver protocol (--steps 20 --warmup 5) by hipGraph length: 5 (the default rule) / 10 / 20
for rep in 1 2; do
  for spg in 5 10 20; do
    timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --steps-per-graph $spg --no-fp32-companion > $O/_l.json 2>$O/b.err || { tail $O/b.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/_l.json').read().strip().splitlines()[-1]); print(json.dumps({'spg': $spg, 'ms_per_step': d['ms_per_step'], 'device_ms_per_step': d['config']['device_ms_per_step'], 'value': d['value']}))" | tee -a $O/lenet_spg.jsonl
  done
done
