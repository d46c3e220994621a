#!/bin/bash
# Round 4: LeNet driver protocol with / without the device-time events inside the timed region.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4z6
mkdir -p $O
for rep in 1 2 3; do
  for ev in 1 0; do
    MLT_BENCH_EVENTS=$ev timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-fp32-companion > $O/_l.json 2>$O/b.err || { tail $O/b.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/_l.json').read().strip().splitlines()[-1]); print(json.dumps({'events': $ev, 'ms_per_step': d['ms_per_step'], 'value': d['value']}))" | tee -a $O/events_ab.jsonl
  done
done
