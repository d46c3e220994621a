#!/bin/bash
# Round 4: LeNet bench with the device-time events moved to the warmup (driver protocol x3, batch 4, default).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4z7
mkdir -p $O
for rep in 1 2 3; do
  timeout -k 10 180 python -u bench.py --steps 20 --warmup 5 > $O/lenet20_$rep.json 2>$O/b.err || { tail $O/b.err; exit 1; }
  tail -1 $O/lenet20_$rep.json | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); c=d['config']; print(d['value'], d['ms_per_step'], c['warmup_device_ms_per_step'], c.get('fp32_samples_per_s'))"
done
timeout -k 10 180 python -u bench.py --batch 4 --steps 20 --warmup 5 --no-fp32-companion > $O/lenet_b4_20.json 2>$O/b.err || { tail $O/b.err; exit 1; }
tail -1 $O/lenet_b4_20.json | cut -c1-160
timeout -k 10 180 python -u bench.py > $O/lenet_default.json 2>$O/b.err || { tail $O/b.err; exit 1; }
tail -1 $O/lenet_default.json | cut -c1-160
