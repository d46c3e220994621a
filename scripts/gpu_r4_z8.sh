#!/bin/bash
# Round 4: LeNet bench without hipEvents in the timed region: driver protocol x3, batch 4, default,
# then the 2-rank rehearsal of the N>1 launch (both ranks on GPU 0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1 HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4z8
mkdir -p $O
for rep in 1 2 3; do
  timeout -k 10 180 python -u bench.py --steps 20 --warmup 5 > $O/lenet20_$rep.json 2>$O/b.err || { tail $O/b.err; exit 1; }
  tail -1 $O/lenet20_$rep.json | cut -c1-200
done
timeout -k 10 180 python -u bench.py --batch 4 --steps 20 --warmup 5 --no-fp32-companion > $O/lenet_b4_20.json 2>$O/b.err || { tail $O/b.err; exit 1; }
tail -1 $O/lenet_b4_20.json | cut -c1-200
timeout -k 10 180 python -u bench.py > $O/lenet_default.json 2>$O/b.err || { tail $O/b.err; exit 1; }
tail -1 $O/lenet_default.json | cut -c1-200
bash scripts/rehearse_2rank.sh || { tail -5 gpurun_out/r2_*.log; exit 1; }
for f in gpurun_out/r2_*.log; do echo "$f: $(tail -1 $f | cut -c1-160)"; done
