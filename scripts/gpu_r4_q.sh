#!/bin/bash
# Round 4: kernel stats of BERT-base b512 and fp8 large b512 with cfg 7 everywhere it applies.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4q
mkdir -p $O
for m in bert-base large; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$m -o run -- \
    python3 -u bench.py --model $m --steps 4 --warmup 2 > $O/$m.log 2>&1 || { tail $O/$m.log; exit 1; }
  f=$(find $O/$m -name "*kernel_stats.csv" | head -1)
  cp $f $O/${m}_stats.csv
  python3 scripts/kstats.py $O/${m}_stats.csv 6 16 | cut -c1-150
done
