#!/bin/bash
# Round 4: BERT-base / fp8 large kernel stats, then the prefetcher copy/compute overlap trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4s
mkdir -p $O
for m in bert-base large; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$m -o run -- \
    python3 -u bench.py --model $m --steps 4 --warmup 2 > $O/$m.log 2>&1 || { tail $O/$m.log; exit 1; }
  f=$(find $O/$m -name "*kernel_stats.csv" | head -1)
  cp $f $O/${m}_stats.csv
  python3 scripts/kstats.py $O/${m}_stats.csv 6 16 | cut -c1-150
done
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/pf -o run -- \
  python3 -u benchmarks/prefetch_overlap_trace.py > $O/pf.log 2>&1 || { tail $O/pf.log; exit 1; }
python3 benchmarks/prefetch_overlap_trace.py --summarize $O/pf > $O/prefetch_overlap.txt
tail -4 $O/prefetch_overlap.txt
