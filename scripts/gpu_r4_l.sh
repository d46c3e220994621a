#!/bin/bash
# Round 4: BERT-base b512 kernel stats with the 4-wave GEMM on / off.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r4l
mkdir -p $O
for w in 1 0; do
  MLT_GEMM_W4=$w timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/w$w -o run -- \
    python3 -u bench.py --model bert-base --steps 5 --warmup 2 > $O/w$w.log 2>&1 || { tail $O/w$w.log; exit 1; }
  f=$(find $O/w$w -name "*kernel_stats.csv" | head -1)
  cp $f $O/bert_w$w.csv
  python3 scripts/kstats.py $O/bert_w$w.csv 7 14 | cut -c1-150
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests -k "attn or attention" \
  > $O/t_attn.log 2>&1 || { tail -30 $O/t_attn.log; exit 1; }
tail -1 $O/t_attn.log
for b in 512 512; do ATTN_B=$b timeout -k 10 120 python3 -u benchmarks/attn_bench.py >> $O/attn_bench.jsonl 2>$O/attn.err || exit 1; done
cat $O/attn_bench.jsonl
