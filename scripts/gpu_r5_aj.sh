# kernel trace of the fp8 `large` step with the LayerNorm-quantised dY (ln_bwd_q8)
set -o pipefail
cd /tmp && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5aj
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o large -- python3 -u bench.py --model large --steps 3 --warmup 2 > $O/p.log 2>&1 || { tail -20 $O/p.log; exit 1; }
grep '^{' $O/p.log | cut -c1-200
f=$(find $O/prof -name '*kernel_stats.csv' | head -1)
grep -E "ln_bwd|cast_transpose_fp8_wide" "$f" | cut -c1-220
