# ln_bwd_q8 with 768 blocks: fp8-fused tests, fp8 `large` A/B (MLT_FP8_LN_Q=1/0), kernel time
set -o pipefail
cd /tmp && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${R5_OUT:-r5ak}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fp8_fused_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
: > $O/large.jsonl
for w in 1 0 1 0; do
  MLT_FP8_LN_Q=$w timeout -k 10 300 python3 -u bench.py --model large --steps 10 --warmup 3 > $O/l.log 2>&1 || { tail -5 $O/l.log; exit 1; }
  echo "{\"ln_q\": $w, \"r\": $(grep '^{' $O/l.log)}" >> $O/large.jsonl
  echo "ln_q=$w $(grep '^{' $O/l.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o large -- python3 -u bench.py --model large --steps 2 --warmup 1 > $O/p.log 2>&1 || { tail -20 $O/p.log; exit 1; }
f=$(find $O/prof -name '*kernel_stats.csv' | head -1)
grep -E "ln_bwd_q8" "$f" | cut -c1-230
