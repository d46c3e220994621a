# LayerNorm backward that quantises the out-proj / FFN2 dY (ln_bwd_q8): fp8 + transformer GPU tests,
# then the fp8 `large` step with MLT_FP8_LN_Q=1/0 alternated
set -o pipefail
cd /tmp && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5ai
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fp8_fused_gpu.py \
  tests/test_fp8_gpu.py tests/test_transformer_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
: > $O/large.jsonl
for w in 1 0 1 0; do
  MLT_FP8_LN_Q=$w timeout -k 10 300 python3 -u bench.py --model large --steps 10 --warmup 3 > $O/l.log 2>&1 || { tail -5 $O/l.log; exit 1; }
  echo "{\"ln_q\": $w, \"r\": $(grep '^{' $O/l.log)}" >> $O/large.jsonl
  echo "ln_q=$w $(grep '^{' $O/l.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["loss_finite"])')"
done
