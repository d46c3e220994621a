# q8 GELU raster width 2 (dGELU 4) vs 4 / 4: fp8-fused tests + fp8 `large` A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5ap
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fp8_fused_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
: > $O/large.jsonl
for g in 0 4 0 4; do
  if [ $g = 0 ]; then unset MLT_GEMM_W4Q8_GROUP_M; else export MLT_GEMM_W4Q8_GROUP_M=$g; fi
  timeout -k 10 300 python3 -u bench.py --model large --steps 10 --warmup 3 > $O/l.log 2>&1 || { tail -5 $O/l.log; exit 1; }
  echo "{\"q_group_m\": \"${g/0/default 2-4}\", \"r\": $(grep '^{' $O/l.log)}" >> $O/large.jsonl
  echo "group_m=$g $(grep '^{' $O/l.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
