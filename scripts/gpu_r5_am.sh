# 4-wave quantising epilogues with the fp8-byte LDS image for the Y^T pass: fp8 tests, decomposition
# A/B (MLT_GEMM_W4Q8=1/0 = 4-wave / ping-pong), fp8 `large` A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5am
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fp8_fused_gpu.py \
  tests/test_fp8_gpu.py tests/test_transformer_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
: > $O/decomp.jsonl
for w in 1 0 1 0; do
  MLT_GEMM_W4Q8=$w timeout -k 10 120 python3 -u benchmarks/fp8_q8_decompose.py > $O/d.log 2>&1 || { tail -5 $O/d.log; exit 1; }
  echo "{\"w4q8\": $w, \"r\": $(tail -1 $O/d.log)}" >> $O/decomp.jsonl
  echo "w4q8=$w $(tail -1 $O/d.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["q8_gelu_ms"], d["q8_dgelu_ms"], d["cfg7_gelu_ms"])')"
done
: > $O/large.jsonl
for w in 1 0 1 0; do
  MLT_GEMM_W4Q8=$w timeout -k 10 300 python3 -u bench.py --model large --steps 10 --warmup 3 > $O/l.log 2>&1 || { tail -5 $O/l.log; exit 1; }
  echo "{\"w4q8\": $w, \"r\": $(grep '^{' $O/l.log)}" >> $O/large.jsonl
  echo "w4q8=$w $(grep '^{' $O/l.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
