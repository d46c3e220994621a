# 4-wave quantising GELU epilogue with its row loop unrolled by 8 (no scratch): fp8-fused tests and
# the FFN decomposition, alternated with the ping-pong form for reference
set -o pipefail
cd /tmp && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5af
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fp8_fused_gpu.py \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
: > $O/decomp.jsonl
for w in 1 0 1 0; do
  MLT_GEMM_W4Q8=$w timeout -k 10 120 python3 -u benchmarks/fp8_q8_decompose.py > $O/d.log 2>&1 || { tail -5 $O/d.log; exit 1; }
  echo "{\"w4q8\": $w, \"r\": $(tail -1 $O/d.log)}" >> $O/decomp.jsonl
  echo "w4q8=$w $(tail -1 $O/d.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["q8_gelu_ms"], d["q8_dgelu_ms"], d["cfg7_gelu_ms"])')"
done
