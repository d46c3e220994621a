# the 4-wave kernel's quantising fp8 GELU epilogue (gemm_w4.hip W4_Q8GELU): fp8 GEMM tests, the
# FFN1 decomposition with MLT_GEMM_W4Q8=1/0, and the fp8 `large` step A/B (alternated)
set -o pipefail
cd /tmp && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5ab
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fp8_fused_gpu.py \
  tests/test_fp8_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
: > $O/decomp.jsonl
for w in 1 0 1 0; do
  MLT_GEMM_W4Q8=$w timeout -k 10 120 python3 -u benchmarks/fp8_q8_decompose.py > $O/d.log 2>&1 || { tail -5 $O/d.log; exit 1; }
  echo "{\"w4q8\": $w, \"r\": $(tail -1 $O/d.log)}" | tee -a $O/decomp.jsonl
done
: > $O/large.jsonl
for w in 1 0 1 0; do
  MLT_GEMM_W4Q8=$w timeout -k 10 300 python3 -u bench.py --model large --steps 10 --warmup 3 > $O/l.log 2>&1 || { tail -5 $O/l.log; exit 1; }
  echo "{\"w4q8\": $w, \"r\": $(grep '^{' $O/l.log)}" | tee -a $O/large.jsonl
done
