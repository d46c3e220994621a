# fp8 training: the attention backward writes the QKV projection's e5m2 dY + transpose + amax
# (no bf16 dQKV, no cast pass): tests (bitwise vs bf16 + cast; a fp8 layer trained both ways;
# the attention / fp8 suites), then the `large` step with MLT_FP8_ATTN_Q=1 / 0 alternated, and
# BERT-base (bf16, unaffected path) once.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r6x
O=gpurun_out/r6x
timeout -k 10 600 python -u -m pytest tests/test_fp8_fused_gpu.py tests/test_fp8_gpu.py tests/test_transformer_gpu.py tests/test_gemm_gpu.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
: > $O/large.jsonl
for rep in 1 2; do
  for q in 1 0; do
    MLT_FP8_ATTN_Q=$q timeout -k 10 300 python3 -u bench.py --model large --steps 20 --warmup 5 > $O/l.log 2>&1 || { tail -5 $O/l.log; exit 1; }
    echo "{\"attn_q\": $q, \"r\": $(grep '^{' $O/l.log)}" >> $O/large.jsonl
  done
done
timeout -k 10 300 python3 -u bench.py --model bert-base --steps 20 --warmup 5 > $O/bert.log 2>&1
echo "rc=$?"
