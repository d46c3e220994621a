# Round-5 profiles of the final kernels: the GEMM / transformer / fp8 GPU tests (incl. the
# cross-kernel GELU bit-equality test), then rocprofv3 kernel stats of the LeNet bf16 step at batch
# 32 and 4, BERT-base at batch 512 and fp8 `large` at batch 512, and the BERT / large benches under
# the driver protocol.
set -o pipefail
cd /tmp && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5l
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gemm_gpu.py tests/test_fp8_gpu.py tests/test_fp8_fused_gpu.py tests/test_transformer_gpu.py \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
prof() {  # name limit args...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" rocprofv3 --kernel-trace --stats --output-format csv -d $O/$name -o run -- python3 -u bench.py "$@" \
    > $O/$name.log 2>&1 || { echo "profile $name failed"; tail -5 $O/$name.log; exit 1; }
  cp "$(ls $O/$name/*/run_kernel_stats.csv 2>/dev/null || ls $O/$name/run_kernel_stats.csv)" $O/${name}_kernel_stats.csv
  tail -1 $O/$name.log
}
prof lenet_b32 180 --steps 3000 --warmup 200 --no-fp32-companion
prof lenet_b4 180 --batch 4 --steps 3000 --warmup 200 --no-fp32-companion
prof bert_b512 300 --model bert-base --batch 512 --steps 6 --warmup 2
prof large_b512 300 --model large --steps 6 --warmup 2
find $O -name "*.csv" -path "*/run*" -newer $O/tests.log | grep -v _kernel_stats.csv$ | xargs rm -f
timeout -k 10 240 python -u bench.py --model bert-base --steps 20 --warmup 5 > $O/bert.log 2>&1 && tail -1 $O/bert.log &&
timeout -k 10 300 python -u bench.py --model large --steps 6 --warmup 2 > $O/large.log 2>&1 && tail -1 $O/large.log
