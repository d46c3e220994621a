set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out &&
timeout -k 10 300 python -u -m pytest tests/test_fp8_gpu.py tests/test_transformer_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/fp8tests.log 2>&1 &&
timeout -k 10 200 python3 -u bench.py --model large --steps 8 --warmup 3 > gpurun_out/bench_large_wide.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_large3 -o large -- python3 -u bench.py --model large --steps 4 --warmup 2 > gpurun_out/prof_large3.log 2>&1
