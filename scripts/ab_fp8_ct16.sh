# fp8 cast-transpose with 16-byte stores (new, in-tree) vs ab/ (old): fp8 tests, then A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && rm -f gpurun_out/ab.jsonl
timeout -k 10 400 python -u -m pytest tests/test_fp8_gpu.py tests/test_fp8_fused_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/fp8_tests.log 2>&1 || exit 1
bash scripts/ab_so.sh "python3 -u benchmarks/fp8_ct_bench.py" "python3 -u bench.py --model large --batch 256 --steps 4 --warmup 2"
