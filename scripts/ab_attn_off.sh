# attention backward with offset-immediate transposed reads (new, in-tree) vs ab/ (old)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && rm -f gpurun_out/ab.jsonl
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py -m gpu -x -q -k "attn or attention" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/attn_tests.log 2>&1 || exit 1
bash scripts/ab_so.sh "ATTN_B=128 python3 -u benchmarks/attn_bench.py" "ATTN_B=512 python3 -u benchmarks/attn_bench.py" "python3 -u bench.py --model bert-base --steps 10 --warmup 3"
