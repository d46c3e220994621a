# lenet_mfma.hip built with -fno-slp-vectorize (new, in-tree) vs without (ab/): bf16 tests, then A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && rm -f gpurun_out/ab.jsonl
timeout -k 10 300 python -u -m pytest tests/test_lenet_bf16.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/lenet_tests.log 2>&1 || exit 1
bash scripts/ab_so.sh "python3 -u bench.py --batch 32" "python3 -u bench.py --batch 4" "python3 -u bench.py --steps 20 --warmup 5"
