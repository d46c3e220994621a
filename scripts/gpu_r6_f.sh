# LeNet chain: v1 (round-6 best) vs v1r (v1 rebuilt from the current source), v8a (+ swizzled fc1 image),
# v8b (+ counted vmcnt before P4a). Tests + phases on the in-tree build (v8a), then A/B.

set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r6f
O=gpurun_out/r6f
timeout -k 10 300 python -u -m pytest tests/test_lenet_bf16.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 &&
timeout -k 10 120 python3 -u benchmarks/lenet_bf16_phases.py 32 > $O/ph32.log 2>&1 &&
bash scripts/ab_multi_so.sh "python -u bench.py --no-fp32-companion" "python -u bench.py --steps 20 --warmup 5 --no-fp32-companion" "python -u bench.py --batch 4 --transport xgmi-loopback --no-fp32-companion" &&
cp gpurun_out/ab_multi.jsonl $O/ab.jsonl
echo "rc=$?"
