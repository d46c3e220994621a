# Role-B activation stores of P7 spread over waves 8-15 (v19) vs on wave 15 (v18): tests on v19
# (incl. the fp32 prewarm), same-box A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r6t
O=gpurun_out/r6t
timeout -k 10 500 python -u -m pytest tests/test_lenet_bf16.py "tests/test_multiproc_gpu.py::test_lenet_bf16_fused_dp_matches_four_launch" -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
bash scripts/ab_multi_so.sh "python -u bench.py --steps 20 --warmup 5" "python -u bench.py --no-fp32-companion" "python -u bench.py --batch 4 --transport xgmi-loopback --no-fp32-companion" &&
cp gpurun_out/ab_multi.jsonl $O/ab.jsonl
echo "rc=$?"
