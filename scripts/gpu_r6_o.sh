# Dry pre-warm replay touching the kernel-argument segments (v14) vs v13 (no dry support): tests on
# v14 (incl. the W=2/8 fused exchange after a dry launch), then a same-box A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r6o
O=gpurun_out/r6o
timeout -k 10 500 python -u -m pytest tests/test_lenet_bf16.py "tests/test_multiproc_gpu.py::test_lenet_bf16_fused_dp_matches_four_launch" -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
bash scripts/ab_multi_so.sh "python -u bench.py --steps 20 --warmup 5 --no-fp32-companion" "python -u bench.py --steps 20 --warmup 5 --no-fp32-companion --no-prewarm" "python -u bench.py --no-fp32-companion" "python -u bench.py --batch 4 --transport xgmi-loopback --no-fp32-companion" &&
cp gpurun_out/ab_multi.jsonl $O/ab.jsonl
echo "rc=$?"
