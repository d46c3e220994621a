# LeNet fc1 image by LDS-DMA: bf16 tests, phase trace, then same-box A/B against ab/ (round start build)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r6b
O=gpurun_out/r6b
timeout -k 10 300 python -u -m pytest tests/test_lenet_bf16.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 &&
timeout -k 10 120 python3 -u benchmarks/lenet_bf16_phases.py 32 > $O/ph32.log 2>&1 &&
rm -f gpurun_out/ab.jsonl &&
bash scripts/ab_so.sh "python -u bench.py --no-fp32-companion" "python -u bench.py --steps 20 --warmup 5 --no-fp32-companion" "python -u bench.py --batch 4 --transport xgmi-loopback --no-fp32-companion" &&
cp gpurun_out/ab.jsonl $O/ab.jsonl
echo "rc=$?"
