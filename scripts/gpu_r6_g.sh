# LeNet chain: the trace stamps compiled out of the shipped kernel (v9a = swizzled fc1 image, v9r =
# round-5 layout) vs v1 (round-6 best so far); tests on the in-tree build (v9a), phases on the
# trace build (ab_trace.so), A/B v1 / v9a / v9r.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r6g
O=gpurun_out/r6g
SO=$(ls ml_trainer_amd/_C*.so)
timeout -k 10 300 python -u -m pytest tests/test_lenet_bf16.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 &&
bash scripts/ab_multi_so.sh "python -u bench.py --no-fp32-companion" "python -u bench.py --steps 20 --warmup 5 --no-fp32-companion" "python -u bench.py --batch 4 --transport xgmi-loopback --no-fp32-companion" &&
cp gpurun_out/ab_multi.jsonl $O/ab.jsonl && cp "$SO" /tmp/intree.so && cp ab_trace.so "$SO" &&
timeout -k 10 120 python3 -u benchmarks/lenet_bf16_phases.py 32 > $O/ph32.log 2>&1
rc=$?
cp /tmp/intree.so "$SO"
echo "rc=$rc"
