# LeNet chain: v10 = one-wave fc tail (fc2 fwd, fc3 + CE, fc3 dgrad, fc2 dgrad back to back on wave 0)
# vs v9r (stamps compiled out, round-5 fc1 layout). Tests on the in-tree build (v10), phases on the
# trace build, A/B v9r / v10 / v11 (v11 = v10 + probe flags and the fp32 kernel stamps compiled out; the
# steady-state command also measures the fp32 companion).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r6h
O=gpurun_out/r6h
SO=$(ls ml_trainer_amd/_C*.so)
timeout -k 10 500 python -u -m pytest tests/test_lenet_bf16.py tests/test_multiproc_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 &&
bash scripts/ab_multi_so.sh "python -u bench.py --steps 1000 --warmup 100" "python -u bench.py --steps 20 --warmup 5 --no-fp32-companion" "python -u bench.py --batch 4 --transport xgmi-loopback --no-fp32-companion" &&
cp gpurun_out/ab_multi.jsonl $O/ab.jsonl && cp "$SO" /tmp/intree.so && cp ab_trace.so "$SO" &&
timeout -k 10 120 python3 -u benchmarks/lenet_bf16_phases.py 32 > $O/ph32.log 2>&1
rc=$?
cp /tmp/intree.so "$SO"
echo "rc=$rc"
