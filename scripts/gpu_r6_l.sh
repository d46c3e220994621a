# LeNet prep blocks from staged raw images:
# v13: wave 7 stages the raw image + target for the prep blocks (one round trip) vs v12.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r6l
O=gpurun_out/r6l
SO=$(ls ml_trainer_amd/_C*.so)
timeout -k 10 500 python -u -m pytest tests/test_lenet_bf16.py tests/test_multiproc_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 &&
bash scripts/ab_multi_so.sh "python -u bench.py --steps 1000 --warmup 100 --no-fp32-companion" "python -u bench.py --steps 20 --warmup 5 --no-fp32-companion" "python -u bench.py --batch 4 --transport xgmi-loopback --no-fp32-companion" &&
cp gpurun_out/ab_multi.jsonl $O/ab.jsonl && cp "$SO" /tmp/intree.so && cp ab_trace.so "$SO" &&
timeout -k 10 120 python3 -u benchmarks/lenet_bf16_phases.py 32 --jsonl $O/ph32.jsonl > $O/ph32.log 2>&1 &&
timeout -k 10 120 python3 -u benchmarks/lenet_phase_trace.py 32 > $O/fp32_ph32.log 2>&1
rc=$?
cp /tmp/intree.so "$SO"
echo "rc=$rc"
exit $rc
