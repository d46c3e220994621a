# LeNet: back to the round-5 barrier-phase fc chain (the one-wave fc tail of r6h measured 1.4 us per
# step slower) with the trace stamps compiled out; phase trace incl. the KW prep blocks.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r6i
O=gpurun_out/r6i
SO=$(ls ml_trainer_amd/_C*.so)
timeout -k 10 500 python -u -m pytest tests/test_lenet_bf16.py tests/test_multiproc_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 &&
timeout -k 10 200 python -u bench.py --steps 1000 --warmup 100 > $O/bench.log 2>&1 &&
timeout -k 10 200 python -u bench.py > $O/bench_default.log 2>&1 &&
cp "$SO" /tmp/intree.so && cp ab_trace.so "$SO" &&
timeout -k 10 120 python3 -u benchmarks/lenet_bf16_phases.py 32 --jsonl $O/ph32.jsonl > $O/ph32.log 2>&1
rc=$?
cp /tmp/intree.so "$SO"
echo "rc=$rc"
exit $rc
