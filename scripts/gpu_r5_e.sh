# One-launch LeNet step, iteration 2 (update spread over the lenet_mw grid, hand-off-only drains):
# bf16 tests, in-launch timeline, benches.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_lenet_bf16.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/e_tests.log 2>&1 &&
timeout -k 10 120 python3 -u benchmarks/lenet_onelaunch_trace.py 32 --jsonl gpurun_out/e_trace.jsonl > gpurun_out/e_trace32.log 2>&1 &&
timeout -k 10 120 python3 -u benchmarks/lenet_onelaunch_trace.py 4 --jsonl gpurun_out/e_trace.jsonl > gpurun_out/e_trace4.log 2>&1 &&
timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > gpurun_out/e_lenet20.log 2>&1 &&
timeout -k 10 120 python -u bench.py > gpurun_out/e_lenet.log 2>&1 &&
timeout -k 10 120 python -u bench.py --batch 4 > gpurun_out/e_lenet_b4.log 2>&1 &&
timeout -k 10 120 python -u bench.py --batch 4 --transport xgmi-loopback > gpurun_out/e_lenet_b4_lb.log 2>&1 &&
MLT_LENET_ONELAUNCH=0 timeout -k 10 120 python -u bench.py > gpurun_out/e_lenet_2l.log 2>&1
