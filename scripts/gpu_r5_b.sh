# One-launch bf16 LeNet step: bf16 tests (bitwise vs the two-launch step), then the driver-protocol
# bench, steady state b32 / b4, the xGMI loopback at b4, and the two-launch A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_lenet_bf16.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/b_tests.log 2>&1 &&
timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > gpurun_out/b_lenet20.log 2>&1 &&
timeout -k 10 120 python -u bench.py > gpurun_out/b_lenet.log 2>&1 &&
timeout -k 10 120 python -u bench.py --batch 4 > gpurun_out/b_lenet_b4.log 2>&1 &&
timeout -k 10 120 python -u bench.py --batch 4 --transport xgmi-loopback > gpurun_out/b_lenet_b4_lb.log 2>&1 &&
MLT_LENET_ONELAUNCH=0 timeout -k 10 120 python -u bench.py > gpurun_out/b_lenet_2l.log 2>&1 &&
MLT_LENET_ONELAUNCH=0 timeout -k 10 120 python -u bench.py --batch 4 --transport xgmi-loopback > gpurun_out/b_lenet_b4_lb_2l.log 2>&1
