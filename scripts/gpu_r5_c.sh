# One-launch step + fused-exchange bring-up: bf16 tests, multi-process transport tests, benches,
# and the available PMC counter list (for the granule-traffic pass).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_lenet_bf16.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/c_tests.log 2>&1 &&
timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > gpurun_out/c_lenet20.log 2>&1 &&
timeout -k 10 120 python -u bench.py > gpurun_out/c_lenet.log 2>&1 &&
timeout -k 10 120 python -u bench.py --batch 4 > gpurun_out/c_lenet_b4.log 2>&1 &&
timeout -k 10 120 python -u bench.py --batch 4 --transport xgmi-loopback > gpurun_out/c_lenet_b4_lb.log 2>&1 &&
MLT_LENET_ONELAUNCH=0 timeout -k 10 120 python -u bench.py > gpurun_out/c_lenet_2l.log 2>&1 &&
MLT_LENET_ONELAUNCH=0 timeout -k 10 120 python -u bench.py --batch 4 --transport xgmi-loopback > gpurun_out/c_lenet_b4_lb_2l.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_multiproc_gpu.py tests/test_trainer_parallel_gpu.py -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/c_mp_tests.log 2>&1
timeout -k 10 60 rocprofv3 --list-avail > gpurun_out/c_counters.txt 2>&1
