# Round 6, first GPU pass after deleting the one-launch step: the bf16 LeNet and multi-process GPU
# tests, then the headline bench (driver protocol + steady state), the weak-scaling W>1 proxies
# at batch 32 (xgmi-loopback / rccl-loopback) and the phase trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r6a
O=gpurun_out/r6a
timeout -k 10 400 python -u -m pytest tests/test_lenet_bf16.py tests/test_multiproc_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 &&
timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-fp32-companion > $O/drv.log 2>&1 &&
timeout -k 10 120 python -u bench.py --no-fp32-companion > $O/ss.log 2>&1 &&
timeout -k 10 120 python -u bench.py --batch 32 --transport xgmi-loopback --no-fp32-companion > $O/lb32_xgmi.log 2>&1 &&
timeout -k 10 120 python -u bench.py --batch 32 --transport rccl-loopback --no-fp32-companion > $O/lb32_rccl.log 2>&1 &&
timeout -k 10 120 python -u bench.py --batch 32 --transport xgmi-loopback --steps 20 --warmup 5 --no-fp32-companion > $O/lb32_xgmi_drv.log 2>&1 &&
timeout -k 10 120 python -u bench.py --batch 32 --transport rccl-loopback --steps 20 --warmup 5 --no-fp32-companion > $O/lb32_rccl_drv.log 2>&1 &&
timeout -k 10 120 python -u bench.py --batch 4 --transport xgmi-loopback --no-fp32-companion > $O/lb4_xgmi.log 2>&1 &&
timeout -k 10 120 python3 -u benchmarks/lenet_bf16_phases.py 32 > $O/ph32.log 2>&1
echo "rc=$?"
