# Next-step input prep in the batch-reduction kernel: bf16 tests, then benches with prep on / off
# (same box, alternated), b32 / b4 / loopback.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_lenet_bf16.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/f_tests.log 2>&1 &&
for rep in 1 2; do
  for pr in 1 0; do
    MLT_LENET_ONELAUNCH=0 MLT_LENET_PREP=$pr timeout -k 10 120 python -u bench.py --no-fp32-companion > gpurun_out/f_b32_p${pr}_$rep.log 2>&1 || exit 1
    MLT_LENET_ONELAUNCH=0 MLT_LENET_PREP=$pr timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-fp32-companion > gpurun_out/f_drv_p${pr}_$rep.log 2>&1 || exit 1
    MLT_LENET_ONELAUNCH=0 MLT_LENET_PREP=$pr timeout -k 10 120 python -u bench.py --batch 4 --no-fp32-companion > gpurun_out/f_b4_p${pr}_$rep.log 2>&1 || exit 1
    MLT_LENET_ONELAUNCH=0 MLT_LENET_PREP=$pr timeout -k 10 120 python -u bench.py --batch 4 --transport xgmi-loopback --no-fp32-companion > gpurun_out/f_lb4_p${pr}_$rep.log 2>&1 || exit 1
  done
done
MLT_LENET_ONELAUNCH=0 timeout -k 10 120 python3 -u benchmarks/lenet_bf16_phases.py 32 > gpurun_out/f_ph32.log 2>&1
