# LeNet chain: v3 = v1 + conv2 dgrad fragments loaded late (P6) + P0 loads on waves 0-7; v4 = v3 with
# conv1 on all 16 waves (MLT_KC1W=16). Tests + phases (in-tree = v3), then A/B v1 / v3 / v4.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r6d
O=gpurun_out/r6d
timeout -k 10 300 python -u -m pytest tests/test_lenet_bf16.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 &&
timeout -k 10 120 python3 -u benchmarks/lenet_bf16_phases.py 32 > $O/ph32.log 2>&1 &&
mkdir -p /tmp/abkeep && mv ab/base.so /tmp/abkeep/ &&
bash scripts/ab_multi_so.sh "python -u bench.py --no-fp32-companion" "python -u bench.py --steps 20 --warmup 5 --no-fp32-companion" "python -u bench.py --batch 4 --transport xgmi-loopback --no-fp32-companion" &&
cp gpurun_out/ab_multi.jsonl $O/ab.jsonl && cp ml_trainer_amd/_C*.so /tmp/intree.so && cp ab/v4.so ml_trainer_amd/_C.cpython-310-x86_64-linux-gnu.so &&
timeout -k 10 120 python3 -u benchmarks/lenet_bf16_phases.py 32 > $O/ph32_v4.log 2>&1; cp /tmp/intree.so ml_trainer_amd/_C.cpython-310-x86_64-linux-gnu.so
echo "rc=$?"
