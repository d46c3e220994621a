# Round-5 baseline on one MI355X: LeNet bf16 step (driver protocol, steady state b32 / b4) and
# its kernel stats, before the one-launch step.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > gpurun_out/a_lenet20.log 2>&1 &&
timeout -k 10 120 python -u bench.py > gpurun_out/a_lenet.log 2>&1 &&
timeout -k 10 120 python -u bench.py --batch 4 > gpurun_out/a_lenet_b4.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/a_prof -o lenet -- python3 -u bench.py --steps 2000 --warmup 100 > gpurun_out/a_prof.log 2>&1
