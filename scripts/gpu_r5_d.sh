# One-launch LeNet step: in-launch timeline (update blocks vs sample blocks), kernel stats, and
# the phase trace of the two-launch step for comparison.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 120 python3 -u benchmarks/lenet_onelaunch_trace.py 32 --jsonl gpurun_out/d_trace.jsonl > gpurun_out/d_trace32.log 2>&1 &&
timeout -k 10 120 python3 -u benchmarks/lenet_onelaunch_trace.py 4 --jsonl gpurun_out/d_trace.jsonl > gpurun_out/d_trace4.log 2>&1 &&
timeout -k 10 120 python3 -u benchmarks/lenet_bf16_phases.py 32 > gpurun_out/d_ph32.log 2>&1 &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/d_prof1 -o one -- python3 -u bench.py --steps 2000 --warmup 100 --no-fp32-companion > gpurun_out/d_prof1.log 2>&1
