set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 120 python3 -u benchmarks/lenet_bf16_phases.py 32 --jsonl gpurun_out/lenet_phases_r3b.jsonl > gpurun_out/ph32.log 2>&1 &&
timeout -k 10 120 python3 -u benchmarks/lenet_bf16_phases.py 4 --jsonl gpurun_out/lenet_phases_r3b.jsonl > gpurun_out/ph4.log 2>&1 &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lenet -o b32 -- python3 -u bench.py --batch 32 --steps 400 --warmup 20 > gpurun_out/prof_lenet.log 2>&1
