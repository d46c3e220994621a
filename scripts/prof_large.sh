set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_large -o large -- python3 -u bench.py --model large --steps 4 --warmup 2 > gpurun_out/prof_large.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py --model large --steps 10 --warmup 3 > gpurun_out/bench_large.log 2>&1
