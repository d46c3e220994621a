set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gputests.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 120 python -u bench.py > gpurun_out/bench.log 2>&1 &&
timeout -k 10 180 python -u bench.py --model bert-base --steps 20 --warmup 5 > gpurun_out/bench_bert.log 2>&1
