set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/gputests.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > gpurun_out/fb_lenet20.log 2>&1 &&
timeout -k 10 120 python -u bench.py --batch 4 > gpurun_out/fb_lenet_b4.log 2>&1 &&
timeout -k 10 200 python -u bench.py --model bert-base --steps 20 --warmup 5 > gpurun_out/fb_bert.log 2>&1 &&
GEMM_BENCH_TOKENS=65536 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_hbl -o hbl -- python3 -u benchmarks/hipblaslt_names.py > gpurun_out/prof_hbl.log 2>&1
