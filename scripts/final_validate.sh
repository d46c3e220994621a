# Round-end validation on one MI355X: full GPU suite, smoke, driver-protocol benches, BERT-base
# kernel stats. Outputs under gpurun_out/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/gputests.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > gpurun_out/fb_lenet20.log 2>&1 &&
timeout -k 10 120 python -u bench.py > gpurun_out/fb_lenet.log 2>&1 &&
timeout -k 10 200 python -u bench.py --model bert-base --steps 20 --warmup 5 > gpurun_out/fb_bert.log 2>&1 &&
timeout -k 10 200 python -u bench.py --model large --steps 6 --warmup 2 > gpurun_out/fb_large.log 2>&1 &&
timeout -k 10 200 python -u bench.py --model bert-large --steps 4 --warmup 2 > gpurun_out/fb_bertlarge.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bert -o bert -- python3 -u bench.py --model bert-base --steps 5 --warmup 2 > gpurun_out/prof_bert.log 2>&1
