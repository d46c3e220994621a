# Round-3 final validation on one MI355X: full GPU suite, smoke, driver-protocol benches for every
# config, kernel stats for LeNet b32 and BERT-base b512. Outputs under gpurun_out/final/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/final && O=gpurun_out/final
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider > $O/gputests.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > $O/lenet20.log 2>&1 &&
timeout -k 10 120 python -u bench.py > $O/lenet.log 2>&1 &&
timeout -k 10 120 python -u bench.py --batch 4 > $O/lenet_b4.log 2>&1 &&
timeout -k 10 200 python -u bench.py --model bert-base --steps 20 --warmup 5 > $O/bert.log 2>&1 &&
timeout -k 10 240 python -u bench.py --model large --steps 6 --warmup 2 > $O/large.log 2>&1 &&
timeout -k 10 200 python -u bench.py --model bert-large --steps 4 --warmup 2 > $O/bertlarge.log 2>&1 &&
timeout -k 10 240 python -u bench.py --model large --batch 256 --steps 6 --warmup 2 > $O/large_b256.log 2>&1 &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_lenet -o b32 -- python3 -u bench.py --steps 400 --warmup 20 > $O/prof_lenet.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bert -o bert -- python3 -u bench.py --model bert-base --steps 5 --warmup 2 > $O/prof_bert.log 2>&1
