# Round-6 validation on one MI355X: full GPU suite + smoke (part 1); driver-protocol benches of
# every BASELINE config and the LeNet kernel stats (part 2: MLT_FINAL_PART=2). Outputs under
# gpurun_out/final_r6/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/final_r6
O=gpurun_out/final_r6
if [ "${MLT_FINAL_PART:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > $O/gputests.log 2>&1 &&
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
  rc=$?; echo "rc=$rc"; exit $rc
fi
timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > $O/lenet20_a.log 2>&1 &&
timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > $O/lenet20_b.log 2>&1 &&
timeout -k 10 200 python -u bench.py > $O/lenet_steady.log 2>&1 &&
timeout -k 10 200 python -u bench.py --batch 4 --transport xgmi-loopback --no-fp32-companion > $O/lenet_b4_lb.log 2>&1 &&
timeout -k 10 300 python -u bench.py --model bert-base --steps 20 --warmup 5 > $O/bert.log 2>&1 &&
timeout -k 10 400 python -u bench.py --model large --steps 20 --warmup 5 > $O/large.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_lenet -o lenet -- python3 -u bench.py --steps 1000 --warmup 100 --no-fp32-companion > $O/prof_lenet.log 2>&1
rc=$?; echo "rc=$rc"; exit $rc
