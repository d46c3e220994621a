# Graph pre-warm (dry replay) + spin sync: LeNet / trainer GPU tests, then the driver protocol
# A/B (prewarm vs --no-prewarm), the steady run, b4 loopback.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r6n
O=gpurun_out/r6n
timeout -k 10 700 python -u -m pytest tests/test_lenet_bf16.py tests/test_lenet_native.py tests/test_multiproc_gpu.py tests/test_trainer_parallel_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
: > $O/ab.jsonl
for rep in 1 2 3; do
  for a in "--steps 20 --warmup 5" "--steps 20 --warmup 5 --no-prewarm"; do
    timeout -k 10 120 python3 -u bench.py $a --no-fp32-companion > $O/last.log 2>&1 || { tail -5 $O/last.log; exit 1; }
    echo "{\"cfg\": \"$a\", \"r\": $(grep '^{' $O/last.log)}" >> $O/ab.jsonl
  done
done
timeout -k 10 200 python3 -u bench.py > $O/steady.log 2>&1 &&
timeout -k 10 200 python3 -u bench.py --batch 4 --transport xgmi-loopback --no-fp32-companion > $O/b4lb.log 2>&1 &&
timeout -k 10 200 python3 -u bench.py --batch 32 --transport xgmi-loopback --no-fp32-companion > $O/b32lb.log 2>&1
echo "rc=$?"
