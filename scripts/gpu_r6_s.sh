# Graph pre-warm by snapshot / launch / restore (kernels unchanged): tests, then the driver protocol
# with and without it (alternated), the steady run and b4 loopback.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r6s
O=gpurun_out/r6s
timeout -k 10 500 python -u -m pytest tests/test_lenet_bf16.py "tests/test_multiproc_gpu.py::test_lenet_bf16_fused_dp_matches_four_launch" -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
: > $O/ab.jsonl
for rep in 1 2 3 4; do
  for a in "--steps 20 --warmup 5" "--steps 20 --warmup 5 --no-prewarm"; do
    timeout -k 10 120 python3 -u bench.py $a --no-fp32-companion > $O/last.log 2>&1 || { tail -5 $O/last.log; exit 1; }
    echo "{\"cfg\": \"$a\", \"r\": $(grep '^{' $O/last.log)}" >> $O/ab.jsonl
  done
done
timeout -k 10 200 python3 -u bench.py > $O/steady.log 2>&1 &&
timeout -k 10 200 python3 -u bench.py --batch 4 --transport xgmi-loopback --no-fp32-companion > $O/b4lb.log 2>&1
echo "rc=$?"
