# bf16 LeNet one-launch step (KS + in-launch KW reducers) vs two launches: tests, then A/B benches
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_lenet_bf16.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/lenet_bf16_tests.log 2>&1 || exit 1
: > gpurun_out/lenet_fused_ab.jsonl
for rep in 1; do
  for f in 0 1; do
    for b in 32 4; do
      MLT_LENET_FUSED=$f timeout -k 10 120 python -u bench.py --batch $b > gpurun_out/ab.log 2>&1 || exit 1
      echo "{\"fused\": $f, \"batch\": $b, \"rep\": $rep, \"steps\": 3000, \"line\": $(grep '^{' gpurun_out/ab.log)}" >> gpurun_out/lenet_fused_ab.jsonl
      MLT_LENET_FUSED=$f timeout -k 10 120 python -u bench.py --batch $b --steps 20 --warmup 5 > gpurun_out/ab.log 2>&1 || exit 1
      echo "{\"fused\": $f, \"batch\": $b, \"rep\": $rep, \"steps\": 20, \"line\": $(grep '^{' gpurun_out/ab.log)}" >> gpurun_out/lenet_fused_ab.jsonl
    done
  done
done
